// q8k.h — quantize_row_q8_K of one 256-value super-block by one wave (ggml INIT for K-quant src0,
// restated in oracle/kquants_cpu.cpp): the first element of largest |x| gives max; iscale =
// -127/max; q = min(127, rne(iscale*x)); bsums = sums of 16; d = 1/iscale (all-zero block: d = 0,
// q = 0).  Lane l holds values 4l..4l+3; all 64 lanes take part.  Divisions in double then rounded:
// equal to fp32 division for fp32 operands.  Shared by the K-quant matvec prologues/epilogues and
// the attention kernel's per-head output image.
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

#ifndef GHIP_Q8K_DPP
#define GHIP_Q8K_DPP 1
#endif
#ifndef GHIP_Q8K_F32DIV
#define GHIP_Q8K_F32DIV 1
#endif
#ifndef GHIP_Q8K_RL
#define GHIP_Q8K_RL 1  // the cross-row levels of the (|x| max, index) reduction by v_readlane
#endif

namespace ghip {

// the (|x| max, first index) reduction's partner value at lane distance `off`: DPP within a row of
// 16 lanes (xor 1, xor 2 by quad permutes; the 4- and 8-lane steps by the half-row / row mirrors,
// which pair each group with its neighbour), ds_bpermute across rows.  The reduction (max, ties to
// the smaller index) is order-independent, so any pairing gives the same result in every lane.
// ggml's float division a / b (quantize_row_q8_K: iscale = -127.f/max, d = 1/iscale), correctly
// rounded: the f32 IEEE division (hipcc's default -fhip-fp32-correctly-rounded-divide-sqrt), which
// equals the double quotient rounded to float for float operands (53 >= 2*24 + 2 bits) — the form
// used before, at twice the latency
__device__ __forceinline__ float q8k_div(float a, float b) {
#if GHIP_Q8K_F32DIV
    return a / b;
#else
    return (float)((double)a / (double)b);
#endif
}

template <int OFF>
__device__ __forceinline__ uint32_t q8k_partner(uint32_t v) {
    if constexpr (OFF == 1) return (uint32_t)__builtin_amdgcn_mov_dpp((int)v, 0xB1, 0xF, 0xF, false);   // quad_perm 1,0,3,2
    else if constexpr (OFF == 2) return (uint32_t)__builtin_amdgcn_mov_dpp((int)v, 0x4E, 0xF, 0xF, false);  // quad_perm 2,3,0,1
    else if constexpr (OFF == 4) return (uint32_t)__builtin_amdgcn_mov_dpp((int)v, 0x141, 0xF, 0xF, false); // row_half_mirror
    else if constexpr (OFF == 8) return (uint32_t)__builtin_amdgcn_mov_dpp((int)v, 0x140, 0xF, 0xF, false); // row_mirror
    else return (uint32_t)__shfl_xor((int)v, OFF);
}
template <int OFF>
__device__ __forceinline__ void q8k_amax_level(float &amax, float &mx, int &idx) {
    const float oa = __builtin_bit_cast(float, q8k_partner<OFF>(__builtin_bit_cast(uint32_t, amax)));
    const float om = __builtin_bit_cast(float, q8k_partner<OFF>(__builtin_bit_cast(uint32_t, mx)));
    const int oi = (int)q8k_partner<OFF>((uint32_t)idx);
    if (oa > amax || (oa == amax && oi < idx)) {
        amax = oa;
        mx = om;
        idx = oi;
    }
}
__device__ __forceinline__ void q8k_amax_reduce(float &amax, float &mx, int &idx) {
    q8k_amax_level<1>(amax, mx, idx);
    q8k_amax_level<2>(amax, mx, idx);
    q8k_amax_level<4>(amax, mx, idx);
    q8k_amax_level<8>(amax, mx, idx);
#if GHIP_Q8K_RL
    // every lane of a 16-lane row now holds the row's best: the four rows by v_readlane (uniform
    // values, no LDS round trip) instead of two ds_bpermute levels — the same winner
    float ba = __builtin_bit_cast(float, __builtin_amdgcn_readlane(__builtin_bit_cast(int, amax), 0));
    float bm = __builtin_bit_cast(float, __builtin_amdgcn_readlane(__builtin_bit_cast(int, mx), 0));
    int bi = __builtin_amdgcn_readlane(idx, 0);
#pragma unroll
    for (int r = 16; r < 64; r += 16) {
        const float ra = __builtin_bit_cast(float, __builtin_amdgcn_readlane(__builtin_bit_cast(int, amax), r));
        const float rm = __builtin_bit_cast(float, __builtin_amdgcn_readlane(__builtin_bit_cast(int, mx), r));
        const int ri = __builtin_amdgcn_readlane(idx, r);
        if (ra > ba || (ra == ba && ri < bi)) {
            ba = ra;
            bm = rm;
            bi = ri;
        }
    }
    amax = ba;
    mx = bm;
    idx = bi;
#else
    q8k_amax_level<16>(amax, mx, idx);
    q8k_amax_level<32>(amax, mx, idx);
#endif
}

__device__ __forceinline__ void q8K_store(const float xv[4], int lane, uint8_t *blk) {
    float amax = 0.0f, mx = 0.0f;
    int idx = 0x7fffffff;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
        const float ax = fabsf(xv[j]);
        if (ax > amax) {
            amax = ax;
            mx = xv[j];
            idx = lane * 4 + j;
        }
    }
#if GHIP_Q8K_DPP
    q8k_amax_reduce(amax, mx, idx);
#else
#pragma unroll
    for (int off = 32; off >= 1; off >>= 1) {
        const float oa = __shfl_xor(amax, off), om = __shfl_xor(mx, off);
        const int oi = __shfl_xor(idx, off);
        if (oa > amax || (oa == amax && oi < idx)) {
            amax = oa;
            mx = om;
            idx = oi;
        }
    }
#endif
    int q[4] = {0, 0, 0, 0};
    float d = 0.0f;
    if (amax != 0.0f) {
        const float iscale = q8k_div(-127.0f, mx);
#pragma unroll
        for (int j = 0; j < 4; ++j) q[j] = min(127, (int)__builtin_rintf(iscale * xv[j]));
        d = q8k_div(1.0f, iscale);
    }
    int bs = q[0] + q[1] + q[2] + q[3];
    bs += (int)q8k_partner<1>((uint32_t)bs);  // sums of 16 (4 lanes): exact integer adds
    bs += (int)q8k_partner<2>((uint32_t)bs);
    *(uint32_t *)(blk + 4 + lane * 4) =
        (uint32_t)(q[0] & 255) | ((uint32_t)(q[1] & 255) << 8) | ((uint32_t)(q[2] & 255) << 16) | ((uint32_t)q[3] << 24);
    if ((lane & 3) == 0) *(int16_t *)(blk + 260 + (lane >> 2) * 2) = (int16_t)bs;
    if (lane == 0) *(float *)blk = d;
}

// q8K_store of N super-blocks at once by one wave (blk + k*stride for block k): the N reductions run
// interleaved level by level, so the cross-lane latency is paid once per level, not N times.
// Bytes identical to N calls of q8K_store.
template <int N>
__device__ __forceinline__ void q8K_store_n(const float (&xv)[N][4], int lane, uint8_t *blk, int stride = 292) {
    float amax[N], mx[N];
    int idx[N];
#pragma unroll
    for (int k = 0; k < N; ++k) {
        amax[k] = 0.0f; mx[k] = 0.0f; idx[k] = 0x7fffffff;
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            const float ax = fabsf(xv[k][j]);
            if (ax > amax[k]) {
                amax[k] = ax;
                mx[k] = xv[k][j];
                idx[k] = lane * 4 + j;
            }
        }
    }
#if GHIP_Q8K_DPP
#pragma unroll
    for (int k = 0; k < N; ++k) q8k_amax_reduce(amax[k], mx[k], idx[k]);
#else
#pragma unroll
    for (int off = 32; off >= 1; off >>= 1) {
        float oa[N], om[N];
        int oi[N];
#pragma unroll
        for (int k = 0; k < N; ++k) {
            oa[k] = __shfl_xor(amax[k], off);
            om[k] = __shfl_xor(mx[k], off);
            oi[k] = __shfl_xor(idx[k], off);
        }
#pragma unroll
        for (int k = 0; k < N; ++k) {
            if (oa[k] > amax[k] || (oa[k] == amax[k] && oi[k] < idx[k])) {
                amax[k] = oa[k];
                mx[k] = om[k];
                idx[k] = oi[k];
            }
        }
    }
#endif
    int bs[N];
#pragma unroll
    for (int k = 0; k < N; ++k) {
        int q[4] = {0, 0, 0, 0};
        float d = 0.0f;
        if (amax[k] != 0.0f) {
            const float iscale = q8k_div(-127.0f, mx[k]);
#pragma unroll
            for (int j = 0; j < 4; ++j) q[j] = min(127, (int)__builtin_rintf(iscale * xv[k][j]));
            d = q8k_div(1.0f, iscale);
        }
        bs[k] = q[0] + q[1] + q[2] + q[3];
        uint8_t *b = blk + k * stride;
        *(uint32_t *)(b + 4 + lane * 4) =
            (uint32_t)(q[0] & 255) | ((uint32_t)(q[1] & 255) << 8) | ((uint32_t)(q[2] & 255) << 16) | ((uint32_t)q[3] << 24);
        if (lane == 0) *(float *)b = d;
    }
#pragma unroll
    for (int k = 0; k < N; ++k) bs[k] += (int)q8k_partner<1>((uint32_t)bs[k]);
#pragma unroll
    for (int k = 0; k < N; ++k) bs[k] += (int)q8k_partner<2>((uint32_t)bs[k]);
#pragma unroll
    for (int k = 0; k < N; ++k)
        if ((lane & 3) == 0) *(int16_t *)(blk + k * stride + 260 + (lane >> 2) * 2) = (int16_t)bs[k];
}

}  // namespace ghip
