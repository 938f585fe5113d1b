// device_util.h — bit-exact numeric helpers shared by the gfx950 kernels.
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

namespace ghip {

__device__ __forceinline__ float h2f(uint32_t bits) {
    return (float)__builtin_bit_cast(_Float16, (uint16_t)(bits & 0xFFFF));
}

// Opaque to the optimiser: LLVM's AMDGPU backend folds fptrunc(fmul(a, b)) into v_fma_mixlo_f16
// (ONE rounding straight to fp16) even under -ffp-contract=off, while ggml rounds the product to
// fp32 first and then to fp16 (two roundings).  The two differ on fp16 ties, so every computed
// value is pinned in a VGPR before conversion.
__device__ __forceinline__ float pin(float x) {
    asm volatile("" : "+v"(x));
    return x;
}

// fp32 -> fp16 bits, round-to-nearest-even (v_cvt_f16_f32), of an already-rounded fp32 value
__device__ __forceinline__ uint32_t f2h(float f) { return (uint32_t)__builtin_bit_cast(uint16_t, (_Float16)pin(f)); }

}  // namespace ghip

namespace ghip {

// ---- DPP lane moves (VALU, ~no latency) instead of ds_bpermute shuffles ----------------------
// dpp_ctrl: quad_perm [1,0,3,2] = xor 1 (0xB1); [2,3,0,1] = xor 2 (0x4E); row_shl:4 = 0x104
// (lane i reads lane i+4 of its 16-lane row); row_half_mirror = 0x141; row_mirror = 0x140.
template <int CTRL>
__device__ __forceinline__ float dpp_f(float v) {
    return __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, v), CTRL, 0xF, 0xF, false));
}
template <int CTRL>
__device__ __forceinline__ uint32_t dpp_u(uint32_t v) {
    return (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, CTRL, 0xF, 0xF, false);
}

// ggml hsum_float_8 over lanes 8g..8g+7: ((a0+a4)+(a2+a6)) + ((a1+a5)+(a3+a7)); exact pairs.
// The result is valid in lane 8g (and 8g+1); float addition is commutative bit for bit.
__device__ __forceinline__ float fold8_dpp(float v) {
    v = v + dpp_f<0x104>(v);  // lanes 0..3 of each 8-group: a_l + a_{l+4}
    v = v + dpp_f<0x4E>(v);   // xor 2
    v = v + dpp_f<0xB1>(v);   // xor 1
    return v;
}

// ggml F16 reduce of accumulator rows held by the 4 lanes of a quad: (acc0+acc2) + (acc1+acc3)
__device__ __forceinline__ float quad_fold_dpp(float v) {
    v = v + dpp_f<0x4E>(v);  // xor 2
    v = v + dpp_f<0xB1>(v);  // xor 1
    return v;
}

// order-free all-reduce over the 64 lanes (max of floats / sum of u64 pieces)
__device__ __forceinline__ float wave_max(float v) {
    v = fmaxf(v, dpp_f<0xB1>(v));
    v = fmaxf(v, dpp_f<0x4E>(v));
    v = fmaxf(v, dpp_f<0x141>(v));
    v = fmaxf(v, dpp_f<0x140>(v));
    const float r0 = __builtin_bit_cast(float, __builtin_amdgcn_readlane(__builtin_bit_cast(int, v), 0));
    const float r1 = __builtin_bit_cast(float, __builtin_amdgcn_readlane(__builtin_bit_cast(int, v), 16));
    const float r2 = __builtin_bit_cast(float, __builtin_amdgcn_readlane(__builtin_bit_cast(int, v), 32));
    const float r3 = __builtin_bit_cast(float, __builtin_amdgcn_readlane(__builtin_bit_cast(int, v), 48));
    return fmaxf(fmaxf(r0, r1), fmaxf(r2, r3));
}

// T / n for the norms' mean: an exact scaling by 2^-k when n = 2^k (no double division on the
// prologue's critical path; the quotient is the same bits), else the IEEE division
__device__ __forceinline__ double div_by_n(double T, int64_t n) {
#ifdef GHIP_DIVN_OLD  // (A/B builds only)
    return T / (double)n;
#endif
    if ((n & (n - 1)) == 0) {
        const int k = __builtin_ctzll((unsigned long long)n);
        return T * __builtin_bit_cast(double, (unsigned long long)(1023 - k) << 52);
    }
    return T / (double)n;
}

// a double's DPP move (two dword moves)
template <int CTRL>
__device__ __forceinline__ double dpp_d(double v) {
    const unsigned long long b = __builtin_bit_cast(unsigned long long, v);
    return __builtin_bit_cast(double, ((unsigned long long)dpp_u<CTRL>((uint32_t)(b >> 32)) << 32) | dpp_u<CTRL>((uint32_t)b));
}
// the wave's sum of a double in every lane, by DPP within 16-lane rows and v_readlane across them
// (no LDS round trips).  The ORDER is this butterfly's, not a sequential one: only for sums whose
// use is order-proof (the rms_norm mean under rms_mean_certain)
__device__ __forceinline__ double wave_sum_f64(double v) {
    v += dpp_d<0xB1>(v);
    v += dpp_d<0x4E>(v);
    v += dpp_d<0x141>(v);
    v += dpp_d<0x140>(v);
    auto rl = [&](int L) {
        const unsigned long long b = __builtin_bit_cast(unsigned long long, v);
        const uint32_t lo = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)b, L);
        const uint32_t hi = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)(b >> 32), L);
        return __builtin_bit_cast(double, ((unsigned long long)hi << 32) | lo);
    };
    return (rl(0) + rl(16)) + (rl(32) + rl(48));
}

__device__ __forceinline__ unsigned long long wave_sum_u64(unsigned long long v) {
    // integer sum is exact in any order; reduce 32-bit halves with carries via 64-bit adds
    unsigned long long t;
    t = ((unsigned long long)dpp_u<0xB1>((uint32_t)(v >> 32)) << 32) | dpp_u<0xB1>((uint32_t)v);
    v += t;
    t = ((unsigned long long)dpp_u<0x4E>((uint32_t)(v >> 32)) << 32) | dpp_u<0x4E>((uint32_t)v);
    v += t;
    t = ((unsigned long long)dpp_u<0x141>((uint32_t)(v >> 32)) << 32) | dpp_u<0x141>((uint32_t)v);
    v += t;
    t = ((unsigned long long)dpp_u<0x140>((uint32_t)(v >> 32)) << 32) | dpp_u<0x140>((uint32_t)v);
    v += t;
    unsigned long long s = 0;
#pragma unroll
    for (int r = 0; r < 64; r += 16) {
        const uint32_t lo = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)v, r);
        const uint32_t hi = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)(v >> 32), r);
        s += ((unsigned long long)hi << 32) | lo;
    }
    return s;
}

// ---- ggml's rms_norm mean, provably --------------------------------------------------
// ggml: sum = Σ_i (double)(x_i*x_i) in index order, rounded after every add; mean = (float)(sum/n).
// The kernels add the same double terms in a tree T and form q = fl64(T/n), mean = (float)q.  All
// terms are ≥ 0, so ANY summation order of them lies within γ_{n−1}·E of the exact sum E (γ_k =
// k·u/(1 − k·u), u = 2^−53; Higham, Accuracy and Stability of Numerical Algorithms, §4.2):
// |S − T| ≤ 2·γ_{n−1}·E ≤ n·2^−52·T·(1 + O(n·u)), so fl64(S/n) lies in q·[1 − ρ, 1 + ρ] with
// ρ = n·2^−51 + 2^−48 (twice that bound plus both divisions' roundings).  Float rounding of a double
// q in the float normal range is decided by the 29 low mantissa bits it drops: the rounding
// boundary (the midpoint to the next float) is where they equal 2^28, and ρ·q is under ρ·2^53 =
// 4n + 32 units of q's last place.  rms_mean_certain checks |low29(q) − 2^28| > 4n + 40: no
// boundary inside q·[1 ± ρ], so S/n and T/n round to the same float — the tree's mean IS ggml's.
// Integer ops on q's bits only (no division, no double compares on the prologue's critical path).
// When it fails (≈ 2·(4n+40)/2^29 ≈ 2^−15 of the norms at n = 2048, or a mean outside the float
// normal range) the caller runs ggml's sequential sum, seq_sumsq_wave.  The binade edge needs no
// case: the float 2^k there is representable and the nearest boundary below it is 2^27 units of q
// away (n ≤ 2^22 keeps 4n + 40 < 2^27).  0, inf and NaN sums are the same in every order.
__device__ __forceinline__ bool rms_mean_certain(double q, int64_t n) {
    const uint64_t b = __builtin_bit_cast(uint64_t, q);
    const uint32_t ex = (uint32_t)(b >> 52) & 0x7FFu;                       // q ≥ 0: no sign bit
    const uint32_t low = (uint32_t)b & 0x1FFFFFFFu;                         // the bits a float drops
    const uint32_t dist = low >= 0x10000000u ? low - 0x10000000u : 0x10000000u - low;
    const bool special = (b == 0) | (ex == 0x7FFu);                         // 0, inf, NaN: certain
    const bool normal = (ex >= 1023u - 126u) & (ex <= 1023u + 127u) & (n <= ((int64_t)1 << 22));
    return special | (normal & (dist > (uint32_t)(4 * n + 40)));
}

// ggml's sequential sum Σ (double)(x_i*x_i), i = 0 … n−1 in order, by ONE wave (all 64 lanes
// active, converged control flow); every lane returns it.  load8(i, v) writes elements i … i+7 (i a
// multiple of 8, i < n) as the caller's tree saw them (elements at or past n as 0: adding +0 to a
// non-negative double leaves it unchanged).  Every wave that needs the value may run it itself (no
// barrier); it is the rare slow path of rms_mean_certain (≈ n dependent double adds).
template <class Load8>
__device__ __forceinline__ double seq_sumsq_wave(int64_t n, Load8 load8) {
    const int lane = (int)(threadIdx.x & 63);
    double s = 0.0;
    for (int64_t base = 0; base < n; base += 512) {
        float v[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
        const int64_t i = base + (int64_t)lane * 8;
        if (i < n) load8(i, v);
        // not unrolled: the rare path's code stays small (unrolled it added ~6 KB to every kernel
        // holding a norm prologue, and the instruction fetch of the hot path paid for it)
#pragma unroll 1
        for (int L = 0; L < 64; ++L) {
#pragma unroll
            for (int j = 0; j < 8; ++j) {
                const float x = __builtin_bit_cast(float, __builtin_amdgcn_readlane(__builtin_bit_cast(int, v[j]), L));
                const float sq = x * x;
                s += (double)sq;
            }
        }
    }
    return s;
}

// ggml's exp table entry table_exp_f16[x16] = fp16(expf(fp32(x16))) (ggml_init), computed instead of
// gathered (the gather is a dependent global round trip in the softmax).  The f16 rounding absorbs
// the f32 error of the hardware exp: for every non-positive f16 input (the only ones the softmax
// forms) __expf, expf and exp(double) all give the glibc-expf table entry (tests/micro/exp_variants;
// the GPU test test_exp_f16_matches_table re-checks this very function on all inputs).
__device__ __forceinline__ uint32_t exp_f16_of(uint32_t x16) {
    return f2h(__expf(h2f(x16)));
}

// ---- Q8_0 activation image (DESIGN.md §Activation image) ----------------------------------------
// The LDS layout the matvec streams against, also used in HBM between a producer kernel and its
// consumer: act u32 [nb/4][8 lanes][4] — dword ((b>>2)*8 + l)*4 + (b&3) holds elements 4l..4l+3
// of block b as int8; ns (optional, Q4_0) the same layout holding -8*sum of those 4; da f32 [nb].
// quantize_row_q8_0: amax = max|v|, d = fp16(amax/127), id = amax ? 127/amax : 0,
// q = rint(v*id).  A quad of threads (consecutive lanes q = 0..3, all active) owns one block;
// thread q holds elements 8q..8q+7.
__device__ __forceinline__ void image_put_quad(uint32_t *act, uint32_t *ns, float *da, int64_t b, int q,
                                               const float v[8]) {
    float amax = 0.0f;
#pragma unroll
    for (int j = 0; j < 8; ++j) amax = fmaxf(amax, fabsf(v[j]));
    amax = fmaxf(amax, dpp_f<0xB1>(amax));  // quad xor 1
    amax = fmaxf(amax, dpp_f<0x4E>(amax));  // quad xor 2
    const float d = amax / 127.f;
    const uint32_t d16 = f2h(d);
    const float id = (amax != 0.0f) ? 127.f / amax : 0.0f;
#pragma unroll
    for (int h = 0; h < 2; ++h) {
        const int l = 2 * q + h;
        int qi[4];
#pragma unroll
        for (int k = 0; k < 4; ++k) qi[k] = (int)__builtin_rintf(v[4 * h + k] * id);
        const uint32_t packed = (uint32_t)(qi[0] & 0xFF) | ((uint32_t)(qi[1] & 0xFF) << 8) |
                                ((uint32_t)(qi[2] & 0xFF) << 16) | ((uint32_t)(qi[3] & 0xFF) << 24);
        const int64_t idx = ((b >> 2) * 8 + l) * 4 + (b & 3);
        act[idx] = packed;
        if (ns) ns[idx] = (uint32_t)(-8 * (qi[0] + qi[1] + qi[2] + qi[3]));
    }
    if (q == 0) da[b] = h2f(d16);
}

}  // namespace ghip
