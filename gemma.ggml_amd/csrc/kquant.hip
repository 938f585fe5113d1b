// kquant.hip — K-quant matvec on gfx950: Q4_K / Q6_K weights
// (ggml row-major super-blocks, 144 / 210 B per 256 values; src/kernals.cl:13-34) against a Q8_K
// activation column (ggml's INIT for K-quant src0: 292 B per 256 values).
//
// Numerics = ggml's AVX2 vec_dot_q4_K_q8_K / vec_dot_q6_K_q8_K lane order (restated in
// oracle/kquants_cpu.cpp): one thread is one AVX2 lane l of one row; per super-block it forms the
// lane's exact int32 sum over bytes 4l..4l+3 of every 32-value chunk (v_dot4_i32_i8 per chunk,
// times the chunk's integer scale), then acc = fmaf(y.d*f16(x.d), (float)isum, acc).  Q4_K adds
// the mins term in lanes 0..3 (fmaf(-y.d*f16(x.dmin), (float)(m·S), accm)); the result is
// hsum_float_8(acc) + ((m0+m2)+(m1+m3)), folded with DPP like the Q4_0 path.
// Bound: HBM (weights read once); 8 rows x 8 lanes per wave, the Q8_K column staged in LDS.
#include <algorithm>
#include <cstdlib>

#include "device_util.h"
#include "kernels.h"
#include "q8k.h"

namespace ghip {
namespace {

constexpr int KQ_THREADS = 256;

__device__ __forceinline__ int sdot4k(uint32_t a, uint32_t b) { return __builtin_amdgcn_sdot4((int)a, (int)b, 0, false); }

// a dword at a 2-byte aligned address (Q6_K blocks are 210 B: odd blocks start 2 mod 4)
__device__ __forceinline__ uint32_t ld_u32_a2(const uint8_t *p) {
    const uint16_t *h = (const uint16_t *)p;
    return (uint32_t)h[0] | ((uint32_t)h[1] << 16);
}

// one super-block s of row `wrow` for AVX2 lane l: the lane's exact int32 sum and the fp32 scale
// d = y.d*f16(x.d); Q4_K also the mins lane k = l & 3 (meaningful in lanes 0..3): prod and dmin
struct kq_term { int sumi; float d; int prod; float dmin; };

// a super-block's weight bytes for AVX2 lane l, loaded ahead of the arithmetic (kq_terms)
template <int WT> struct kq_raw;
template <> struct kq_raw<T_Q4_K> { uint4 h; uint32_t q[4]; };
template <> struct kq_raw<T_Q6_K> { uint32_t qla[2], qlb[2], qh[2], sc[4]; uint32_t d; };

// Lane-contiguous device layout of K-quant rows (launch_kq_retile; the engine's weights, `TL`):
// row-major rows, row_bytes unchanged, only the bytes inside a row move so that each AVX2 lane's
// operands are one contiguous, aligned vector:
//   Q4_K, per super-block (144 B): header [d, dmin, scales] (16 B) unchanged; quant dword j of lane
//     l (ggml byte 16 + 32j + 4l) -> 16 + 16l + 4j: one 16-B load per lane instead of four.
//   Q6_K, per group of 8 super-blocks (1680 B, 16-aligned): [8 x ql 128 B][8 x qh 64 B]
//     [8 x scales 16 B][8 x d 2 B]; within super-block i: ql dword k of lane l (ggml byte 32k + 4l)
//     -> 128i + 16l + 4k, qh dword j (ggml byte 128 + 32j + 4l) -> 1024 + 64i + 8l + 4j; scales
//     -> 1536 + 16i, d -> 1664 + 2i: four loads per lane instead of ~21 two-byte-aligned ones.
// Same bytes, same arithmetic: the dots are unchanged.
// Non-temporal lane-contiguous weight loads (GHIP_KQ_NT bits: 1 Q4_K, 2 Q6_K, 4 the lane-own quant bytes only; as the Q4_0 matvecs load theirs):
// measured slower, Q4_K_M decode 1,059-1,064 (plain) vs 1,036-1,037 (Q4_K nt) / 1,019-1,028 (Q6_K nt)
// tok/s, 1,028-1,034 (lane-own quant bytes nt, headers plain) (same box, interleaved) — off
#ifndef GHIP_KQ_NT
#define GHIP_KQ_NT 0
#endif
typedef uint32_t kq_v4u __attribute__((ext_vector_type(4)));
typedef uint32_t kq_v2u __attribute__((ext_vector_type(2)));
template <int WT, bool LANE = false>  // LANE: each lane its own bytes (not a wave-shared header)
__device__ __forceinline__ uint4 kq_ld16(const uint8_t *p) {
    if constexpr ((GHIP_KQ_NT & (WT == T_Q4_K ? 1 : 2)) || (LANE && (GHIP_KQ_NT & 4))) {
        const kq_v4u v = __builtin_nontemporal_load((const kq_v4u *)p);
        return make_uint4(v.x, v.y, v.z, v.w);
    }
    return *(const uint4 *)p;
}
template <int WT, bool LANE = false>
__device__ __forceinline__ uint2 kq_ld8(const uint8_t *p) {
    if constexpr ((GHIP_KQ_NT & (WT == T_Q4_K ? 1 : 2)) || (LANE && (GHIP_KQ_NT & 4))) {
        const kq_v2u v = __builtin_nontemporal_load((const kq_v2u *)p);
        return make_uint2(v.x, v.y);
    }
    return *(const uint2 *)p;
}
template <int WT, bool TL = false>
__device__ __forceinline__ kq_raw<WT> kq_load(const uint8_t *wrow, int s, int l) {
    kq_raw<WT> r;
    if constexpr (TL && WT == T_Q4_K) {
        const uint8_t *blk = wrow + (int64_t)s * 144;
        r.h = kq_ld16<WT>(blk);
        const uint4 q = kq_ld16<WT, true>(blk + 16 + 16 * l);
        r.q[0] = q.x; r.q[1] = q.y; r.q[2] = q.z; r.q[3] = q.w;
        return r;
    }
    if constexpr (TL && WT == T_Q6_K) {
        const uint8_t *g = wrow + (int64_t)(s >> 3) * 1680;
        const int i = s & 7;
        const uint4 ql = kq_ld16<WT, true>(g + 128 * i + 16 * l);
        const uint2 qh = kq_ld8<WT, true>(g + 1024 + 64 * i + 8 * l);
        const uint4 sc = kq_ld16<WT>(g + 1536 + 16 * i);
        r.qla[0] = ql.x; r.qlb[0] = ql.y; r.qla[1] = ql.z; r.qlb[1] = ql.w;
        r.qh[0] = qh.x; r.qh[1] = qh.y;
        r.sc[0] = sc.x; r.sc[1] = sc.y; r.sc[2] = sc.z; r.sc[3] = sc.w;
        r.d = *(const uint16_t *)(g + 1664 + 2 * i);
        return r;
    }
    if constexpr (WT == T_Q4_K) {
        const uint8_t *blk = wrow + (int64_t)s * 144;
        r.h = *(const uint4 *)blk;  // d, dmin, scales[12]
#pragma unroll
        for (int j = 0; j < 4; ++j) r.q[j] = *(const uint32_t *)(blk + 16 + 32 * j + 4 * l);
    } else {
        const uint8_t *blk = wrow + (int64_t)s * 210;
#pragma unroll
        for (int j = 0; j < 2; ++j) {
            r.qla[j] = ld_u32_a2(blk + 64 * j + 4 * l);
            r.qlb[j] = ld_u32_a2(blk + 64 * j + 32 + 4 * l);
            r.qh[j] = ld_u32_a2(blk + 128 + 32 * j + 4 * l);
        }
#pragma unroll
        for (int k = 0; k < 4; ++k) r.sc[k] = ld_u32_a2(blk + 192 + 4 * k);
        r.d = *(const uint16_t *)(blk + 208);
    }
    return r;
}

template <int WT>
__device__ __forceinline__ kq_term kq_terms(const kq_raw<WT> &r, const uint8_t *xs, int s, int l) {
    kq_term t;
    const uint8_t *xb = xs + s * 292;
    const float yd = *(const float *)xb;
    const int8_t *q8 = (const int8_t *)(xb + 4);
    if constexpr (WT == T_Q4_K) {
        // six-bit scales / mins (src/kernals.cl:79-84)
        const uint32_t u0 = r.h.y, u1 = r.h.z, u2 = r.h.w;
        const uint32_t s03 = u0 & 0x3f3f3f3fu;                                      // sc 0..3
        const uint32_t s47 = (u2 & 0x0f0f0f0fu) | (((u0 >> 6) & 0x03030303u) << 4);  // sc 4..7
        const uint32_t m03 = u1 & 0x3f3f3f3fu;                                      // mins 0..3
        const uint32_t m47 = ((u2 >> 4) & 0x0f0f0f0fu) | (((u1 >> 6) & 0x03030303u) << 4);
        int sumi = 0;
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            const uint32_t scw = j < 2 ? s03 : s47;
            const int sc_lo = (scw >> (16 * (j & 1))) & 0xFF, sc_hi = (scw >> (16 * (j & 1) + 8)) & 0xFF;
            const uint32_t alo = *(const uint32_t *)(q8 + 64 * j + 4 * l);
            const uint32_t ahi = *(const uint32_t *)(q8 + 64 * j + 32 + 4 * l);
            sumi += sc_lo * sdot4k(r.q[j] & 0x0F0F0F0Fu, alo) + sc_hi * sdot4k((r.q[j] >> 4) & 0x0F0F0F0Fu, ahi);
        }
        t.sumi = sumi;
        t.d = yd * pin(h2f(r.h.x));
        t.dmin = -yd * pin(h2f(r.h.x >> 16));
        const int16_t *bs = (const int16_t *)(xb + 260);
        const int k = l & 3;
        const int S0 = (int)bs[4 * k] + (int)bs[4 * k + 1], S1 = (int)bs[4 * k + 2] + (int)bs[4 * k + 3];
        const uint32_t mw = k < 2 ? m03 : m47;
        const int mn0 = (mw >> (16 * (k & 1))) & 0xFF, mn1 = (mw >> (16 * (k & 1) + 8)) & 0xFF;
        t.prod = mn0 * S0 + mn1 * S1;
    } else {
        int sumi = 0;
#pragma unroll
        for (int j = 0; j < 2; ++j) {
            const uint32_t qla = r.qla[j], qlb = r.qlb[j], qh = r.qh[j];
            const uint32_t q6[4] = {(qla & 0x0F0F0F0Fu) | ((qh & 0x03030303u) << 4),
                                    (qlb & 0x0F0F0F0Fu) | (((qh >> 2) & 0x03030303u) << 4),
                                    ((qla >> 4) & 0x0F0F0F0Fu) | (((qh >> 4) & 0x03030303u) << 4),
                                    ((qlb >> 4) & 0x0F0F0F0Fu) | (((qh >> 6) & 0x03030303u) << 4)};
#pragma unroll
            for (int i = 0; i < 4; ++i) {
                const uint32_t av = *(const uint32_t *)(q8 + 128 * j + 32 * i + 4 * l);
                const int p = sdot4k(q6[i], av) - sdot4k(0x20202020u, av);
                const int bi = 8 * j + 2 * i + (l >> 2);  // scale byte 192 + bi
                const int sc = (int)(int8_t)(uint8_t)(r.sc[bi >> 2] >> (8 * (bi & 3)));
                sumi += sc * p;
            }
        }
        t.sumi = sumi;
        t.d = yd * pin(h2f(r.d));
        t.prod = 0;
        t.dmin = 0.0f;
    }
    return t;
}

template <int WT>
__device__ __forceinline__ kq_term kq_block(const uint8_t *wrow, const uint8_t *xs, int s, int l) {
    return kq_terms<WT>(kq_load<WT>(wrow, s, l), xs, s, l);
}

// KQ_PF super-blocks' weight loads are issued before any of their arithmetic (one memory round trip
// per group instead of one per super-block)
#ifndef GHIP_KQ_PF
#define GHIP_KQ_PF 2  // Q4_K_M decode, same box: 1 / 2 / 3 / 4 / 8 -> 1.170 / 1.132 / 1.140 / 1.155 / 1.315 ms/token
#endif
constexpr int KQ_PF = GHIP_KQ_PF;
#ifndef GHIP_KQ_EARLY
#define GHIP_KQ_EARLY 2  // 1: first weight round issued before the Q8_K staging; 2: after every wave's
                         // activation loads (one s_barrier): Q4_K_M 1,066-1,067 vs 1,053-1,066 tok/s
#endif
#ifndef GHIP_KQ_NORM1
#define GHIP_KQ_NORM1 2  // 2: DPP wave sums + one LDS word per wave (order-free under rms_mean_certain);
                         // 1: the pairwise tree with one barrier (every wave runs the lane levels)
#endif

// the column's Q8_K image into LDS: 16-B loads, all of a thread's loads issued before the first
// store (a plain copy loop waits one memory round trip per iteration, behind the weight loads
// issued earlier — it cost the Q6_K down ~µs)
__device__ __forceinline__ void stage_q8k(const kq_args &a, uint8_t *xs, int col, int tid, int nth) {
    const uint8_t *src = a.x + (int64_t)col * a.x_col_stride;
    const int bytes = a.nsb * 292;
    if ((bytes & 15) == 0 && ((uintptr_t)src & 15) == 0) {
        const int n16 = bytes >> 4;
        const uint4 *s4 = (const uint4 *)src;
        uint4 *d4 = (uint4 *)xs;
        for (int i0 = 0; i0 < n16; i0 += 4 * nth) {
            uint4 v[4];
#pragma unroll
            for (int k = 0; k < 4; ++k) {
                const int i = i0 + tid + k * nth;
                v[k] = s4[i < n16 ? i : 0];
            }
#pragma unroll
            for (int k = 0; k < 4; ++k) {
                const int i = i0 + tid + k * nth;
                if (i < n16) d4[i] = v[k];
            }
        }
        return;
    }
    const uint32_t *s1 = (const uint32_t *)src;
    uint32_t *d1 = (uint32_t *)xs;
    for (int i = tid; i < a.nsb * 73; i += nth) d1[i] = s1[i];
}

// The column's Q8_K image in LDS = ggml's INIT for K-quant src0, fused into the matvec (no separate
// k_norm_q8K / k_quant_q8_K launch): KQP_COPY copies precomputed Q8_K rows (x); KQP_F32 runs
// quantize_row_q8_K on f32 xf (k_quant_q8_K: one wave per super-block); KQP_NORM first applies
// rms_norm(xf)*norm_w.  Its double sum of squares is a DPP wave sum plus one LDS word per wave (any
// order): rms_mean_certain (device_util.h) proves the resulting float mean equal to
// ggml's sequential sum's, else seq_sumsq_wave runs ggml's own order — so the bytes equal the
// separate kernels' (k_norm_q8K takes the same certified-tree-or-sequential path).
// Two halves: kq_pro_load issues every f32 load of this wave's super-blocks (wave w takes
// w, w+nw, ...; at most XJ of them; surplus slots load a clamped block and are ignored) BEFORE the
// weight prologue loads, so one counted wait covers them and the serial load -> quantize round
// trips of a per-block loop are gone; kq_pro_build quantizes from registers into LDS.
template <int XJ>
struct kq_pro_regs {
    float4 x[XJ], w[XJ];
};

template <int XJ>
__device__ __forceinline__ void kq_pro_load(const kq_args &a, int col, int wave, int nw, int lane, kq_pro_regs<XJ> &r) {
    if (a.pro == KQP_COPY) return;
    const float *x = a.xf + (int64_t)col * a.xf_col_stride;
#pragma unroll
    for (int j = 0; j < XJ; ++j) {
        const int sb = min(wave + nw * j, a.nsb - 1);
        r.x[j] = *(const float4 *)(x + (int64_t)sb * 256 + lane * 4);
        if (a.pro == KQP_NORM) r.w[j] = *(const float4 *)(a.norm_w + (int64_t)sb * 256 + lane * 4);
    }
}

// 1/sqrtf(mean + eps) of the column's rms_norm from the prologue's tree sum T (*q = T/n; the caller
// checks it with rms_mean_certain after the image is built)
__device__ __forceinline__ float kq_norm_scale(const kq_args &a, double T, double *q) {
    *q = div_by_n(T, (int64_t)a.nsb * 256);
    return 1.0f / sqrtf((float)*q + a.eps);
}
// the same from ggml's sequential sum (every wave runs it itself: the rare slow path)
__device__ __forceinline__ float kq_seq_scale(const kq_args &a, int col) {
    const int64_t n = (int64_t)a.nsb * 256;
    const float *x = a.xf + (int64_t)col * a.xf_col_stride;
    const float mean = (float)(seq_sumsq_wave(n, [&](int64_t i0, float v[8]) {
                                   const float4 u = *(const float4 *)(x + i0), w = *(const float4 *)(x + i0 + 4);
                                   v[0] = u.x; v[1] = u.y; v[2] = u.z; v[3] = u.w; v[4] = w.x; v[5] = w.y; v[6] = w.z; v[7] = w.w;
                               }) / (double)n);
    return 1.0f / sqrtf(mean + a.eps);
}

template <int XJ>
__device__ void kq_pro_build(const kq_args &a, uint8_t *xs, double *red, int col, int tid, int nth,
                             const kq_pro_regs<XJ> &r) {
    if (a.pro == KQP_COPY) {
        stage_q8k(a, xs, col, tid, nth);
        return;
    }
    const int nw = nth >> 6, lane = tid & 63, wave = tid >> 6;
    float scale = 1.0f;
    double q = 0.0;  // the tree's T/n (rms_mean_certain)
    // this wave holds super-blocks wave and wave + nw: the tree's first level (h = nw*64) pairs
    // exactly them, so it runs in registers, and their two quantizations interleave
    const bool two = XJ == 2 && a.nsb == 2 * nw;
    if (a.pro == KQP_NORM) {
        double part[XJ];
#pragma unroll
        for (int j = 0; j < XJ; ++j) {
            double pj = 0.0;
            pj += (double)(r.x[j].x * r.x[j].x);
            pj += (double)(r.x[j].y * r.x[j].y);
            pj += (double)(r.x[j].z * r.x[j].z);
            pj += (double)(r.x[j].w * r.x[j].w);
            part[j] = pj;
        }
        int n = a.nsb * 64;
        const int R = two ? nw : a.nsb;  // rows of 64 partials in the tree
        if (GHIP_KQ_NORM1 == 2) {
            // any summation order is ggml's once rms_mean_certain holds: the wave's
            // partials by DPP (wave_sum_f64), one LDS word per wave, one barrier — instead of the
            // pairwise tree's six dependent ds_bpermute levels
            double p = 0.0;
#pragma unroll
            for (int j = 0; j < XJ; ++j)
                if (wave + nw * j < a.nsb) p += part[j];
            p = wave_sum_f64(p);
            if (lane == 0) red[wave] = p;
            __syncthreads();
            double T = 0.0;
            for (int w = 0; w < nw; ++w) T += red[w];
            scale = kq_norm_scale(a, T, &q);
            n = 0;  // done
        } else if (GHIP_KQ_NORM1 && (R == 2 || R == 4 || R == 8)) {
            // the same pairwise tree (h = n/2 per level over R rows of 64 partials, then the six lane
            // levels) with ONE barrier: every wave reads its lane's R partials and runs the row levels
            // in registers and the lane levels itself, so no wave waits for wave 0's tree
            if (two) {
                red[wave * 64 + lane] = part[0] + part[XJ - 1];
            } else {
#pragma unroll
                for (int j = 0; j < XJ; ++j)
                    if (wave + nw * j < a.nsb) red[(wave + nw * j) * 64 + lane] = part[j];
            }
            __syncthreads();
            double rv[8];
#pragma unroll
            for (int k = 0; k < 8; ++k) rv[k] = k < R ? red[k * 64 + lane] : 0.0;
#pragma unroll
            for (int h = 4; h >= 1; h >>= 1)
                if (h < R)
#pragma unroll
                    for (int k = 0; k < 4; ++k)
                        if (k < h) rv[k] += rv[k + h];
            double v = rv[0];
            for (int m = 64; m > 1;) {
                const int h = (m + 1) >> 1;
                const double o = __shfl_down(v, h);
                if (lane + h < m) v += o;
                m = h;
            }
            v = __shfl(v, 0);
            scale = kq_norm_scale(a, v, &q);
            n = 0;  // done
        } else if (two) {
            red[wave * 64 + lane] = part[0] + part[XJ - 1];
            n = nw * 64;
        } else {
#pragma unroll
            for (int j = 0; j < XJ; ++j)
                if (wave + nw * j < a.nsb) red[(wave + nw * j) * 64 + lane] = part[j];
        }
        if (n) {
        __syncthreads();
        while (n > 64) {  // cross-wave levels through LDS
            const int h = (n + 1) >> 1;
            for (int i = tid; i + h < n; i += nth) red[i] += red[i + h];
            __syncthreads();
            n = h;
        }
        if (wave == 0) {  // the last levels (n <= 64) in wave 0's registers: the same adds
            double v = lane < n ? red[lane] : 0.0;
            while (n > 1) {
                const int h = (n + 1) >> 1;
                const double o = __shfl_down(v, h);
                if (lane + h < n) v += o;
                n = h;
            }
            if (lane == 0) red[0] = v;
        }
        __syncthreads();
        scale = kq_norm_scale(a, red[0], &q);
        }
    }
    auto emit = [&](const kq_pro_regs<XJ> &rv, float sc) {
        float y[XJ][4];
#pragma unroll
        for (int j = 0; j < XJ; ++j) {
            y[j][0] = rv.x[j].x; y[j][1] = rv.x[j].y; y[j][2] = rv.x[j].z; y[j][3] = rv.x[j].w;
            if (a.pro == KQP_NORM) {
                y[j][0] = pin(y[j][0] * sc) * rv.w[j].x;
                y[j][1] = pin(y[j][1] * sc) * rv.w[j].y;
                y[j][2] = pin(y[j][2] * sc) * rv.w[j].z;
                y[j][3] = pin(y[j][3] * sc) * rv.w[j].w;
            }
        }
        if (two) {
            q8K_store_n<XJ>(y, lane, xs + (int64_t)wave * 292, nw * 292);
            return;
        }
#pragma unroll
        for (int j = 0; j < XJ; ++j) {
            const int sb = wave + nw * j;
            if (sb < a.nsb) q8K_store(y[j], lane, xs + (int64_t)sb * 292);  // wave-uniform
        }
    };
    // the check before the one image build (a few integer ops); rare, workgroup-uniform: ggml's own
    // order.  (A second, fallback image build after the first cost the Q4_K_M step 2.5 % — 1,034 vs
    // 1,060 tok/s with the check compiled out — through ~6 KB more code per kernel.)
#ifndef GHIP_KQ_NOCHK  // (A/B builds only: the check's cost)
    if (__builtin_expect(a.pro == KQP_NORM && !rms_mean_certain(q, (int64_t)a.nsb * 256), 0)) scale = kq_seq_scale(a, col);
#endif
    emit(r, scale);
}

__device__ __forceinline__ double *kq_red(uint8_t *xs, int nsb) {
    return (double *)(xs + (((size_t)nsb * 292 + 15) & ~(size_t)15));
}

// write-through (sc1) global accesses for the in-launch hand-off (MI355X_MICROARCH sc1 table row 1,
// the pattern attn_impl.h documents): values read back inside the launch are stored and loaded sc1
typedef __attribute__((address_space(1))) float kq_gfloat;
typedef __attribute__((address_space(1))) unsigned kq_guint;
__device__ __forceinline__ void kq_st_sc1(float *p, float v) {
    __hip_atomic_store((kq_gfloat *)p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ float4 kq_ld4_sc1(const float *p, bool plain = false) {
    if (plain) return *(const float4 *)p;
    return make_float4(__hip_atomic_load((const kq_gfloat *)p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT),
                       __hip_atomic_load((const kq_gfloat *)p + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT),
                       __hip_atomic_load((const kq_gfloat *)p + 2, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT),
                       __hip_atomic_load((const kq_gfloat *)p + 3, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT));
}
__device__ __forceinline__ void kq_put(const kq_args &a, int64_t o, float v) {
    if (a.q8_mode != KQO_NONE && !(a.q8_abl & 4)) kq_st_sc1(a.y + o, v);
    else a.y[o] = v;
}

// Producer-side INIT of the next matvec (kq_args::q8_mode), run by each wave after its rows of group
// g are stored write-through: the wave drains its stores and counts the group on its super-block's
// counter (32 groups); the wave completing a super-block quantizes it (KQO_QUANT) or, for KQO_NORM,
// counts the super-block on the column's counter, and the wave completing the column runs the norm
// and writes all its super-blocks — the bytes k_quant_q8_K / k_norm_q8K write, without their
// launches.  Two counter levels keep each address to <= 32 atomics (one counter per column took
// 256 serialised atomics).  Completing waves reset their counters (the next launch starts at zero).
// Counters: per column, nsb_y super-block slots then the column slot, 32 u32 (128 B) apart.
__device__ __forceinline__ bool kq_count(unsigned *cnt, unsigned target, int lane) {
    unsigned old = 0;
    if (lane == 0) old = __hip_atomic_fetch_add((kq_guint *)cnt, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    old = __builtin_amdgcn_readfirstlane(old);
    if (old != target - 1) return false;
    if (lane == 0) __hip_atomic_store((kq_guint *)cnt, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    return true;
}

// The hand-off tail's sum of squares over the column: partial p = the squares of elements 4p..4p+3
// (p = j*64 + lane, held as part[j]), then a pairwise tree h = (n+1)/2 — levels whose halves are whole
// 64-partial rows combine registers, the last six (n <= 64) combine lanes; anything else goes through
// `lds` (free: every dot loop of the grid has finished).  Returns the total in every lane.  The tree's
// order is not ggml's: the caller keeps its mean only when rms_mean_certain proves it equal to the
// sequential sum's, and otherwise runs seq_sumsq_wave.
__device__ __forceinline__ double kq_tree(double part[8], int J, int lane, double *lds) {
    int n = J * 64;
    bool regs = true;
    while (n > 64) {
        const int h = (n + 1) >> 1;
        if (regs && h % 64 == 0) {
            const int jh = h / 64, jn = n / 64;
#pragma unroll
            for (int j = 0; j < 8; ++j)
                if (j + jh < jn) part[j] += part[j + jh];
        } else {
            if (regs) {  // spill the live rows once, finish the wide levels in LDS
#pragma unroll
                for (int j = 0; j < 8; ++j)
                    if (j * 64 < n) lds[j * 64 + lane] = part[j];
                regs = false;
            }
            __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "wavefront");
            __builtin_amdgcn_wave_barrier();
            for (int i = lane; i + h < n; i += 64) lds[i] += lds[i + h];
        }
        n = h;
    }
    double v = part[0];
    if (!regs) {
        __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "wavefront");
        __builtin_amdgcn_wave_barrier();
        v = lane < n ? lds[lane] : 0.0;
    }
    while (n > 1) {
        const int h = (n + 1) >> 1;
        const double o = __shfl_down(v, h);
        if (lane + h < n) v += o;
        n = h;
    }
    return __shfl(v, 0);
}

// HO: the hand-off kind as a template constant (0 none, 1 KQO_QUANT, 2 KQO_NORM; -1 read from
// a.q8_mode): the norm tail holds the whole column in registers (~200 VGPRs), so a kernel that
// compiles it in runs at 2 waves per SIMD even when it only quantizes (111 VGPRs without it)
template <int HO = -1>
__device__ __forceinline__ void kq_handoff(const kq_args &a, int col, int64_t g, int lane, uint8_t *lds) {
    if (HO == 0 || (HO < 0 && a.q8_mode == KQO_NONE)) return;
    if (a.q8_abl & 2) return;
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    const int nsb_y = (int)(a.rows / 256);
    const bool quant = HO == 1 || (HO < 0 && a.q8_mode == KQO_QUANT);
    const int idx = (int)(g / 32);
    unsigned *cnt = a.q8_cnt + (int64_t)col * (quant ? nsb_y : nsb_y + 1) * 32;
    if (!kq_count(cnt + idx * 32, 32u, lane)) return;
    if ((a.q8_abl & 1) || ((a.q8_abl & 16) && !quant) || ((a.q8_abl & 32) && quant)) return;
    const float *y = a.y + (int64_t)col * a.y_col_stride;
    uint8_t *out = a.q8_out + (int64_t)col * nsb_y * 292;
    if (quant) {
        const float4 v = kq_ld4_sc1(y + (int64_t)idx * 256 + lane * 4, a.q8_abl & 8);
        const float xv[4] = {v.x, v.y, v.z, v.w};
        q8K_store(xv, lane, out + (int64_t)idx * 292);
        return;
    }
    if (HO == 1) return;
    if (!kq_count(cnt + nsb_y * 32, (unsigned)nsb_y, lane)) return;
    // nsb_y <= 8 (launch_matvec_kq checks): the column in registers
    float4 xv[8], wv[8];
    double part[8];
#pragma unroll
    for (int k = 0; k < 8; ++k) {
        const int sb = min(k, nsb_y - 1);
        xv[k] = kq_ld4_sc1(y + (int64_t)sb * 256 + lane * 4, a.q8_abl & 8);
        wv[k] = *(const float4 *)(a.q8_norm + (int64_t)sb * 256 + lane * 4);
    }
#pragma unroll
    for (int k = 0; k < 8; ++k) {
        double p = 0.0;
        p += (double)(xv[k].x * xv[k].x);
        p += (double)(xv[k].y * xv[k].y);
        p += (double)(xv[k].z * xv[k].z);
        p += (double)(xv[k].w * xv[k].w);
        part[k] = p;
    }
    const double sum = kq_tree(part, nsb_y, lane, (double *)lds);
    const double q = div_by_n(sum, a.rows);
    float mean = (float)q;
    if (__builtin_expect(!rms_mean_certain(q, a.rows), 0))  // rare: ggml's own order, from the same sc1 loads
        mean = (float)(seq_sumsq_wave(a.rows, [&](int64_t i0, float v[8]) {
                           const float4 u = kq_ld4_sc1(y + i0, a.q8_abl & 8), w = kq_ld4_sc1(y + i0 + 4, a.q8_abl & 8);
                           v[0] = u.x; v[1] = u.y; v[2] = u.z; v[3] = u.w; v[4] = w.x; v[5] = w.y; v[6] = w.z; v[7] = w.w;
                       }) / (double)a.rows);
    const float scale = 1.0f / sqrtf(mean + a.eps);
    float yv[8][4];
#pragma unroll
    for (int k = 0; k < 8; ++k) {
        yv[k][0] = pin(xv[k].x * scale) * wv[k].x;
        yv[k][1] = pin(xv[k].y * scale) * wv[k].y;
        yv[k][2] = pin(xv[k].z * scale) * wv[k].z;
        yv[k][3] = pin(xv[k].w * scale) * wv[k].w;
    }
    if (nsb_y == 8) {
        q8K_store_n<8>(yv, lane, out);
    } else {
#pragma unroll
        for (int k = 0; k < 8; ++k)
            if (k < nsb_y) q8K_store(yv[k], lane, out + (int64_t)k * 292);
    }
}

// fold the 8 lanes (and the 4 mins lanes) of each row; lane 0 of the 8-group stores
template <int WT>
__device__ __forceinline__ void kq_store(const kq_args &a, int col, int64_t row_raw, int l, float acc, float accm) {
    float v = fold8_dpp(acc);  // ((a0+a4)+(a2+a6))+((a1+a5)+(a3+a7)) in lane 0 of the 8-group
    if (WT == T_Q4_K) v = v + quad_fold_dpp(accm);  // (m0+m2)+(m1+m3) in lane 0
    if (l == 0 && row_raw < a.rows) {
        const int64_t o = (int64_t)col * a.y_col_stride + row_raw;
        if (a.gate_in) {  // gelu(gate) then ggml_mul by up (src/gemma_model.cpp:444-452)
            const float g = a.gate_in[o];
            const float gl = (a.gelu_clamp && g <= -10.0f) ? 0.0f : (a.gelu_clamp && g >= 10.0f) ? g : h2f(a.gelu_tab[f2h(g)]);
            v = gl * v;
        } else if (a.resid) {
            v = v + a.resid[o];
        }
        kq_put(a, o, v);
    }
}

// gate and up of one row: y = gelu(gate) * up (src/gemma_model.cpp:444-452), the gate's value
// rounded exactly as the separate launches stored and re-read it
template <int WT>
__device__ __forceinline__ void kq_store_gu(const kq_args &a, int col, int64_t row_raw, int l, float acc, float accm,
                                            float acc2, float accm2) {
    float g = fold8_dpp(acc), u = fold8_dpp(acc2);
    if (WT == T_Q4_K) {
        g = g + quad_fold_dpp(accm);
        u = u + quad_fold_dpp(accm2);
    }
    if (l == 0 && row_raw < a.rows) {
        const float gl = (a.gelu_clamp && g <= -10.0f) ? 0.0f : (a.gelu_clamp && g >= 10.0f) ? g : h2f(a.gelu_tab[f2h(g)]);
        kq_put(a, (int64_t)col * a.y_col_stride + row_raw, gl * u);
    }
}

#ifndef GHIP_KQ_HEAD_WGS
#define GHIP_KQ_HEAD_WGS 1024  // the single-column output head's grid cap (0: every row group its own wave); Q6_K head cold, same box: uncapped / 512 / 768 / 1024 / 1280 / 2048 / 4096 WGs -> 102.0 / 92.4 / 104.0 / 92.2 / 99.2 / 95.0 / 99.3 us
#endif
#ifndef GHIP_KQ_PAIRW
#define GHIP_KQ_PAIRW 1  // the q|k + v pair as two row groups per 16-wave workgroup (k_matvec_kq_ks2w)
#endif
#ifndef GHIP_KQ_XJ8
#define GHIP_KQ_XJ8 1  // prologue super-blocks per wave of the 8-wave K-split launches when K <= 2048 (q|k+v,
                        // attn-out): 1 = one per wave, no clamped surplus loads; Q4_K_M decode, same box:
                        // 1,160-1,164 vs 1,132-1,141 tok/s with 2
#endif
#ifndef GHIP_KQ_WPE
#define GHIP_KQ_WPE 0  // k_matvec_kq: minimum waves per SIMD the compiler must fit (0: its choice)
#endif
// NT: threads per workgroup.  Every workgroup builds the column's whole Q8_K image (norm + quantize)
// in its prologue, so two 4-wave workgroups per CU build it twice: the gate/up launch (2,048 row
// groups) runs one 8-wave workgroup per CU instead (NT = 512, XJ = 1: one super-block per wave)
template <int WT, bool DUAL, int XJ, bool TL, int HO, int NSB = 0, int PF = KQ_PF, int NT = KQ_THREADS>
__global__ void __launch_bounds__(NT)
#if GHIP_KQ_WPE
__attribute__((amdgpu_waves_per_eu(GHIP_KQ_WPE)))
#endif
k_matvec_kq(kq_args a) {
    extern __shared__ __attribute__((aligned(16))) uint8_t xs[];  // the column's Q8_K blocks
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, rr = lane >> 3, l = lane & 7;
    const int col = blockIdx.y;
    const int64_t n_groups = (a.rows + 7) / 8;
    const int64_t g0 = (int64_t)blockIdx.x * (NT / 64) + wave;
#define KQ_STAMP(i)                                                                                              \
    do {                                                                                                         \
        if (GHIP_STAMPS && a.dbg_t && tid == 0)                                                                  \
            a.dbg_t[((int64_t)blockIdx.y * gridDim.x + blockIdx.x) * 16 + (i)] = __builtin_amdgcn_s_memrealtime(); \
    } while (0)
    KQ_STAMP(0);
    // the first round of weight loads goes out before the Q8_K staging, so its HBM round trip
    // overlaps the activation copy into LDS (the Q4_0 matvec's ring-before-prologue)
    // DUAL (ffn gate and up in one launch): the up matrix w2 (same type and shape) streams beside the
    // gate rows, each in its own ordered chain; the epilogue forms gelu(gate) * up in registers
    kq_pro_regs<XJ> pr;
    kq_pro_load<XJ>(a, col, wave, NT / 64, lane, pr);
    // NSB > 0 (compile-time super-blocks per row, one row group per wave): the rounds of PF
    // super-blocks are software-pipelined — round k + 1's loads go out before round k's arithmetic,
    // into the other half of rb — instead of each round's load waiting behind the previous round's
    // arithmetic (NSB / PF dependent round trips: 6 of the K-quant gate/up's 12 µs, stamps)
    kq_raw<WT> rb[2][PF], rb2[2][DUAL ? PF : 1];
    kq_raw<WT>(&r)[PF] = rb[0];
    kq_raw<WT>(&r2)[DUAL ? PF : 1] = rb2[0];
#if GHIP_KQ_EARLY
    {
        // GHIP_KQ_EARLY 2: every wave's activation loads go out before ANY wave's weight loads (one
        // s_barrier; no wait): a wave's x / w requests no longer queue behind its neighbours' weights
        if (GHIP_KQ_EARLY == 2 && a.pro != KQP_COPY) __builtin_amdgcn_s_barrier();
        const int64_t row0 = g0 * 8 + rr < a.rows ? g0 * 8 + rr : a.rows - 1;
#pragma unroll
        for (int p = 0; p < PF; ++p) {
            r[p] = kq_load<WT, TL>(a.w + row0 * a.row_bytes, p < a.nsb ? p : 0, l);
            if (DUAL) r2[p] = kq_load<WT, TL>(a.w2 + row0 * a.row_bytes, p < a.nsb ? p : 0, l);
        }
    }
    bool early = true;
#else
    constexpr bool early = false;
#endif
    if (GHIP_STAMPS == 1 && a.dbg_t) {  // stamps: the activation loads have landed (the first weight
        // round, issued after them, stays in flight: 2 loads per super-block and matrix, TL Q4_K)
        if (DUAL && TL && WT == T_Q4_K && PF == 2) asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
        else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        KQ_STAMP(6);
    }
    kq_pro_build<XJ>(a, xs, kq_red(xs, a.nsb), col, tid, NT, pr);
    KQ_STAMP(1);
    __syncthreads();
    KQ_STAMP(2);
    if constexpr (NSB > 0 && GHIP_KQ_EARLY) {
        static_assert(NSB % PF == 0, "whole rounds");
        constexpr int NR = NSB / PF;
        static_assert(NR % 2 == 0, "a group's rounds end on the buffer they started on");
        // a wave takes row groups g0, g0 + stride, ... (one, when the grid gives every group its own
        // wave); the pipeline runs ACROSS groups: a group's last round prefetches the next group's
        // first, so a capped grid keeps its loads in flight without a per-workgroup prologue each
        const int64_t stride = (int64_t)gridDim.x * (NT / 64);
        for (int64_t g = g0; g < n_groups; g += stride) {  // wave-uniform
            const int64_t row_raw = g * 8 + rr;
            const int64_t row = row_raw < a.rows ? row_raw : a.rows - 1;
            const uint8_t *wrow = a.w + row * a.row_bytes;
            const uint8_t *wrow2 = DUAL ? a.w2 + row * a.row_bytes : nullptr;
            const bool more = g + stride < n_groups;
            const int64_t row_n = more ? (g + stride) * 8 + rr < a.rows ? (g + stride) * 8 + rr : a.rows - 1 : row;
            const uint8_t *wrow_n = a.w + row_n * a.row_bytes;
            const uint8_t *wrow2_n = DUAL ? a.w2 + row_n * a.row_bytes : nullptr;
            float acc = 0.0f, accm = 0.0f, acc2 = 0.0f, accm2 = 0.0f;
#pragma unroll
            for (int rd = 0; rd < NR; ++rd) {
                if (rd + 1 < NR) {
#pragma unroll
                    for (int p = 0; p < PF; ++p) {
                        rb[(rd + 1) & 1][p] = kq_load<WT, TL>(wrow, (rd + 1) * PF + p, l);
                        if (DUAL) rb2[(rd + 1) & 1][p] = kq_load<WT, TL>(wrow2, (rd + 1) * PF + p, l);
                    }
                } else if (more) {  // the next group's first round
#pragma unroll
                    for (int p = 0; p < PF; ++p) {
                        rb[0][p] = kq_load<WT, TL>(wrow_n, p, l);
                        if (DUAL) rb2[0][p] = kq_load<WT, TL>(wrow2_n, p, l);
                    }
                }
#pragma unroll
                for (int p = 0; p < PF; ++p) {
                    const int sb = rd * PF + p;
                    const kq_term t = kq_terms<WT>(rb[rd & 1][p], xs, sb, l);
                    acc = __builtin_fmaf(t.d, (float)t.sumi, acc);
                    if (WT == T_Q4_K && l < 4) accm = __builtin_fmaf(t.dmin, (float)t.prod, accm);
                    if (DUAL) {
                        const kq_term u = kq_terms<WT>(rb2[rd & 1][p], xs, sb, l);
                        acc2 = __builtin_fmaf(u.d, (float)u.sumi, acc2);
                        if (WT == T_Q4_K && l < 4) accm2 = __builtin_fmaf(u.dmin, (float)u.prod, accm2);
                    }
                }
            }
            KQ_STAMP(3);
            if (DUAL) kq_store_gu<WT>(a, col, row_raw, l, acc, accm, acc2, accm2);
            else kq_store<WT>(a, col, row_raw, l, acc, accm);
            KQ_STAMP(4);
            kq_handoff<HO>(a, col, g, lane, xs);
        }
        KQ_STAMP(5);
        return;
    }
    for (int64_t g = g0; g < n_groups; g += (int64_t)gridDim.x * (NT / 64)) {
        const int64_t row_raw = g * 8 + rr;
        const int64_t row = row_raw < a.rows ? row_raw : a.rows - 1;  // all lanes stay active for the folds
        const uint8_t *wrow = a.w + row * a.row_bytes;
        const uint8_t *wrow2 = DUAL ? a.w2 + row * a.row_bytes : nullptr;
        float acc = 0.0f, accm = 0.0f, acc2 = 0.0f, accm2 = 0.0f;
        for (int s0 = 0; s0 < a.nsb; s0 += PF) {
            if (!early) {
#pragma unroll
                for (int p = 0; p < PF; ++p) {
                    r[p] = kq_load<WT, TL>(wrow, s0 + p < a.nsb ? s0 + p : s0, l);
                    if (DUAL) r2[p] = kq_load<WT, TL>(wrow2, s0 + p < a.nsb ? s0 + p : s0, l);
                }
            }
#if GHIP_KQ_EARLY
            early = false;
#endif
#pragma unroll
            for (int p = 0; p < PF; ++p) {
                if (s0 + p >= a.nsb) break;
                const kq_term t = kq_terms<WT>(r[p], xs, s0 + p, l);
                acc = __builtin_fmaf(t.d, (float)t.sumi, acc);
                if (WT == T_Q4_K && l < 4) accm = __builtin_fmaf(t.dmin, (float)t.prod, accm);
                if (DUAL) {
                    const kq_term u = kq_terms<WT>(r2[p], xs, s0 + p, l);
                    acc2 = __builtin_fmaf(u.d, (float)u.sumi, acc2);
                    if (WT == T_Q4_K && l < 4) accm2 = __builtin_fmaf(u.dmin, (float)u.prod, accm2);
                }
            }
        }
        KQ_STAMP(3);
        if (DUAL) kq_store_gu<WT>(a, col, row_raw, l, acc, accm, acc2, accm2);
        else kq_store<WT>(a, col, row_raw, l, acc, accm);
        KQ_STAMP(4);
        kq_handoff<HO>(a, col, g, lane, xs);
    }
    KQ_STAMP(5);
#undef KQ_STAMP
}

// T-column form (the batched prefill): NC columns per workgroup share every weight load, so the
// weights leave L2 / HBM once per NC prompt rows instead of once per row; each (row, column) is
// still the decode dot in ggml's lane order (one fmaf chain per lane and column), so the result is
// bit-identical.  Q8_K columns precomputed (KQP_COPY), no hand-off.
template <int WT, bool DUAL, int NC, bool TL>
__global__ void __launch_bounds__(KQ_THREADS) k_matmul_kq(kq_args a) {
    extern __shared__ __attribute__((aligned(16))) uint8_t xs[];  // NC columns' Q8_K images
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, rr = lane >> 3, l = lane & 7;
    const int c0 = blockIdx.y * NC;
    const int nc = min(NC, a.ncols - c0);
    const int64_t img = (int64_t)a.nsb * 292;
    for (int c = 0; c < nc; ++c) {
        const uint32_t *src = (const uint32_t *)(a.x + (int64_t)(c0 + c) * a.x_col_stride);
        uint32_t *dst = (uint32_t *)(xs + c * img);
        for (int i = tid; i < a.nsb * 73; i += KQ_THREADS) dst[i] = src[i];
    }
    __syncthreads();
    const int64_t n_groups = (a.rows + 7) / 8;
    for (int64_t g = (int64_t)blockIdx.x * (KQ_THREADS / 64) + wave; g < n_groups;
         g += (int64_t)gridDim.x * (KQ_THREADS / 64)) {
        const int64_t row_raw = g * 8 + rr;
        const int64_t row = row_raw < a.rows ? row_raw : a.rows - 1;
        const uint8_t *wrow = a.w + row * a.row_bytes;
        const uint8_t *wrow2 = DUAL ? a.w2 + row * a.row_bytes : nullptr;
        float acc[NC], accm[NC], acc2[NC], accm2[NC];
#pragma unroll
        for (int c = 0; c < NC; ++c) acc[c] = accm[c] = acc2[c] = accm2[c] = 0.0f;
        for (int s0 = 0; s0 < a.nsb; s0 += KQ_PF) {
            kq_raw<WT> r[KQ_PF], r2[DUAL ? KQ_PF : 1];
#pragma unroll
            for (int p = 0; p < KQ_PF; ++p) {
                r[p] = kq_load<WT, TL>(wrow, s0 + p < a.nsb ? s0 + p : s0, l);
                if (DUAL) r2[p] = kq_load<WT, TL>(wrow2, s0 + p < a.nsb ? s0 + p : s0, l);
            }
#pragma unroll
            for (int p = 0; p < KQ_PF; ++p) {
                if (s0 + p >= a.nsb) break;
#pragma unroll
                for (int c = 0; c < NC; ++c) {
                    const kq_term t = kq_terms<WT>(r[p], xs + c * img, s0 + p, l);
                    acc[c] = __builtin_fmaf(t.d, (float)t.sumi, acc[c]);
                    if (WT == T_Q4_K && l < 4) accm[c] = __builtin_fmaf(t.dmin, (float)t.prod, accm[c]);
                    if (DUAL) {
                        const kq_term u = kq_terms<WT>(r2[p], xs + c * img, s0 + p, l);
                        acc2[c] = __builtin_fmaf(u.d, (float)u.sumi, acc2[c]);
                        if (WT == T_Q4_K && l < 4) accm2[c] = __builtin_fmaf(u.dmin, (float)u.prod, accm2[c]);
                    }
                }
            }
        }
#pragma unroll
        for (int c = 0; c < NC; ++c) {
            if (c >= nc) break;  // wave-uniform
            if (DUAL) kq_store_gu<WT>(a, c0 + c, row_raw, l, acc[c], accm[c], acc2[c], accm2[c]);
            else kq_store<WT>(a, c0 + c, row_raw, l, acc[c], accm[c]);
        }
    }
}

// K split for tall-K / few-row shapes (e.g. ffn_down, 2048 x 16384): one row group per workgroup,
// KS waves each take nsb/KS super-blocks.  Waves 1..KS-1 stash their exact terms (sumi, d[, prod,
// dmin]) in LDS; wave 0 runs its own segment, then continues ITS chain through the stash in
// super-block order — the identical fmaf sequence (the Q4_0 path's ordered carry).
// The body with the prologue's work split over npro threads (ptid this thread's index among them)
// and the dot over this row group's KS waves (htid), its stash at `stash` (the paired form,
// k_matvec_kq_ks2w, runs two row groups per workgroup over one shared Q8_K image built from pa)
template <int WT, int KS, int XJ, int PF, bool TL>
__device__ __forceinline__ void kq_ks_body_g(const kq_args &a, const kq_args &pa, const int gx, const int htid,
                                             const int ptid, const int npro, uint8_t *stash, const bool act) {
    extern __shared__ __attribute__((aligned(16))) uint8_t xs[];
    const int tid = htid, lane = tid & 63, wave = tid >> 6, rr = lane >> 3, l = lane & 7;
    const int col = blockIdx.y, nsb = a.nsb, seg = nsb / KS;
    int *st_i = (int *)stash;                   // [nsb][64] lane sums
    float *st_d = (float *)(st_i + nsb * 64);   // [nsb][8]  per-row d
    int *st_p = (int *)(st_d + nsb * 8);        // [nsb][64] mins products (Q4_K)
    float *st_m = (float *)(st_p + nsb * 64);   // [nsb][8]  per-row dmin (Q4_K)
    const int64_t row_raw = (int64_t)gx * 8 + rr;
    const int64_t row = row_raw < a.rows ? row_raw : a.rows - 1;
    const uint8_t *wrow = a.w + row * a.row_bytes;
    // first round of weight loads before the Q8_K staging (as in k_matvec_kq)
    kq_pro_regs<XJ> pr;
    kq_pro_load<XJ>(pa, col, ptid >> 6, npro >> 6, ptid & 63, pr);
    kq_raw<WT> r[PF];
#if GHIP_KQ_EARLY
    // (the k_matvec_kq EARLY=2 barrier here too — every wave's activation loads first: measured
    // slower, 1,094-1,099 vs 1,104-1,108 tok/s, removed)
#pragma unroll
    for (int p = 0; p < PF; ++p) r[p] = kq_load<WT, TL>(wrow, p < seg ? wave * seg + p : wave * seg, l);
    bool early = true;
#else
    constexpr bool early = false;
#endif
    kq_pro_build<XJ>(pa, xs, kq_red(xs, nsb), col, ptid, npro, pr);  // red overlaps the stash (used before it)
    __syncthreads();
    float acc = 0.0f, accm = 0.0f;
    for (int s0 = wave * seg; s0 < (wave + 1) * seg; s0 += PF) {
    if (!early) {
#pragma unroll
        for (int p = 0; p < PF; ++p) r[p] = kq_load<WT, TL>(wrow, s0 + p < (wave + 1) * seg ? s0 + p : s0, l);
    }
#if GHIP_KQ_EARLY
    early = false;
#endif
#pragma unroll
    for (int p = 0; p < PF; ++p) {
        const int s = s0 + p;
        if (s >= (wave + 1) * seg) break;
        const kq_term t = kq_terms<WT>(r[p], xs, s, l);
        if (wave == 0) {
            acc = __builtin_fmaf(t.d, (float)t.sumi, acc);
            if (WT == T_Q4_K && l < 4) accm = __builtin_fmaf(t.dmin, (float)t.prod, accm);
        } else {
            st_i[s * 64 + lane] = t.sumi;
            if (l == 0) st_d[s * 8 + rr] = t.d;
            if (WT == T_Q4_K) {
                st_p[s * 64 + lane] = t.prod;
                if (l == 0) st_m[s * 8 + rr] = t.dmin;
            }
        }
    }
    }
    __syncthreads();
    if (wave != 0) return;
    for (int s = seg; s < nsb; ++s) {
        acc = __builtin_fmaf(st_d[s * 8 + rr], (float)st_i[s * 64 + lane], acc);
        if (WT == T_Q4_K && l < 4) accm = __builtin_fmaf(st_m[s * 8 + rr], (float)st_p[s * 64 + lane], accm);
    }
    if (!act) return;
    kq_store<WT>(a, col, row_raw, l, acc, accm);
    kq_handoff(a, col, gx, lane, xs);  // waves 1.. are gone: LDS is free
}

template <int WT, int KS, int XJ, int PF, bool TL>
__device__ __forceinline__ void kq_ks_body(const kq_args &a, const int gx) {
    extern __shared__ __attribute__((aligned(16))) uint8_t xs[];
    kq_ks_body_g<WT, KS, XJ, PF, TL>(a, a, gx, (int)threadIdx.x, (int)threadIdx.x, 64 * KS, xs + a.nsb * 292, true);
}

template <int WT, int KS, int XJ, int PF, bool TL>
__global__ void __launch_bounds__(64 * KS) k_matvec_kq_ks(kq_args a) {
    kq_ks_body<WT, KS, XJ, PF, TL>(a, (int)blockIdx.x);
}

// Round-pipelined K split (matvec_rr.hip's form, for the K-quant down shape: 8 x NR super-blocks
// per row, a precomputed Q8_K column).  One row group per workgroup; 8 loader waves interleave over
// K by rounds (round r: loader w takes super-block w + 8r, so a round is 8 consecutive
// super-blocks), each keeping D rounds of its weight loads in flight; a loader turns its
// super-block into the exact terms (sumi, d [, prod, dmin]) of kq_terms and stashes them in one of
// two LDS slots; the 9th wave, the carrier, chains round r-1's eight super-blocks in order while
// the loaders convert round r.  The carrier's chain is the same fmaf sequence over super-blocks
// 0, 1, ... as k_matvec_kq_ks's wave 0 (own segment, then the stash): identical bits.  The column
// goes out first (its loads are the oldest, so its wait never waits for a weight load).
constexpr int KR_NL = 8, KR_NTH = 64 * (KR_NL + 1);
__device__ __forceinline__ void kr_barrier() { asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory"); }

template <int WT, int NR, int D>
__global__ void __launch_bounds__(KR_NTH) k_matvec_kq_rr(kq_args a) {
    extern __shared__ __attribute__((aligned(16))) uint8_t xs[];
    const int tid = threadIdx.x, lane = tid & 63, wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int rr = lane >> 3, l = lane & 7, col = blockIdx.y;
    constexpr int NSB = KR_NL * NR;
    const bool loader = wave < KR_NL;
    const int64_t row_raw = (int64_t)blockIdx.x * 8 + rr;
    const int64_t row = row_raw < a.rows ? row_raw : a.rows - 1;
    const uint8_t *wrow = a.w + row * a.row_bytes;
    constexpr size_t IMG = ((size_t)NSB * 292 + 15) & ~(size_t)15;
    int *st_i = (int *)(xs + IMG);        // [2][8][64] lane sums
    float *st_d = (float *)(st_i + 1024); // [2][8][8]  per-row d
    int *st_p = (int *)(st_d + 128);      // [2][8][64] mins products (Q4_K)
    float *st_m = (float *)(st_p + 1024); // [2][8][8]  per-row dmin (Q4_K)
    // 0) the column (oldest loads), then D rounds of weights, then the column into LDS
    constexpr int N16 = NSB * 292 / 16, CPN = (N16 + KR_NTH - 1) / KR_NTH;
    const uint4 *src = (const uint4 *)(a.x + (int64_t)col * a.x_col_stride);
    uint4 cv[CPN];
#pragma unroll
    for (int k = 0; k < CPN; ++k) {
        const int i = tid + k * KR_NTH;
        cv[k] = src[i < N16 ? i : 0];
    }
    const int w8 = loader ? wave : 0;  // the carrier re-reads loader 0's rounds (L2 hits, unused)
    kq_raw<WT> r[D];
#pragma unroll
    for (int p = 0; p < D; ++p) r[p] = kq_load<WT, true>(wrow, w8 + KR_NL * (p < NR ? p : 0), l);
#pragma unroll
    for (int k = 0; k < CPN; ++k) {
        const int i = tid + k * KR_NTH;
        if (i < N16) ((uint4 *)xs)[i] = cv[k];
    }
    kr_barrier();
    float acc = 0.0f, accm = 0.0f;
    auto chain = [&](int rc) {
        const int sl = rc & 1;
#pragma unroll
        for (int w = 0; w < KR_NL; ++w) {
            acc = __builtin_fmaf(st_d[(sl * 8 + w) * 8 + rr], (float)st_i[(sl * 8 + w) * 64 + lane], acc);
            if (WT == T_Q4_K && l < 4) accm = __builtin_fmaf(st_m[(sl * 8 + w) * 8 + rr], (float)st_p[(sl * 8 + w) * 64 + lane], accm);
        }
    };
    if (!loader) __builtin_amdgcn_s_setprio(3);  // the chain is the critical path
#pragma unroll
    for (int r0 = 0; r0 < NR; ++r0) {
        if (loader) {
            const kq_term t = kq_terms<WT>(r[r0 % D], xs, wave + KR_NL * r0, l);
            if (r0 + D < NR) r[r0 % D] = kq_load<WT, true>(wrow, wave + KR_NL * (r0 + D), l);
            const int sl = r0 & 1;
            st_i[(sl * 8 + wave) * 64 + lane] = t.sumi;
            if (l == 0) st_d[(sl * 8 + wave) * 8 + rr] = t.d;
            if (WT == T_Q4_K) {
                st_p[(sl * 8 + wave) * 64 + lane] = t.prod;
                if (l == 0) st_m[(sl * 8 + wave) * 8 + rr] = t.dmin;
            }
        } else if (r0 > 0) {
            chain(r0 - 1);
        }
        kr_barrier();
    }
    if (loader) return;
    chain(NR - 1);
    kq_store<WT>(a, col, row_raw, l, acc, accm);
}

// Two matrices of one input column in one launch (a layer's q|k and v: Q4_K and Q6_K in Q4_K_M
// files): workgroups [0, g1) run matrix a, the rest matrix b, each exactly as k_matvec_kq_ks would.
template <int WT1, int WT2, int KS, int XJ, int PF, bool TL>
__global__ void __launch_bounds__(64 * KS) k_matvec_kq_ks2(kq_args a, kq_args b, int g1) {
    if ((int)blockIdx.x < g1) kq_ks_body<WT1, KS, XJ, PF, TL>(a, (int)blockIdx.x);
    else kq_ks_body<WT2, KS, XJ, PF, TL>(b, (int)blockIdx.x - g1);
}

// The same pair with TWO row groups per 16-wave workgroup (groups 2w and 2w + 1; g1 even, so a
// workgroup's halves are always of one matrix and its barriers uniform): the Q8_K image of the
// shared input is built once per two groups — 320 one-group workgroups on 256 CUs put two prologues
// on 64 CUs (the launch ends with them)
template <int WT1, int WT2, int XJ, int PF, bool TL>
__global__ void __launch_bounds__(1024) k_matvec_kq_ks2w(kq_args a, kq_args b, int g1, int gt) {
    extern __shared__ __attribute__((aligned(16))) uint8_t xs[];
    const int tid = threadIdx.x, half = tid >> 9;
    const int grp = 2 * (int)blockIdx.x + half;
    const bool act = grp < gt;
    const int g = act ? grp : gt - 1;
    uint8_t *stash = xs + a.nsb * 292 + (size_t)half * a.nsb * (64 * 4 * 2 + 8 * 4 * 2);
    if (2 * (int)blockIdx.x < g1) kq_ks_body_g<WT1, 8, XJ, PF, TL>(a, a, g, tid & 511, tid, 1024, stash, act);
    else kq_ks_body_g<WT2, 8, XJ, PF, TL>(b, a, g - g1, tid & 511, tid, 1024, stash, act);
}

}  // namespace

namespace {

// ggml quantize_row_q8_K (INIT for K-quant src0, restated in oracle/kquants_cpu.cpp): per 256
// values the first element of largest |x| gives max; iscale = -127/max; q = min(127, rne(iscale*x));
// bsums = sums of 16; d = 1/iscale (all-zero block: d = 0, q = 0).  One wave per super-block, 4
// values per lane (all 64 lanes take part).  Divisions in double then rounded: equal to fp32
// division for fp32 operands.
__global__ void __launch_bounds__(64) k_quant_q8_K(const float *x, int64_t ldx, uint8_t *out, int64_t ld_out) {
    const int sb = blockIdx.x, c = blockIdx.y, lane = threadIdx.x;
    const float4 v = *(const float4 *)(x + (int64_t)c * ldx + (int64_t)sb * 256 + lane * 4);
    const float xv[4] = {v.x, v.y, v.z, v.w};
    q8K_store(xv, lane, out + (int64_t)c * ld_out + (int64_t)sb * 292);
}

// rms_norm(x) * w (src/gemma_model.cpp:438-442; ggml: double sum of the fp32 squares, mean as
// float, scale = 1/sqrtf(mean + eps), y = (x*scale)*w) then quantize_row_q8_K: the tied output's
// INIT when token_embd is Q6_K.  One workgroup per row, one wave per super-block (E <= 4096).
__global__ void __launch_bounds__(1024) k_norm_q8K(const float *x, int64_t ldx, const float *w, int E, float eps,
                                                   uint8_t *out, int64_t ld_out) {
    __shared__ double red[1024];
    const int r = blockIdx.x, tid = threadIdx.x, nt = blockDim.x;
    const float4 v = *(const float4 *)(x + (int64_t)r * ldx + tid * 4);
    const float xv[4] = {v.x, v.y, v.z, v.w};
    double part = 0.0;
#pragma unroll
    for (int j = 0; j < 4; ++j) part += (double)(xv[j] * xv[j]);
    // any order (the mean is certified below): DPP wave sums, one word per wave, one
    // barrier — instead of a pairwise tree with a barrier per level
    part = wave_sum_f64(part);
    if ((tid & 63) == 0) red[tid >> 6] = part;
    __syncthreads();
    double tot = 0.0;
    for (int w = 0; w < (nt >> 6); ++w) tot += red[w];
    const double q = div_by_n(tot, E);
    float mean = (float)q;
    if (__builtin_expect(!rms_mean_certain(q, E), 0)) {  // workgroup-uniform; rare: ggml's own order
        const float *xr = x + (int64_t)r * ldx;
        mean = (float)(seq_sumsq_wave(E, [&](int64_t i0, float v[8]) {
                           const float4 u = *(const float4 *)(xr + i0), w4 = *(const float4 *)(xr + i0 + 4);
                           v[0] = u.x; v[1] = u.y; v[2] = u.z; v[3] = u.w; v[4] = w4.x; v[5] = w4.y; v[6] = w4.z; v[7] = w4.w;
                       }) / (double)E);
    }
    const float scale = 1.0f / sqrtf(mean + eps);
    const float4 wv = *(const float4 *)(w + tid * 4);
    const float ww[4] = {wv.x, wv.y, wv.z, wv.w};
    float y[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) y[j] = pin(xv[j] * scale) * ww[j];
    q8K_store(y, tid & 63, out + (int64_t)r * ld_out + (int64_t)(tid >> 6) * 292);
}

// ---- Q6_K token_embd / tied output (llama.cpp's choice for Q4_0 / Q8_0 Gemma files) -------------
// dequantize_row_q6_K of element e of a row (y = d*sc*(q6 - 32), left to right)
// the same element in the lane-contiguous layout (kq_load's TL form)
__device__ __forceinline__ float q6K_elem_t(const uint8_t *row, int64_t i) {
    const int64_t sb = i >> 8;
    const uint8_t *g = row + (sb >> 3) * 1680;
    const int si = (int)(sb & 7), e = (int)(i & 255), n = e >> 7, gq = (e >> 5) & 3, l = e & 31;
    auto qlb = [&](int o) {  // ggml ql byte o (0..127) of this super-block
        const int k = o >> 5, r = o & 31;
        return g[128 * si + 16 * (r >> 2) + 4 * k + (r & 3)];
    };
    auto qhb = [&](int o) {  // ggml qh byte o (0..63)
        const int j = o >> 5, r = o & 31;
        return g[1024 + 64 * si + 8 * (r >> 2) + 4 * j + (r & 3)];
    };
    const int lo = (gq & 1) ? qlb(n * 64 + l + 32) : qlb(n * 64 + l);
    const int q = (((gq & 2) ? lo >> 4 : lo & 15) | (((qhb(n * 32 + l) >> (2 * gq)) & 3) << 4)) - 32;
    const int8_t scv = (int8_t)g[1536 + 16 * si + n * 8 + l / 16 + 2 * gq];
    return pin(h2f(*(const uint16_t *)(g + 1664 + 2 * si)) * (float)scv) * (float)q;
}

__device__ __forceinline__ float q6K_elem(const uint8_t *row, int64_t i) {
    const uint8_t *blk = row + (i >> 8) * 210;
    const int e = (int)(i & 255), n = e >> 7, g = (e >> 5) & 3, l = e & 31;
    const uint8_t *ql = blk + n * 64, *qh = blk + 128 + n * 32;
    const int lo = (g & 1) ? ql[l + 32] : ql[l];
    const int q = (((g & 2) ? lo >> 4 : lo & 15) | (((qh[l] >> (2 * g)) & 3) << 4)) - 32;
    const int8_t scv = ((const int8_t *)(blk + 192))[n * 8 + l / 16 + 2 * g];
    return pin(h2f(*(const uint16_t *)(blk + 208)) * (float)scv) * (float)q;
}

// get_rows(token_embd, tokens) * sqrt(E) (src/gemma_model.cpp:677-679): row t reads token
// tokens[*pos] (decode: the engine's device-side position) or tokens[t] (prefill)
template <bool TL>
__global__ void k_embed_q6K(const uint8_t *embd, int64_t row_bytes, const int *tokens, const int *pos, int E,
                            float scale, float *out) {
    const int t = blockIdx.x;
    const int tok = pos ? tokens[*pos] : tokens[t];
    const uint8_t *row = embd + (int64_t)tok * row_bytes;
    for (int i = threadIdx.x; i < E; i += blockDim.x) out[(int64_t)t * E + i] = (TL ? q6K_elem_t(row, i) : q6K_elem(row, i)) * scale;
}

// ggml rows <-> the lane-contiguous layout of kq_load<WT, true> (one thread per (row, super-block);
// TO: ggml -> lane-contiguous, else back).  src and dst are distinct buffers.
template <int WT, bool TO>
__global__ void k_kq_retile(const uint8_t *src, uint8_t *dst, int64_t rows, int nsb) {
    const int64_t gid = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (gid >= rows * nsb) return;
    const int64_t row = gid / nsb;
    const int sb = (int)(gid % nsb);
    auto mv = [&](int64_t raw, int64_t til) {
        if (TO) dst[til] = src[raw];
        else dst[raw] = src[til];
    };
    if (WT == T_Q4_K) {
        const int64_t b = row * (int64_t)nsb * 144 + (int64_t)sb * 144;
        for (int o = 0; o < 16; ++o) mv(b + o, b + o);
        for (int o = 0; o < 128; ++o) {  // ggml byte 16 + 32j + 4l + c -> 16 + 16l + 4j + c
            const int j = o >> 5, l = (o & 31) >> 2, c = o & 3;
            mv(b + 16 + o, b + 16 + 16 * l + 4 * j + c);
        }
    } else {
        const int64_t rb = (int64_t)nsb * 210, raw = row * rb + (int64_t)sb * 210, g = row * rb + (int64_t)(sb >> 3) * 1680;
        const int i = sb & 7;
        for (int o = 0; o < 128; ++o) {  // ql: ggml byte 32k + 4l + c -> 128i + 16l + 4k + c
            const int k = o >> 5, l = (o & 31) >> 2, c = o & 3;
            mv(raw + o, g + 128 * i + 16 * l + 4 * k + c);
        }
        for (int o = 0; o < 64; ++o) {  // qh: ggml byte 128 + 32j + 4l + c -> 1024 + 64i + 8l + 4j + c
            const int j = o >> 5, l = (o & 31) >> 2, c = o & 3;
            mv(raw + 128 + o, g + 1024 + 64 * i + 8 * l + 4 * j + c);
        }
        for (int o = 0; o < 16; ++o) mv(raw + 192 + o, g + 1536 + 16 * i + o);
        for (int o = 0; o < 2; ++o) mv(raw + 208 + o, g + 1664 + 2 * i + o);
    }
}

// device twin of oracle orc_synth_kquant (splitmix64 stream: draw n of the matrix is mix(st0 +
// (n + 1)·γ), block b's draws start at b·DRAWS) plus make_kmat's rescale d' = f16(f32(d)·f)
__device__ __forceinline__ uint64_t sm64_draw(uint64_t st0, uint64_t n) {
    uint64_t z = st0 + (n + 1) * 0x9E3779B97F4A7C15ull;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}
__device__ __forceinline__ float div1000(float a) { return (float)((double)a / 1000.0); }

template <int WT>
__global__ void k_synth_kquant(uint8_t *out, int64_t nblk, uint64_t st0, float f) {
    const int64_t b = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (b >= nblk) return;
    uint64_t n = (uint64_t)b * (WT == T_Q4_K ? 142u : 209u);
    if (WT == T_Q4_K) {
        uint8_t *x = out + b * 144;
        const uint32_t d = f2h(1e-3f + div1000(3e-3f * (float)(sm64_draw(st0, n++) % 1000)));
        const uint32_t dm = f2h(div1000(2e-3f * (float)(sm64_draw(st0, n++) % 1000)));
        for (int i = 0; i < 12; ++i) x[4 + i] = (uint8_t)sm64_draw(st0, n++);
        for (int i = 0; i < 128; ++i) x[16 + i] = (uint8_t)sm64_draw(st0, n++);
        const uint32_t d2 = f2h(pin(h2f(d) * f)), dm2 = f2h(pin(h2f(dm) * f));
        x[0] = (uint8_t)d2; x[1] = (uint8_t)(d2 >> 8);
        x[2] = (uint8_t)dm2; x[3] = (uint8_t)(dm2 >> 8);
    } else {
        uint8_t *x = out + b * 210;
        for (int i = 0; i < 128; ++i) x[i] = (uint8_t)sm64_draw(st0, n++);
        for (int i = 0; i < 64; ++i) x[128 + i] = (uint8_t)sm64_draw(st0, n++);
        for (int i = 0; i < 16; ++i) x[192 + i] = (uint8_t)(int8_t)((int)(int8_t)(uint8_t)(sm64_draw(st0, n++) % 255) - 127);
        const uint32_t d = f2h(2e-4f + div1000(6e-4f * (float)(sm64_draw(st0, n++) % 1000)));
        const uint32_t d2 = f2h(pin(h2f(d) * f));
        x[208] = (uint8_t)d2; x[209] = (uint8_t)(d2 >> 8);
    }
}

}  // namespace

int launch_quant_q8_K(const float *x, int64_t ldx, int64_t K, int ncols, uint8_t *out, int64_t ld_out,
                      hipStream_t s) {
    if (K % 256 || K <= 0 || ncols <= 0 || ldx % 4 || ld_out % 4 || ((uintptr_t)x & 15)) {
        set_error("quant_q8_K: K must be a multiple of 256 with 16-byte aligned rows");
        return -1;
    }
    hipLaunchKernelGGL(k_quant_q8_K, dim3((unsigned)(K / 256), (unsigned)ncols), dim3(64), 0, s, x, ldx, out, ld_out);
    GHIP_CHECK(hipGetLastError());
    return 0;
}

int launch_norm_q8K(const float *x, int64_t ldx, const float *w, int E, float eps, int rows, uint8_t *out,
                    int64_t ld_out, hipStream_t s) {
    if (E % 256 || E > 4096 || rows <= 0 || ldx % 4 || ld_out % 4) {
        set_error("norm_q8K: needs n_embd % 256 == 0 and n_embd <= 4096");
        return -1;
    }
    hipLaunchKernelGGL(k_norm_q8K, dim3((unsigned)rows), dim3(E / 4), 0, s, x, ldx, w, E, eps, out, ld_out);
    GHIP_CHECK(hipGetLastError());
    return 0;
}

int launch_embed_q6K(const uint8_t *embd, int64_t row_bytes, const int *tokens, const int *pos, int T, int E,
                     float scale, float *out, hipStream_t s, bool tiled) {
    if (E % 256 || T <= 0) {
        set_error("embed_q6K: needs n_embd % 256 == 0");
        return -1;
    }
    if (tiled && E % 2048) {
        set_error("embed_q6K: the lane-contiguous layout needs n_embd % 2048 == 0");
        return -1;
    }
    if (tiled) hipLaunchKernelGGL(k_embed_q6K<true>, dim3((unsigned)T), dim3(256), 0, s, embd, row_bytes, tokens, pos, E, scale, out);
    else hipLaunchKernelGGL(k_embed_q6K<false>, dim3((unsigned)T), dim3(256), 0, s, embd, row_bytes, tokens, pos, E, scale, out);
    GHIP_CHECK(hipGetLastError());
    return 0;
}

int launch_synth_kquant(int wtype, uint8_t *out, int64_t rows, int64_t K, uint64_t seed, float f, hipStream_t s) {
    if ((wtype != T_Q4_K && wtype != T_Q6_K) || K % 256) {
        set_error("synth_kquant: Q4_K / Q6_K with K % 256 == 0");
        return -1;
    }
    const int64_t nblk = rows * (K / 256);
    const uint64_t st0 = seed * 0x2545F4914F6CDD1Dull + (uint64_t)wtype;  // orc_synth_kquant's state
    const unsigned grid = (unsigned)((nblk + 255) / 256);
    if (wtype == T_Q4_K) hipLaunchKernelGGL(k_synth_kquant<T_Q4_K>, dim3(grid), dim3(256), 0, s, out, nblk, st0, f);
    else hipLaunchKernelGGL(k_synth_kquant<T_Q6_K>, dim3(grid), dim3(256), 0, s, out, nblk, st0, f);
    GHIP_CHECK(hipGetLastError());
    return 0;
}

int launch_kq_retile(int wtype, const uint8_t *src, uint8_t *dst, int64_t rows, int64_t K, bool to_tiled, hipStream_t s) {
    if ((wtype != T_Q4_K && wtype != T_Q6_K) || K % 256 || (wtype == T_Q6_K && K % 2048) || rows <= 0 || src == dst) {
        set_error("kq_retile: Q4_K (K % 256 == 0) or Q6_K (K % 2048 == 0), distinct buffers");
        return -1;
    }
    const int nsb = (int)(K / 256);
    const unsigned grid = (unsigned)((rows * nsb + 255) / 256);
    if (wtype == T_Q4_K && to_tiled) hipLaunchKernelGGL((k_kq_retile<T_Q4_K, true>), dim3(grid), dim3(256), 0, s, src, dst, rows, nsb);
    else if (wtype == T_Q4_K) hipLaunchKernelGGL((k_kq_retile<T_Q4_K, false>), dim3(grid), dim3(256), 0, s, src, dst, rows, nsb);
    else if (to_tiled) hipLaunchKernelGGL((k_kq_retile<T_Q6_K, true>), dim3(grid), dim3(256), 0, s, src, dst, rows, nsb);
    else hipLaunchKernelGGL((k_kq_retile<T_Q6_K, false>), dim3(grid), dim3(256), 0, s, src, dst, rows, nsb);
    GHIP_CHECK(hipGetLastError());
    return 0;
}

int launch_matvec_kq2(int t1, const kq_args &a, int t2, const kq_args &b, hipStream_t s) {
    const bool ok = (t1 == T_Q4_K || t1 == T_Q6_K) && (t2 == T_Q4_K || t2 == T_Q6_K) && a.nsb == b.nsb &&
                    a.nsb % 8 == 0 && a.nsb >= 8 && a.nsb <= 16 && a.ncols == 1 && b.ncols == 1 && a.pro == b.pro &&
                    a.q8_mode == KQO_NONE && b.q8_mode == KQO_NONE && !a.w2 && !b.w2 && a.tiled == b.tiled &&
                    a.rows % 8 == 0 && b.rows > 0 && (a.rows + 7) / 8 + (b.rows + 7) / 8 < 2048 &&
                    (a.pro == KQP_COPY ? (a.x && b.x) : (a.xf && b.xf && !((uintptr_t)a.xf & 15) && a.xf_col_stride % 4 == 0 &&
                                                           (a.pro != KQP_NORM || (a.norm_w && !((uintptr_t)a.norm_w & 15)))));
    if (!ok) {
        set_error("matvec_kq2: the pair needs one K <= 4096 (multiple of 2048), one column, the same prologue, no hand-off");
        return -1;
    }
    const size_t img0 = (size_t)a.nsb * 292;
    const size_t red = a.pro == KQP_NORM ? ((img0 + 15) & ~(size_t)15) + (size_t)a.nsb * 64 * sizeof(double) : 0;
    const size_t lds = std::max((size_t)a.nsb * (292 + 64 * 4 * 2 + 8 * 4 * 2), red);
    const int g1 = (int)((a.rows + 7) / 8), g2 = (int)((b.rows + 7) / 8);
    const dim3 grid((unsigned)(g1 + g2), 1);
    const bool wide2 = GHIP_KQ_PAIRW && a.tiled && a.nsb <= 8 && b.nsb <= 8 && g1 % 2 == 0;
    const size_t lds2 = std::max((size_t)a.nsb * (292 + 2 * (64 * 4 * 2 + 8 * 4 * 2)), red);
    const dim3 grid2((unsigned)((g1 + g2 + 1) / 2), 1);
#define GHIP_KQ2(A, B)                                                                                       \
    do {                                                                                                     \
        if (wide2)                                                                                           \
            hipLaunchKernelGGL((k_matvec_kq_ks2w<A, B, 1, 2, true>), grid2, dim3(1024), lds2, s, a, b, g1, g1 + g2); \
        else if (a.tiled && a.nsb <= 8 && b.nsb <= 8)                                                        \
            hipLaunchKernelGGL((k_matvec_kq_ks2<A, B, 8, GHIP_KQ_XJ8, 2, true>), grid, dim3(512), lds, s, a, b, g1); \
        else if (a.tiled) hipLaunchKernelGGL((k_matvec_kq_ks2<A, B, 8, 2, 2, true>), grid, dim3(512), lds, s, a, b, g1); \
        else hipLaunchKernelGGL((k_matvec_kq_ks2<A, B, 8, 2, 2, false>), grid, dim3(512), lds, s, a, b, g1);          \
    } while (0)
    if (t1 == T_Q4_K && t2 == T_Q4_K) GHIP_KQ2(T_Q4_K, T_Q4_K);
    else if (t1 == T_Q4_K) GHIP_KQ2(T_Q4_K, T_Q6_K);
    else if (t2 == T_Q4_K) GHIP_KQ2(T_Q6_K, T_Q4_K);
    else GHIP_KQ2(T_Q6_K, T_Q6_K);
#undef GHIP_KQ2
    GHIP_CHECK(hipGetLastError());
    return 0;
}

int launch_matvec_kq(int wtype, const kq_args &a, hipStream_t s) {
    if ((wtype != T_Q4_K && wtype != T_Q6_K) || a.nsb <= 0 || a.rows <= 0 || a.ncols <= 0 || a.x_col_stride % 4 ||
        a.nsb * 292 > 64 * 1024) {
        set_error("matvec_kq: unsupported type or shape");
        return -1;
    }
    if (a.pro != KQP_COPY &&
        (!a.xf || ((uintptr_t)a.xf & 15) || a.xf_col_stride % 4 || (a.pro == KQP_NORM && (!a.norm_w || ((uintptr_t)a.norm_w & 15))) ||
         (a.pro != KQP_F32 && a.pro != KQP_NORM))) {
        set_error("matvec_kq: fused Q8_K prologue needs 16-byte aligned f32 rows (and norm weights)");
        return -1;
    }
    if (a.tiled && (wtype == T_Q6_K ? a.nsb % 8 : 0)) {
        set_error("matvec_kq: the lane-contiguous Q6_K layout needs K % 2048 == 0");
        return -1;
    }
    if (a.pro == KQP_COPY && !a.x) {
        set_error("matvec_kq: no Q8_K activation");
        return -1;
    }
    if (a.w2 && (a.gate_in || a.resid || !a.gelu_tab)) {
        set_error("matvec_kq: fused gate/up takes the gelu table and no other epilogue");
        return -1;
    }
    if (a.q8_mode != KQO_NONE) {
        const int64_t need = (int64_t)a.ncols * (a.rows / 256 + (a.q8_mode == KQO_NORM ? 1 : 0));
        if ((a.q8_mode != KQO_QUANT && a.q8_mode != KQO_NORM) || a.rows % 256 || !a.q8_out || !a.q8_cnt ||
            (a.q8_mode == KQO_NORM && a.rows > 2048) ||
            need > a.q8_cnt_cap || (a.q8_mode == KQO_NORM && (!a.q8_norm || ((uintptr_t)a.q8_norm & 15))) ||
            a.y_col_stride % 4 || ((uintptr_t)a.y & 15)) {
            set_error("matvec_kq: Q8_K hand-off needs rows % 256 == 0, aligned output, counters and the norm");
            return -1;
        }
    }
    const int64_t groups = (a.rows + 7) / 8;
    const size_t img0 = (size_t)a.nsb * 292;
    const size_t img = std::max(img0, a.q8_mode == KQO_NORM ? (size_t)a.rows * 2 : (size_t)0);  // + the hand-off's tree
    const size_t red = a.pro == KQP_NORM ? ((img0 + 15) & ~(size_t)15) + (size_t)a.nsb * 64 * sizeof(double) : 0;
    // few row groups and a long K: split K over 8 waves (the ordered carry keeps the fmaf chain)
    const size_t lds_ks = std::max(std::max((size_t)a.nsb * (292 + 64 * 4 * 2 + 8 * 4 * 2), red), img);
    // (min super-blocks per row for the split: 8 — the small q|k / v / o shapes then fill 256+
    // workgroups instead of rows/32)
    constexpr int ks_min = 8;
    // many columns (the batched prefill): NC = 4 columns per workgroup share the weight loads
    if (a.ncols >= 4 && a.pro == KQP_COPY && a.q8_mode == KQO_NONE && 4 * img0 <= 160 * 1024) {
        const size_t lds4 = 4 * img0;
        const unsigned gx = (unsigned)std::min<int64_t>((groups + 3) / 4, 4096);
        const dim3 grid(gx, (unsigned)((a.ncols + 3) / 4));
        auto go = [&](const void *fn) -> int {
            if (lds4 > 64 * 1024) GHIP_CHECK(hipFuncSetAttribute(fn, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds4));
            void *args[] = {(void *)&a};
            GHIP_CHECK(hipLaunchKernel(fn, grid, dim3(KQ_THREADS), args, lds4, s));
            return 0;
        };
        const bool d = a.w2 != nullptr;
        if (wtype == T_Q4_K) {
            if (a.tiled) return d ? go((const void *)k_matmul_kq<T_Q4_K, true, 4, true>) : go((const void *)k_matmul_kq<T_Q4_K, false, 4, true>);
            return d ? go((const void *)k_matmul_kq<T_Q4_K, true, 4, false>) : go((const void *)k_matmul_kq<T_Q4_K, false, 4, false>);
        }
        if (a.tiled) return d ? go((const void *)k_matmul_kq<T_Q6_K, true, 4, true>) : go((const void *)k_matmul_kq<T_Q6_K, false, 4, true>);
        return d ? go((const void *)k_matmul_kq<T_Q6_K, true, 4, false>) : go((const void *)k_matmul_kq<T_Q6_K, false, 4, false>);
    }
    // the down shape (64 super-blocks per row, precomputed column, engine layout): round-pipelined,
    // 4 rounds in flight per loader (Q4_K_M decode, same box: the K-split form 1,013-1,015 tok/s;
    // rounds 2 / 3 / 4 / 6 / 8 in flight: 1,032-1,038 / 1,042-1,047 / 1,052 / 1,041-1,044 / 1,017-1,020)
    if (!a.w2 && a.tiled && a.nsb == 64 && a.pro == KQP_COPY && a.q8_mode == KQO_NONE && a.x_col_stride % 16 == 0 &&
        ((uintptr_t)a.x & 15) == 0) {
        const size_t lds_rr = (((size_t)64 * 292 + 15) & ~(size_t)15) + 2 * (1024 + 128) * 4;
        const dim3 grid((unsigned)groups, a.ncols);
        if (wtype == T_Q4_K) hipLaunchKernelGGL((k_matvec_kq_rr<T_Q4_K, 8, 4>), grid, dim3(KR_NTH), lds_rr, s, a);
        else hipLaunchKernelGGL((k_matvec_kq_rr<T_Q6_K, 8, 4>), grid, dim3(KR_NTH), lds_rr, s, a);
        GHIP_CHECK(hipGetLastError());
        return 0;
    }
    if (!a.w2 && groups < 2048 && a.nsb % 8 == 0 && a.nsb >= ks_min && a.nsb <= 64 && lds_ks <= 64 * 1024) {
        const dim3 grid((unsigned)groups, a.ncols);
        // prefetch depth of a wave's segment: 2 (Q4_K_M decode, same box: 2 / 4 / 8 -> 1.158 / 1.174 /
        // 1.214 ms/token; 8 super-blocks of Q6_K raw rows exceed the 63 outstanding loads vmcnt counts)
#define GHIP_KQ_KS(XJ, PF)                                                                                  \
    do {                                                                                                    \
        if (a.tiled) {                                                                                      \
            if (wtype == T_Q4_K) hipLaunchKernelGGL((k_matvec_kq_ks<T_Q4_K, 8, XJ, PF, true>), grid, dim3(512), lds_ks, s, a); \
            else hipLaunchKernelGGL((k_matvec_kq_ks<T_Q6_K, 8, XJ, PF, true>), grid, dim3(512), lds_ks, s, a);            \
        } else {                                                                                            \
            if (wtype == T_Q4_K) hipLaunchKernelGGL((k_matvec_kq_ks<T_Q4_K, 8, XJ, PF, false>), grid, dim3(512), lds_ks, s, a); \
            else hipLaunchKernelGGL((k_matvec_kq_ks<T_Q6_K, 8, XJ, PF, false>), grid, dim3(512), lds_ks, s, a);            \
        }                                                                                                   \
    } while (0)
        if (a.nsb <= 8) GHIP_KQ_KS(GHIP_KQ_XJ8, 2);
        else if (a.nsb <= 16) GHIP_KQ_KS(2, 2);
        else GHIP_KQ_KS(8, 2);
#undef GHIP_KQ_KS
        GHIP_CHECK(hipGetLastError());
        return 0;
    }
    if (a.pro != KQP_COPY && a.nsb > 32) {
        set_error("matvec_kq: fused Q8_K prologue takes at most 32 super-blocks per row on this shape");
        return -1;
    }
    // the output head (single matrix, precomputed image, 32,000 row groups): every row group its own
    // wave (the grid uncapped) and its rounds software-pipelined (Q4_K_M 1,089-1,094 -> 1,103-1,109
    // tok/s; the uncapped grid alone: 1,091-1,094; the gate/up rounds pipelined too: neutral, removed)
    const bool single_out = !a.w2 && a.pro == KQP_COPY && a.q8_mode == KQO_NONE && a.ncols == 1;
    const bool uncap = single_out;
    const unsigned grid_x = (unsigned)std::min<int64_t>((groups + 3) / 4, uncap ? (GHIP_KQ_HEAD_WGS ? GHIP_KQ_HEAD_WGS : (int64_t)1 << 30) : 4096);
    const size_t lds = std::max(img, red);
    if (lds > 64 * 1024) {
        set_error("matvec_kq: row too long for the LDS image");
        return -1;
    }
    const dim3 grid(grid_x, a.ncols);
    const int ho = a.q8_mode == KQO_NONE ? 0 : a.q8_mode == KQO_QUANT ? 1 : 2;
#define GHIP_KQ_LAUNCH_HO(DUAL, XJ, HO, NSB)                                                                  \
    do {                                                                                                      \
        if (a.tiled) {                                                                                        \
            if (wtype == T_Q4_K) hipLaunchKernelGGL((k_matvec_kq<T_Q4_K, DUAL, XJ, true, HO, NSB>), grid, dim3(KQ_THREADS), lds, s, a); \
            else hipLaunchKernelGGL((k_matvec_kq<T_Q6_K, DUAL, XJ, true, HO, NSB>), grid, dim3(KQ_THREADS), lds, s, a);            \
        } else {                                                                                              \
            if (wtype == T_Q4_K) hipLaunchKernelGGL((k_matvec_kq<T_Q4_K, DUAL, XJ, false, HO, NSB>), grid, dim3(KQ_THREADS), lds, s, a); \
            else hipLaunchKernelGGL((k_matvec_kq<T_Q6_K, DUAL, XJ, false, HO, NSB>), grid, dim3(KQ_THREADS), lds, s, a);            \
        }                                                                                                     \
    } while (0)
#define GHIP_KQ_LAUNCH(DUAL, XJ)                 \
    do {                                         \
        if (ho == 0) GHIP_KQ_LAUNCH_HO(DUAL, XJ, 0, 0); \
        else if (ho == 1) GHIP_KQ_LAUNCH_HO(DUAL, XJ, 1, 0); \
        else GHIP_KQ_LAUNCH_HO(DUAL, XJ, 2, 0);  \
    } while (0)
    const bool wide = a.pro != KQP_COPY && a.nsb > 8;  // more than 2 super-blocks per wave
    // the output head's rows of 8 super-blocks: the software-pipelined rounds (NSB = 8) when every row
    // group has its own wave (the gate/up in that form measured 1,044-1,045 vs 1,044-1,054 tok/s
    // without it: dropped)
    const bool pipe8 = GHIP_KQ_EARLY && a.nsb == 8 && !wide;  // (a capped grid: several groups per wave, one pipeline)
    if (a.w2 && !wide && a.nsb <= 8 && a.tiled && wtype == T_Q4_K && ho == 1) {
        // one 8-wave workgroup per CU, so each CU builds the Q8_K image once (the 4-wave form builds
        // it in both of a CU's workgroups: stamps put the build at 2.9 us of a 14 us launch)
        const dim3 g8((unsigned)std::min<int64_t>((groups + 7) / 8, 4096), a.ncols);
        // (its rounds software-pipelined, NSB = 8: 816 vs 1,132-1,141 tok/s — not kept)
        hipLaunchKernelGGL((k_matvec_kq<T_Q4_K, true, 1, true, 1, 0, KQ_PF, 512>), g8, dim3(512), lds, s, a);
    } else if (a.w2) {
        if (wide) GHIP_KQ_LAUNCH(true, 8);
        else GHIP_KQ_LAUNCH(true, 2);
    } else if (single_out && pipe8) {
        GHIP_KQ_LAUNCH_HO(false, 2, 0, 8);
    } else {
        if (wide) GHIP_KQ_LAUNCH(false, 8);
        else GHIP_KQ_LAUNCH(false, 2);
    }
#undef GHIP_KQ_LAUNCH
#undef GHIP_KQ_LAUNCH_HO
    GHIP_CHECK(hipGetLastError());
    return 0;
}

}  // namespace ghip
