// attn_impl.h — one token's attention for one query head (the per-head form), shared by the
// standalone decode kernel (ops.hip k_attn_head) and the fused layer-front kernel (layer_front.hip).
//
// RoPE-NEOX (src/gemma_model.cpp:698-716) + q scale (:708) + KV store (:499-518) + KQ (:474) +
// soft_max_ext (:476) + KQV (:485) + permute/cont (:487-489) with ggml's AVX/F16C vec_dot_f16 order
//  and the fp16 exp table (A.6).  SC1: the q|k|v input was handed off inside the same
// launch (sc1 loads) and the output's Q8_0 image is handed on (sc1 stores) — MI355X_MICROARCH
// §inter-workgroup visibility, row 1 of the sc1 table.
#pragma once

#include "device_util.h"
#include "kernels.h"
#include "q8k.h"

namespace ghip {
namespace {

// ---- ggml_vec_dot_f16 order on 32 per-thread accumulators -------------------------
__device__ __forceinline__ float reduce_f16_acc(const float acc[4][8]) {
    float x0[8];
#pragma unroll
    for (int l = 0; l < 8; ++l) {
        const float a = acc[0][l] + acc[2][l];
        const float b = acc[1][l] + acc[3][l];
        x0[l] = a + b;
    }
    float t0[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) t0[i] = x0[i] + x0[i + 4];
    const float h0 = t0[0] + t0[1], h1 = t0[2] + t0[3];
    return h0 + h1;
}

// 32 fp16 of x (global/LDS) against 32 fp16 of y: one "step" of the AVX loop
__device__ __forceinline__ void f16_step(float acc[4][8], const uint4 *x4, const uint4 *y4) {
#pragma unroll
    for (int j = 0; j < 4; ++j) {
        const uint4 xv = x4[j], yv = y4[j];
        const uint32_t xs[4] = {xv.x, xv.y, xv.z, xv.w}, ys[4] = {yv.x, yv.y, yv.z, yv.w};
#pragma unroll
        for (int w = 0; w < 4; ++w) {
            acc[j][2 * w] = __builtin_fmaf(h2f(xs[w]), h2f(ys[w]), acc[j][2 * w]);
            acc[j][2 * w + 1] = __builtin_fmaf(h2f(xs[w] >> 16), h2f(ys[w] >> 16), acc[j][2 * w + 1]);
        }
    }
}

#ifndef GHIP_ATT_THREADS
#define GHIP_ATT_THREADS 1024
#endif
constexpr int ATT_THREADS = GHIP_ATT_THREADS;
constexpr int ATT_QUADS = ATT_THREADS / 4;  // one KQ (position, head) or KQV (dim, head) pair per quad
constexpr int ATT_VW = 256;                 // V positions staged in LDS per dimension row (n_kv <= 256)
constexpr int ATT_STG = 2;                  // staging uint4 per thread for each of K and V
constexpr int ATT_MAXWG = 256;              // co-resident workgroups (in-kernel hand-off)

// ggml_vec_dot_f16 with accumulator row j = t4 held by lane t4 of a quad: fold the
// quad exactly as sum0+=sum2, sum1+=sum3, sum0+=sum1 (xor-2 then xor-1), then halves and hadds.
__device__ __forceinline__ float quad_reduce_f16(const float acc[8]) {
    float x0[8];
#pragma unroll
    for (int l = 0; l < 8; ++l) x0[l] = quad_fold_dpp(acc[l]);
    float t0[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) t0[i] = x0[i] + x0[i + 4];
    const float h0 = t0[0] + t0[1], h1 = t0[2] + t0[3];
    return h0 + h1;
}

// acc = fmaf((float)x16, (float)y16, acc) in ONE instruction: v_fma_mix_f32 converts its f16
// operands exactly and rounds the fused result once — the F16C/FMA step of ggml_vec_dot_f16.
__device__ __forceinline__ float fma_mix_lo(uint32_t x, uint32_t y, float acc) {
    float r;
    asm("v_fma_mix_f32 %0, %1, %2, %3 op_sel_hi:[1,1,0]" : "=v"(r) : "v"(x), "v"(y), "v"(acc));
    return r;
}
__device__ __forceinline__ float fma_mix_hi(uint32_t x, uint32_t y, float acc) {
    float r;
    asm("v_fma_mix_f32 %0, %1, %2, %3 op_sel:[1,1,0] op_sel_hi:[1,1,0]" : "=v"(r) : "v"(x), "v"(y), "v"(acc));
    return r;
}
__device__ __forceinline__ void f16_step8(float acc[8], uint4 xv, uint4 yv) {
    const uint32_t xs[4] = {xv.x, xv.y, xv.z, xv.w}, ys[4] = {yv.x, yv.y, yv.z, yv.w};
#pragma unroll
    for (int w = 0; w < 4; ++w) {
        acc[2 * w] = fma_mix_lo(xs[w], ys[w], acc[2 * w]);
        acc[2 * w + 1] = fma_mix_hi(xs[w], ys[w], acc[2 * w + 1]);
    }
}

// positions per KQ block (PS) and dims per KQV workgroup (DS): quads = PS*G and DS*G <= 64, and
// the staged K rows (PS*hd halfs) and V rows (DS*ATT_VW halfs) fit ATT_STG uint4 per thread
struct attn_split {
    int ps, ds;
};
__host__ __device__ inline attn_split attn_split_of(int G, int hd) {
    // KQV slices of at most 32 dims: one Q8_0 block of each head's output per workgroup (image)
    int ps = ATT_QUADS / G, ds = ATT_QUADS / G < 32 ? ATT_QUADS / G : 32;
    const int cap = ATT_STG * ATT_THREADS * 8;  // halfs
    if (ps * hd > cap) ps = cap / hd;
    if (ds * ATT_VW > cap) ds = cap / ATT_VW;
    return {ps, ds};
}

// Cross-workgroup hand-off (MI355X_MICROARCH §inter-workgroup visibility, row 1 of the sc1 table):
// every byte handed off is stored and loaded with global sc1 accesses; each storing wave drains
// vmcnt before the workgroup barrier, then one lane adds to the counter; the consumer polls the
// counter with an sc1 load and joins a barrier before any of its sc1 loads.
typedef __attribute__((address_space(1))) float gfloat_t;
typedef __attribute__((address_space(1))) int gint_t;
__device__ __forceinline__ void st_sc1(float *p, float v) {
    __hip_atomic_store((gfloat_t *)p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ float ld_sc1(const float *p) {
    return __hip_atomic_load((const gfloat_t *)p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ int ld_sc1_i(const int *p) {
    return __hip_atomic_load((const gint_t *)p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}


typedef __attribute__((address_space(1))) uint32_t guint_t;
__device__ __forceinline__ void st_sc1_u(uint32_t *p, uint32_t v) {
    __hip_atomic_store((guint_t *)p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ uint32_t ld_sc1_u(const uint32_t *p) {
    return __hip_atomic_load((const guint_t *)p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
template <bool SC1>
__device__ __forceinline__ float4 ld4(const float *p) {
    if (!SC1) return *(const float4 *)p;
    return make_float4(ld_sc1(p), ld_sc1(p + 1), ld_sc1(p + 2), ld_sc1(p + 3));
}
template <bool SC1>
__device__ __forceinline__ float ld1(const float *p) {
    return SC1 ? ld_sc1(p) : *p;
}
// image_put_quad with write-through (sc1) stores (device_util.h)
__device__ __forceinline__ void image_put_quad_sc1(uint32_t *act, float *da, int64_t b, int q, const float v[8]) {
    float amax = 0.0f;
#pragma unroll
    for (int j = 0; j < 8; ++j) amax = fmaxf(amax, fabsf(v[j]));
    amax = fmaxf(amax, dpp_f<0xB1>(amax));
    amax = fmaxf(amax, dpp_f<0x4E>(amax));
    const float d = amax / 127.f;
    const uint32_t d16 = f2h(d);
    const float id = (amax != 0.0f) ? 127.f / amax : 0.0f;
#pragma unroll
    for (int hh = 0; hh < 2; ++hh) {
        const int l = 2 * q + hh;
        int qi[4];
#pragma unroll
        for (int k = 0; k < 4; ++k) qi[k] = (int)__builtin_rintf(v[4 * hh + k] * id);
        const uint32_t packed = (uint32_t)(qi[0] & 0xFF) | ((uint32_t)(qi[1] & 0xFF) << 8) |
                                ((uint32_t)(qi[2] & 0xFF) << 16) | ((uint32_t)(qi[3] & 0xFF) << 24);
        st_sc1_u(act + ((b >> 2) * 8 + l) * 4 + (b & 3), packed);
    }
    if (q == 0) st_sc1(da + b, h2f(d16));
}

// image_put_quad publishing {payload, tag} granules (the persistent token launch's hand-off,
// MI355X_MICROARCH handoff-1to1): granule i of act is dword i of the image, da[b] the block scale
typedef __attribute__((address_space(1))) unsigned long long gull_t;
__device__ __forceinline__ void put_granule(unsigned long long *g, uint32_t tag, uint32_t v) {
    __hip_atomic_store((gull_t *)g, ((unsigned long long)tag << 32) | v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ void image_put_quad_gran(unsigned long long *act, unsigned long long *da, uint32_t tag, int64_t b,
                                                    int q, const float v[8]) {
    float amax = 0.0f;
#pragma unroll
    for (int j = 0; j < 8; ++j) amax = fmaxf(amax, fabsf(v[j]));
    amax = fmaxf(amax, dpp_f<0xB1>(amax));
    amax = fmaxf(amax, dpp_f<0x4E>(amax));
    const float d = amax / 127.f;
    const uint32_t d16 = f2h(d);
    const float id = (amax != 0.0f) ? 127.f / amax : 0.0f;
#pragma unroll
    for (int hh = 0; hh < 2; ++hh) {
        const int l = 2 * q + hh;
        int qi[4];
#pragma unroll
        for (int k = 0; k < 4; ++k) qi[k] = (int)__builtin_rintf(v[4 * hh + k] * id);
        const uint32_t packed = (uint32_t)(qi[0] & 0xFF) | ((uint32_t)(qi[1] & 0xFF) << 8) |
                                ((uint32_t)(qi[2] & 0xFF) << 16) | ((uint32_t)(qi[3] & 0xFF) << 24);
        put_granule(act + ((b >> 2) * 8 + l) * 4 + (b & 3), tag, packed);
    }
    if (q == 0) put_granule(da + b, tag, __builtin_bit_cast(uint32_t, h2f(d16)));
}

constexpr int AH_THREADS = 1024;  // per-head form: 256 quads = 256 KQ positions / KQV dims per pass
#ifndef GHIP_AH_PF
#define GHIP_AH_PF 4
#endif
#ifndef GHIP_AH_KPF
#define GHIP_AH_KPF GHIP_AH_PF
#endif
#ifndef GHIP_AH_VPF
#define GHIP_AH_VPF GHIP_AH_PF
#endif
constexpr int AH_KPF = GHIP_AH_KPF;  // K steps (of 32 elements) prefetched per lane: hd <= 256
constexpr int AH_VPF = GHIP_AH_VPF;  // V steps (of 32 positions) prefetched per lane: n_kv <= 256

#ifndef GHIP_AH_SPOS
#define GHIP_AH_SPOS 1  // the position by a scalar load, the wave index uniform (readfirstlane)
#endif
// (measured slower and removed, DESIGN.md §10: dead-load trims of the V / K prefetch, the RoPE on the
// last wave with its prefetch after it, V loads issued after the K dots)
#ifndef GHIP_AH_ABL
#define GHIP_AH_ABL 0  // timing ablations only (wrong results): 1 every K load reads row 0, 2 no KQ dots,
                       // 4 no KQ phase at all, 8 no KQV dots, 16 KQ dots over 4 of 8 steps
#endif
#define AH_STAMP(i)                                                                                         \
    do {                                                                                                    \
        if (GHIP_STAMPS && a.dbg_t && tid == 0) a.dbg_t[(int64_t)h * 8 + (i)] = __builtin_amdgcn_s_memrealtime(); \
    } while (0)
// stamps build 3: the workgroup's shader-clock cycles (s_memtime) and 10 ns ticks (s_memrealtime)
// from its start to its end in slots 5 / 6 (split 0 only), so the host reads the core clock it ran at
#define AH_CLK0()                                                                                           \
    unsigned long long clk_c0 = 0, clk_r0 = 0;                                                              \
    if (GHIP_STAMPS == 3) { clk_c0 = __builtin_amdgcn_s_memtime(); clk_r0 = __builtin_amdgcn_s_memrealtime(); }
#define AH_CLK1()                                                                                           \
    do {                                                                                                    \
        if (GHIP_STAMPS == 3 && a.dbg_t && tid == 0 && sp == 0) {                                           \
            const unsigned long long c1 = __builtin_amdgcn_s_memtime(), r1 = __builtin_amdgcn_s_memrealtime(); \
            a.dbg_t[(int64_t)h * 8 + 5] = c1 - clk_c0;                                                      \
            a.dbg_t[(int64_t)h * 8 + 6] = r1 - clk_r0;                                                      \
        }                                                                                                   \
    } while (0)

// Workgroup barrier on LDS traffic only (s_waitcnt lgkmcnt(0); s_barrier): __syncthreads() would
// also drain vmcnt, i.e. hold every wave at the RoPE barrier until its K / V prefetch has landed.
// Register operands of global loads stay guarded by the compiler's counted vmcnt waits at their use.
__device__ __forceinline__ void attn_barrier() { asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory"); }

// K/V rows of the first pass (no dependence on this token's q|k|v): KPF K steps of 32 elements for
// position `quad`, VPF V steps of 32 positions for dimension `quad`, and the published position
template <int KPF, int VPF>
struct attn_pre {
    uint4 k[KPF], v[VPF];
    int pos_v;
};
template <int NTH, int KPF, int VPF>
__device__ __forceinline__ void attn_prefetch(const attn_args &a, const int h, attn_pre<KPF, VPF> &p, int d_lo = 0,
                                              int d_hi = 1 << 30, int tid_in = -1) {
    const int hd = a.hd, tid = tid_in >= 0 ? tid_in : (int)threadIdx.x, t4 = tid & 3, quad = tid >> 2;
    const int G = a.H / a.Hkv, kvh = h / G, kvw = a.Hkv * hd;
    // published with the row (k_advance / begin); a scalar load (constant address space): its own
    // counter, so reading pos waits for no vector load
#if GHIP_AH_SPOS
    p.pos_v = *((const __attribute__((address_space(4))) int *)a.rope_cur + hd);
#else
    p.pos_v = ((const int *)a.rope_cur)[hd];
#endif
    {
        const int j = (GHIP_AH_ABL & 1) ? 0 : quad < a.ctx ? quad : 0;  // no dependency on pos: rows >= pos are masked
        const uint16_t *krow = a.kc + (int64_t)j * kvw + (int64_t)kvh * hd + t4 * 8;
#pragma unroll
        for (int s = 0; s < KPF; ++s) p.k[s] = *(const uint4 *)(krow + (s * 32 < hd ? s * 32 : 0));
    }
    const int d0 = d_lo + quad < (hd < d_hi ? hd : d_hi) ? d_lo + quad : d_lo;
    const uint16_t *vrow0 = a.vc + ((int64_t)kvh * hd + d0) * a.ctx;
#pragma unroll
    for (int s = 0; s < VPF; ++s) p.v[s] = *(const uint4 *)(vrow0 + (s * 32 < a.ctx ? s * 32 : 0) + t4 * 8);
}

// One token's attention for query head h by one NTH-thread workgroup (SURVEY A.4/A.6 order).
// PRE: the K/V prefetch `pre` was issued by the caller (the fused kernel issues it before waiting
// for q|k|v); otherwise it is issued here, after the RoPE inputs (issue order = wait order).
// sp: with a.dsplit = S > 1, S workgroups serve head h, each the whole KQ / softmax (K rows are
// shared through the XCD's L2) and the KQV of output dims [sp*hd/S, (sp+1)*hd/S) — each output
// is still one vec_dot_f16 in ggml's order, so the split changes no bits, only how much of V
// each CU streams.
// SC1O: the output's Q8_0 image stored write-through (sc1) for a consumer inside the same launch
// (k_attn_o, layer_front.hip); defaults to SC1 (the inputs were handed off in-launch too)
template <int NTH, bool SC1, int KPF = AH_KPF, int VPF = AH_VPF, bool PRE = false, bool SC1O = SC1>
__device__ void attn_head_dev(const attn_args &a, const int h, uint8_t *smem, const attn_pre<KPF, VPF> *pre = nullptr,
                              const int sp = 0, const int tid_in = -1) {
    // tid_in: the caller's (opaque) thread index, so that a persistent caller's loop does not keep
    // this function's per-lane addresses live across its other phases
    const int hd = a.hd, half = hd / 2, tid = tid_in >= 0 ? tid_in : (int)threadIdx.x, t4 = tid & 3, quad = tid >> 2;
    const int dsz = hd / (a.dsplit > 1 ? a.dsplit : 1), d_lo = sp * dsz, d_hi = d_lo + dsz;
    // wave: uniform for the compiler too (readfirstlane), so branches on it are scalar branches
    const int lane = tid & 63, wave = GHIP_AH_SPOS ? __builtin_amdgcn_readfirstlane(tid >> 6) : tid >> 6, nwave = NTH / 64;
    const int G = a.H / a.Hkv, kvh = h / G;
    AH_STAMP(0);
    AH_CLK0();
    const int kvw = a.Hkv * hd;
    const float *qh = a.qkv + (int64_t)h * hd;
    const float *kh = a.qkv + (int64_t)a.H * hd + (int64_t)kvh * hd;
    const float *vh = a.qkv + (int64_t)a.H * hd + kvw + (int64_t)kvh * hd;
    const float *cs = a.rope_cur, *sn = a.rope_cur + half;
    // ---- early loads (issue order = wait order): RoPE inputs + pos, then K rows, then V rows
    // RoPE inputs: only the RoPE wave loads them (every load instruction costs the CU's load path
    // ~16 clk whatever its addresses; a wave-uniform branch skips the others)
    const int rl = tid;  // the RoPE lanes: wave 0 (hd <= 512: 64 lanes suffice)
    const int n4 = half / 4, i4 = (rl >= 0 && rl < n4 ? rl : 0) * 4;
    float4 qa{}, qb{}, ka{}, kb{}, ca{}, sa{};
    if (wave * 64 < n4) {
        qa = ld4<SC1>(qh + i4); qb = ld4<SC1>(qh + i4 + half);
        ka = ld4<SC1>(kh + i4); kb = ld4<SC1>(kh + i4 + half);
        ca = *(const float4 *)(cs + i4); sa = *(const float4 *)(sn + i4);
    }
    attn_pre<KPF, VPF> own;
    if (!PRE) attn_prefetch<NTH, KPF, VPF>(a, h, own, d_lo, d_hi, tid);
    const attn_pre<KPF, VPF> &P = PRE ? *pre : own;
    const uint4 *kpre = P.k, *vpre = P.v;
    const int d0 = d_lo + quad < d_hi ? d_lo + quad : d_lo;
    const float vx0 = ld1<SC1>(vh + d0);

    uint16_t *q16 = (uint16_t *)smem;  // hd
    uint16_t *k16 = q16 + hd;          // hd (this token's k, post-rope)
    float *S = (float *)(smem + ((2 * hd * 2 + 15) & ~15));  // ctx
    uint16_t *P16 = (uint16_t *)(S + a.ctx);                 // ctx
    // softmax reduction words (8-aligned, after P16): the row max as an order-preserving key, and
    // the exact integer sum of the e values (both order-independent, so partial results combine in
    // any order and the bits equal a one-wave reduction's)
    uint32_t *mx_key = (uint32_t *)(smem + ((((2 * hd * 2 + 15) & ~15) + a.ctx * 6 + 7) & ~7));
    unsigned long long *e_sum = (unsigned long long *)(mx_key + 2);

    // RoPE NEOX on q (then * q_scale) and on k; f32 -> f16 (ggml_cpy / MUL_MAT INIT conversions)
    auto rope4 = [&](float4 x0v, float4 x1v, float scale, bool scaled, uint16_t *lo, uint16_t *hi) {
        const float x0s[4] = {x0v.x, x0v.y, x0v.z, x0v.w}, x1s[4] = {x1v.x, x1v.y, x1v.z, x1v.w};
        const float cs4[4] = {ca.x, ca.y, ca.z, ca.w}, sn4[4] = {sa.x, sa.y, sa.z, sa.w};
        uint32_t l2[2] = {0, 0}, h2[2] = {0, 0};
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            const float x0 = x0s[k], x1 = x1s[k], c = cs4[k], s = sn4[k];
            const float p0 = x0 * c, p1 = x1 * s, p2 = x0 * s, p3 = x1 * c;
            const float r0 = p0 - p1, r1 = p2 + p3;
            const uint32_t a0 = scaled ? f2h(r0 * scale) : f2h(r0), a1 = scaled ? f2h(r1 * scale) : f2h(r1);
            l2[k >> 1] |= a0 << (16 * (k & 1));
            h2[k >> 1] |= a1 << (16 * (k & 1));
        }
        *(uint2 *)lo = make_uint2(l2[0], l2[1]);
        *(uint2 *)hi = make_uint2(h2[0], h2[1]);
    };
    if (rl >= 0 && rl < n4) {
        rope4(qa, qb, a.q_scale, true, q16 + i4, q16 + i4 + half);
        rope4(ka, kb, 1.0f, false, k16 + i4, k16 + i4 + half);
    }
    if (rl == 0) {  // (the RoPE wave: its loads are drained here; another wave could wait on them)
        *mx_key = 0u;  // below the key of every float, -inf included
        *e_sum = 0ull;
    }
    const int pos = __builtin_amdgcn_readfirstlane(P.pos_v);
    const int n_total = pos + 1;
    int n_kv = 32 * (n_total / 32 + 1);  // src/gemma_model.cpp:429
    if (n_kv > a.ctx) n_kv = a.ctx;
    attn_barrier();  // LDS only: the K / V prefetch stays in flight
    AH_STAMP(1);
    // this token's cache entries (src/gemma_model.cpp:506-517), by the group's first head; readers
    // in this launch use k16 / the v values instead
    if (h % G == 0 && sp == 0) {
        for (int i = tid; i < hd; i += NTH) a.kc[(int64_t)pos * kvw + (int64_t)kvh * hd + i] = k16[i];
        for (int d = quad; d < hd; d += NTH / 4)
            if (t4 == 0) a.vc[((int64_t)kvh * hd + d) * a.ctx + pos] = f2h(d == d0 ? vx0 : ld1<SC1>(vh + d));
    }
    // ---- KQ (vec_dot_f16 over hd per kv position) + mask (j > pos -> -inf), scale 1.0
    float lmax = -INFINITY;
    // q in registers: every position's dot reads the same hd/32 steps (one LDS round trip here
    // instead of one per step and position)
    uint4 qr[8];
#pragma unroll
    for (int s = 0; s < 8; ++s) qr[s] = *(const uint4 *)(q16 + (s * 32 < hd ? s * 32 : 0) + t4 * 8);
    if (GHIP_STAMPS == 4) {  // KQ sub-stamps (stamps build 4): q in registers
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        AH_STAMP(5);
    }
    for (int j0 = 0; j0 < n_kv; j0 += NTH / 4) {
        const int j = j0 + quad;
        // a wave whose 16 positions all lie past n_kv has nothing to store: skip its dots (wave-
        // uniform; its lmax stays -inf, below every stored score)
        if (j0 + wave * 16 >= n_kv || (GHIP_AH_ABL & 4)) continue;
        float acc[8];
#pragma unroll
        for (int y = 0; y < 8; ++y) acc[y] = 0.0f;
        if (j0 == 0) {
            // the row's remaining K steps (hd <= 256: at most 8 - KPF) issued together before the
            // prefetched steps' arithmetic: one round trip, not one per step
            const uint16_t *krow = a.kc + (int64_t)((GHIP_AH_ABL & 1) ? 0 : j < a.ctx ? j : 0) * kvw + (int64_t)kvh * hd;
            constexpr int KR = 8 - KPF > 0 ? 8 - KPF : 1;
            uint4 kx[8];
#pragma unroll
            for (int r = 0; r < KR; ++r) {
                const int s = KPF + r;
                if (s < 8) kx[s < 8 ? s : 0] = *(const uint4 *)(krow + (s * 32 < hd ? s * 32 : 0) + t4 * 8);
            }
#pragma unroll
            for (int s = 0; s < KPF; ++s)
                if (s < 8) kx[s] = kpre[s];
            // this token's own row (its cache store may not be visible): only the quad of j == pos
            // swaps its operands for k16 from LDS — one divergent LDS read, not a second dot
            if (j == pos) {
#pragma unroll
                for (int s = 0; s < 8; ++s)
                    if (s * 32 < hd) kx[s] = *(const uint4 *)(k16 + s * 32 + t4 * 8);
            }
            if (GHIP_STAMPS == 4 && j0 + wave * 16 == 0) {  // the first K steps have landed
                asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
                AH_STAMP(6);
            }
            if (GHIP_AH_ABL & 2) {
#pragma unroll
                for (int s = 0; s < 8; ++s) acc[s] = __builtin_bit_cast(float, kx[s].x ^ qr[s].y);
            } else
#pragma unroll
            for (int s = 0; s < 8; ++s)
                if (s * 32 < hd && (!(GHIP_AH_ABL & 16) || s < 4)) f16_step8(acc, kx[s], qr[s]);
        } else if (j == pos) {
#pragma unroll
            for (int s = 0; s < 8; ++s)
                if (s * 32 < hd) f16_step8(acc, *(const uint4 *)(k16 + s * 32 + t4 * 8), qr[s]);
        } else {
            const int jc = j < pos ? j : 0;  // j > pos is masked below
            const uint16_t *krow = a.kc + (int64_t)jc * kvw + (int64_t)kvh * hd;
#pragma unroll
            for (int s = 0; s < 8; ++s)
                if (s * 32 < hd) f16_step8(acc, *(const uint4 *)(krow + s * 32 + t4 * 8), qr[s]);
        }
        const float kq = quad_reduce_f16(acc);
        if (GHIP_STAMPS == 4 && j0 == 0) AH_STAMP(7);  // dots folded (wave 0)
        if (t4 == 0 && j < n_kv) {
            const float w = (j > pos) ? -INFINITY : kq * 1.0f + 0.0f;
            S[j] = w;
            lmax = fmaxf(lmax, w);
            if (a.dbg_w) a.dbg_w[(int64_t)h * a.ctx + j] = w;
        }
    }
    // the row max, partial per wave (DPP) then one LDS max per wave, in the same barrier as S
    lmax = wave_max(lmax);
    if (lane == 0) {
        const uint32_t b = __builtin_bit_cast(uint32_t, lmax);
        atomicMax(mx_key, (b & 0x80000000u) ? ~b : (b | 0x80000000u));
    }
    attn_barrier();  // LDS only: the K / V prefetch stays in flight
    AH_STAMP(2);
    // ---- soft_max_ext: e = f16(exp(f16(w - max))) per position, its exact integer
    // sum, P16 = f16(e * (float)(1 / sum)).  The position's quad lane 0 (which formed S[j]) forms e;
    // the sum is exact in any order (e = k * 2^-24, k <= 2^24), reduced per wave by DPP and across
    // waves by one LDS add per wave: the bits equal a serial pass, and no wave repeats the row
    {
        const uint32_t key = *mx_key;
        const float mx = __builtin_bit_cast(float, (key & 0x80000000u) ? (key & 0x7fffffffu) : ~key);
        if (GHIP_STAMPS == 1) AH_STAMP(5);
        unsigned long long isum = 0;
        for (int j = quad; j < n_kv; j += NTH / 4) {
            if (t4 != 0) break;
            const float w = S[j];
            const float e = w != -INFINITY ? h2f(exp_f16_of(f2h(w - mx))) : 0.0f;
            isum += (unsigned long long)(uint32_t)(e * 16777216.0f);  // e*2^24 <= 2^24: exact
            P16[j] = (uint16_t)f2h(e);  // e is an f16 value: kept exactly for the second pass
        }
        isum = wave_sum_u64(isum);
        if (lane == 0 && isum) atomicAdd(e_sum, isum);
        attn_barrier();  // LDS only: the K / V prefetch stays in flight
        if (GHIP_STAMPS == 1) AH_STAMP(6);
        const double sum = (double)*e_sum * (1.0 / 16777216.0);
        const float inv = (float)(1.0 / sum);
        if (GHIP_STAMPS == 1) AH_STAMP(7);
        if (a.dbg_inv && tid == 0) a.dbg_inv[h] = inv;
        for (int j = quad; j < n_kv; j += NTH / 4) {
            if (t4 != 0) break;
            const float e = h2f(P16[j]);  // this lane's own e from the first pass (no second exp)
            P16[j] = f2h(e * inv);
            if (a.dbg_p) a.dbg_p[(int64_t)h * a.ctx + j] = P16[j];
        }
    }
    attn_barrier();
    AH_STAMP(3);
    // ---- KQV: out[d] = vec_dot_f16(n_kv, V[kvh][d][0..n_kv), P16); lane t4 runs accumulator j = t4
    for (int d = d_lo + quad; d < d_hi; d += NTH / 4) {
        float acc[8];
#pragma unroll
        for (int y = 0; y < 8; ++y) acc[y] = 0.0f;
        const uint16_t *vr = a.vc + ((int64_t)kvh * hd + d) * a.ctx;
        const float vx = d == d0 ? vx0 : ld1<SC1>(vh + d);
        // this token's V: its cache write may not be visible.  Element pos sits in step pos/32, on
        // quad lane (pos/8)%4, dword (pos%8)/2, half pos%2 — all wave-uniform but the lane test, so
        // the patch holds no per-step VGPRs (the per-step e0 form was hoisted and spilled)
        const int p_s = pos >> 5, p_t = (pos >> 3) & 3, p_w = (pos >> 1) & 3;
        const uint32_t p_sh = 16 * (pos & 1), p_msk = ~(0xFFFFu << p_sh);
        auto patch = [&](uint4 &xv, int s) {
            if (s == p_s && t4 == p_t) {
                const uint32_t hv = f2h(vx) << p_sh;
                if (p_w == 0) xv.x = (xv.x & p_msk) | hv;
                else if (p_w == 1) xv.y = (xv.y & p_msk) | hv;
                else if (p_w == 2) xv.z = (xv.z & p_msk) | hv;
                else xv.w = (xv.w & p_msk) | hv;
            }
        };
        if (n_kv <= 256) {
            // every step's V load issued before the first step's arithmetic (one round trip);
            // the prefetched steps of the first dimension come from the early loads; P16 (the same
            // for every dimension) read into registers once
            uint4 xs8[8], pr8[8];
            const bool first = d == d0;
#pragma unroll
            for (int s = 0; s < 8; ++s) {
                const int e0 = s * 32 + t4 * 8;
                if (s < VPF && first) xs8[s] = vpre[s < VPF ? s : 0];
                else xs8[s] = *(const uint4 *)(vr + (s * 32 < n_kv ? e0 : t4 * 8));
            }
#pragma unroll
            for (int s = 0; s < 8; ++s)
                pr8[s] = *(const uint4 *)(P16 + (s * 32 < n_kv ? s * 32 : 0) + t4 * 8);
            if (GHIP_STAMPS == 2 && d == d_lo + quad) {  // operands in registers (stamps build 2)
                asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
                AH_STAMP(5);
            }
#pragma unroll
            for (int s = 0; s < 8; ++s) {
                if (s * 32 >= n_kv) break;
                uint4 xv = xs8[s];
                patch(xv, s);
                if (GHIP_AH_ABL & 8) acc[s] = __builtin_bit_cast(float, xv.x ^ pr8[s].y);
                else f16_step8(acc, xv, pr8[s]);
            }
        } else
        for (int st = 0, s = 0; st < n_kv; st += 32, ++s) {
            const int e0 = st + t4 * 8;
            uint4 xv;
            if (d == d0 && s < VPF) {
                xv = vpre[0];  // statically-indexed pick from the early loads
#pragma unroll
                for (int k = 1; k < VPF; ++k)
                    if (s == k) xv = vpre[k];
            } else {
                xv = *(const uint4 *)(vr + e0);
            }
            patch(xv, s);
            f16_step8(acc, xv, *(const uint4 *)(P16 + e0));
        }
        const float o = quad_reduce_f16(acc);
        if (GHIP_STAMPS == 2 && d == d_lo + quad) AH_STAMP(6);  // chains folded
        if (t4 == 0) {
            a.out[(int64_t)h * hd + d] = o;
            if (a.out_act || a.out_q8k || a.out_gran) ((float *)smem)[d] = o;  // q16|k16 (hd floats) are dead after KQ
        }
    }
    if (a.out_gran) {  // the same image, handed on as granules inside the persistent launch
        __syncthreads();
        if (tid < dsz / 8) {
            const int b = d_lo / 32 + (tid >> 2);
            const float *o = (const float *)smem + b * 32 + (tid & 3) * 8;
            float v[8];
#pragma unroll
            for (int j = 0; j < 8; ++j) v[j] = o[j];
            image_put_quad_gran(a.out_gran, a.out_gran_da, a.gran_tag, (int64_t)h * (hd / 32) + b, tid & 3, v);
        }
    }
    if (a.out_act) {
        // this head's hd/32 blocks of the Q8_0 activation image of `out` (attn-out's PRO_IMG input;
        // the same quantize_row_q8_0 the consumer would run, DESIGN.md §Activation image)
        __syncthreads();
        if (GHIP_STAMPS == 2) AH_STAMP(7);  // the image's barrier passed
        if (tid < dsz / 8) {  // this workgroup's dims: dsz / 32 whole blocks
            const int b = d_lo / 32 + (tid >> 2);
            const float *o = (const float *)smem + b * 32 + (tid & 3) * 8;
            float v[8];
#pragma unroll
            for (int j = 0; j < 8; ++j) v[j] = o[j];
            if (SC1O) image_put_quad_sc1(a.out_act, a.out_da, (int64_t)h * (hd / 32) + b, tid & 3, v);
            else image_put_quad(a.out_act, nullptr, a.out_da, (int64_t)h * (hd / 32) + b, tid & 3, v);
        }
    }
    if (a.out_q8k) {
        // this head's 256 outputs are one Q8_K super-block of `out` (the K-quant attn-out's INIT,
        // quantize_row_q8_K as k_quant_q8_K runs it); launch_attn_decode checks hd == 256
        __syncthreads();
        if (tid < 64) {
            const float4 v = *(const float4 *)((const float *)smem + tid * 4);
            const float xv[4] = {v.x, v.y, v.z, v.w};
            q8K_store(xv, tid, a.out_q8k + (int64_t)h * 292);
        }
    }
    AH_CLK1();
    AH_STAMP(4);
}


}  // namespace
}  // namespace ghip
