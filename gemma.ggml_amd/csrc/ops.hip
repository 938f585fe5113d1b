// ops.hip — weight preparation and the small decode-step ops around the matvec (gfx950).
//
//  * k_repack / k_untile: ggml row-major Q4_0/Q8_0 blocks <-> the tiled HBM layout (common.h).
//  * k_synth_*: the synthetic-weight generator (same integer stream and reference quantizers as
//    oracle/gemma_cpu.cpp; DESIGN.md §Synthetic weights), writing straight into the tiled layout.
//  * k_attn_decode: RoPE-NEOX (src/gemma_model.cpp:698-716) + q scale (:708) + KV store (:499-518)
//    + KQ (:474) + soft_max_ext (:476) + KQV (:485) + permute/cont (:487-489) for one token, with
//    ggml's AVX/F16C vec_dot_f16 order and the fp16 exp table (A.6); split over the
//    workgroups of each kv group with one in-kernel sc1 hand-off of the scores.
//  * k_embed, k_advance (greedy token feedback), k_mul_mat_f16 (C-ABI F16 path).
#include <algorithm>

#include "attn_impl.h"
#include "device_util.h"
#include "kernels.h"

namespace ghip {
namespace {


__device__ __forceinline__ uint64_t splitmix64(uint64_t x) {
    x += 0x9E3779B97F4A7C15ull;
    uint64_t z = x;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}
__device__ __forceinline__ int32_t synth_int(uint64_t key, uint64_t idx) {
    const uint64_t h = splitmix64(key + idx);
    return (int32_t)((h & 0xFFFF) + ((h >> 16) & 0xFFFF) + ((h >> 32) & 0xFFFF) + (h >> 48)) - 131070;
}

// ggml element e (0..31) of a row-major block -> its 4-bit code / int8 value
__device__ __forceinline__ uint32_t q4_nib(const uint8_t *blk, int e) {
    const uint8_t b = blk[2 + (e & 15)];
    return e < 16 ? (b & 15u) : (uint32_t)(b >> 4);
}

// ---- ggml row-major -> tiled ------------------------------------------------------------------
template <int WT>
__global__ void k_repack(tiled_mat m, const uint8_t *src, int64_t row_bytes) {
    constexpr int BT = wfmt<WT>::BT, BB = wfmt<WT>::BLOCK_BYTES;
    const int64_t gid = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    const int64_t tile = gid >> 6;
    if (tile >= m.n_rt * m.n_bt) return;
    const int t = (int)(gid & 63), rr = t >> 3, l = t & 7;
    const int64_t rt = tile / m.n_bt, bt = tile % m.n_bt, row = rt * 8 + rr;
    uint32_t out[4];
    uint16_t sc[8];
#pragma unroll
    for (int i = 0; i < 8; ++i) sc[i] = 0;
#pragma unroll
    for (int p = 0; p < 4; ++p) {
        uint32_t w = 0;
        if (WT == T_Q4_0) {
            const int64_t b0 = bt * 8 + 2 * p;
#pragma unroll
            for (int h = 0; h < 2; ++h) {
                const int64_t b = b0 + h;
                if (row < m.rows && b < m.nb) {
                    const uint8_t *blk = src + row * row_bytes + b * BB;
#pragma unroll
                    for (int k = 0; k < 4; ++k) w |= q4_nib(blk, 4 * l + k) << (8 * k + 4 * h);
                    sc[2 * p + h] = (uint16_t)(blk[0] | (blk[1] << 8));
                }
            }
        } else {
            const int64_t b = bt * 4 + p;
            if (row < m.rows && b < m.nb) {
                const uint8_t *blk = src + row * row_bytes + b * BB;
#pragma unroll
                for (int k = 0; k < 4; ++k) w |= (uint32_t)blk[2 + 4 * l + k] << (8 * k);
                sc[p] = (uint16_t)(blk[0] | (blk[1] << 8));
            }
        }
        out[p] = w;
    }
    ((uint4 *)m.qs)[tile * 64 + t] = make_uint4(out[0], out[1], out[2], out[3]);
    if (l == 0) {
        uint16_t *dst = (uint16_t *)(m.sc + (tile * 8 + rr) * wfmt<WT>::SCALE_BYTES);
#pragma unroll
        for (int i = 0; i < BT; ++i) dst[i] = sc[i];
    }
}

// ---- tiled -> ggml row-major (for tests / the C-ABI round trip) -------------------------------
template <int WT>
__global__ void k_untile(tiled_mat m, uint8_t *dst) {
    constexpr int BT = wfmt<WT>::BT, BB = wfmt<WT>::BLOCK_BYTES;
    const int64_t gid = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (gid >= m.rows * m.nb) return;
    const int64_t row = gid / m.nb, b = gid % m.nb;
    const int64_t rt = row >> 3, rr = row & 7, bt = b / BT, bi = b % BT, tile = rt * m.n_bt + bt;
    uint8_t *blk = dst + gid * BB;
    const uint16_t d16 = ((const uint16_t *)(m.sc + (tile * 8 + rr) * wfmt<WT>::SCALE_BYTES))[bi];
    blk[0] = d16 & 0xFF;
    blk[1] = d16 >> 8;
    if (WT == T_Q4_0) {
        uint8_t codes[32];
        for (int e = 0; e < 32; ++e) {
            const int l = e >> 2, k = e & 3;
            const uint8_t byte = m.qs[tile * 1024 + (rr * 8 + l) * 16 + (bi >> 1) * 4 + k];
            codes[e] = (bi & 1) ? (byte >> 4) : (byte & 15);
        }
        for (int j = 0; j < 16; ++j) blk[2 + j] = (uint8_t)(codes[j] | (codes[j + 16] << 4));
    } else {
        for (int e = 0; e < 32; ++e) {
            const int l = e >> 2, k = e & 3;
            blk[2 + e] = m.qs[tile * 1024 + (rr * 8 + l) * 16 + bi * 4 + k];
        }
    }
}

// ---- synthetic weights, generated block-pair / block wise straight into the tiled layout -------
// q4_0 reference quantizer, restated exactly as oracle orc_quantize_row_q4_0_ref
__device__ __forceinline__ void quant_q4_0_ref(const float *x, uint32_t &d16, uint8_t codes[32]) {
    float amax = 0.0f, max = 0.0f;
    for (int j = 0; j < 32; j++) {
        const float v = x[j];
        if (amax < fabsf(v)) { amax = fabsf(v); max = v; }
    }
    const float d = max / -8.0f;
    const float id = d != 0.0f ? 1.0f / d : 0.0f;
    d16 = f2h(d);
    for (int j = 0; j < 32; ++j) {
        const float x0 = x[j] * id;
        const float t = x0 + 8.5f;
        int q = (int)(int8_t)(int)t;
        codes[j] = (uint8_t)(q < 15 ? q : 15);
    }
}
__device__ __forceinline__ void quant_q8_0_ref(const float *x, uint32_t &d16, int8_t q[32]) {
    float amax = 0.0f;
    for (int j = 0; j < 32; j++) amax = fmaxf(amax, fabsf(x[j]));
    const float d = amax / 127.0f;
    const float id = d != 0.0f ? 1.0f / d : 0.0f;
    d16 = f2h(d);
    for (int j = 0; j < 32; ++j) q[j] = (int8_t)roundf(x[j] * id);
}

template <int WT>
__global__ void k_synth_tiled(tiled_mat m, uint64_t key, float scale, int64_t row_off) {
    constexpr int BT = wfmt<WT>::BT;
    constexpr int BPU = WT == T_Q4_0 ? 2 : 1;  // blocks per work unit (Q4_0 pairs share bytes)
    const int64_t units_per_row = m.n_bt * BT / BPU;
    const int64_t gid = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (gid >= m.n_rt * 8 * units_per_row) return;
    const int64_t row = gid / units_per_row, u = gid % units_per_row;
    const int64_t rt = row >> 3, rr = row & 7;
    const int64_t b0 = u * BPU, bt = b0 / BT, bi = b0 % BT, tile = rt * m.n_bt + bt;
    uint32_t lanes[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    uint32_t d16s[2] = {0, 0};
    for (int h = 0; h < BPU; ++h) {
        const int64_t b = b0 + h;
        if (row >= m.rows || b >= m.nb) continue;
        float x[32];
        const uint64_t base = (uint64_t)(row + row_off) * (uint64_t)(m.nb * 32) + (uint64_t)b * 32;
        for (int j = 0; j < 32; ++j) x[j] = (float)synth_int(key, base + j) * scale;
        if (WT == T_Q4_0) {
            uint8_t codes[32];
            quant_q4_0_ref(x, d16s[h], codes);
            for (int l = 0; l < 8; ++l)
                for (int k = 0; k < 4; ++k) lanes[l] |= (uint32_t)codes[4 * l + k] << (8 * k + 4 * h);
        } else {
            int8_t q[32];
            quant_q8_0_ref(x, d16s[h], q);
            for (int l = 0; l < 8; ++l)
                for (int k = 0; k < 4; ++k) lanes[l] |= (uint32_t)(uint8_t)q[4 * l + k] << (8 * k);
        }
    }
    const int p = WT == T_Q4_0 ? (int)(bi >> 1) : (int)bi;
    uint32_t *qs = (uint32_t *)(m.qs + tile * 1024);
    for (int l = 0; l < 8; ++l) qs[(rr * 8 + l) * 4 + p] = lanes[l];
    uint16_t *sc = (uint16_t *)(m.sc + (tile * 8 + rr) * wfmt<WT>::SCALE_BYTES);
    for (int h = 0; h < BPU; ++h) sc[bi + h] = (uint16_t)d16s[h];
}

__global__ void k_synth_norm(float *dst, int64_t n, uint64_t key, float scale) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) dst[i] = 1.0f + (float)synth_int(key, (uint64_t)i) * scale;
}

// ---- embedding row lookup (get_rows + scale; src/gemma_model.cpp:677-679) ---------------------
template <int WT>
__global__ void k_embed(const uint8_t *qs, const uint8_t *sc, int64_t n_bt, const int *token, float scale, float *out,
                        int64_t E) {
    constexpr int BT = wfmt<WT>::BT;
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= E) return;
    const int64_t row = token[blockIdx.y];
    const int64_t b = i >> 5;
    const int e = (int)(i & 31);
    const int64_t rt = row >> 3, rr = row & 7, bt = b / BT, bi = b % BT, tile = rt * n_bt + bt;
    const int l = e >> 2, k = e & 3;
    const uint16_t d16 = ((const uint16_t *)(sc + (tile * 8 + rr) * wfmt<WT>::SCALE_BYTES))[bi];
    const uint8_t *t = qs + tile * 1024 + (rr * 8 + l) * 16;
    int q;
    if (WT == T_Q4_0) {
        const uint8_t byte = t[(bi >> 1) * 4 + k];
        q = (int)((bi & 1) ? (byte >> 4) : (byte & 15)) - 8;
    } else {
        q = (int)(int8_t)t[bi * 4 + k];
    }
    out[(int64_t)blockIdx.y * E + i] = ((float)q * pin(h2f(d16))) * scale;
}

#define ATT_STAMP(i)                                                                                        \
    do {                                                                                                    \
        if (GHIP_STAMPS && a.dbg_t && tid == 0) a.dbg_t[(int64_t)(kvh * a.nwg + wg) * 8 + (i)] = __builtin_amdgcn_s_memrealtime(); \
    } while (0)

// One token's attention for the G = H/Hkv query heads of kv head kvh = blockIdx.x / nwg, split over
// the group's nwg workgroups (wg = blockIdx.x % nwg) in two phases joined by an in-kernel hand-off:
//  A) KQ: position blocks of PS positions, block b -> workgroup b % nwg.  Quad q scores (position
//     q / G, head q % G) from the block's K rows staged once in LDS.  Scores (masked j > pos ->
//     -inf) go to sbuf[kvh][j][h].
//  B) softmax + KQV: every workgroup re-derives each head's exact softmax from all scores (the
//     reduction is exact, so redundancy is free of order effects), then workgroup wg < nb computes
//     out[h][d] for d in [wg*DS, +DS): quad q owns (dim q / G, head q % G).
// The per-position / per-output arithmetic is exactly that of a single-workgroup form: RoPE, f16
// conversions, vec_dot_f16 order, exp table, integer-exact sum, (float)(1/sum).
__global__ void __launch_bounds__(ATT_THREADS) k_attn_decode(attn_args a) {
    extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
    const int hd = a.hd, half = hd / 2, tid = threadIdx.x, t4 = tid & 3, quad = tid >> 2;
    const int lane = tid & 63, wave = tid >> 6;
    // a kv group's nwg workgroups share blockIdx % 8 (one XCD under round-robin placement: the
    // hand-off stays in one L2 — speed only, the protocol is placement-independent)
    const int G = a.H / a.Hkv, nwg = a.nwg;
    const int slot = blockIdx.x >> 3, kvh = (slot / nwg) * 8 + (int)(blockIdx.x & 7), wg = slot % nwg;
    if (kvh >= a.Hkv) return;
    const attn_split sp = attn_split_of(G, hd);
    const int PS = sp.ps, DS = sp.ds;
    const int nb = (hd + DS - 1) / DS;  // workgroups with KQV work
    const int kvw = a.Hkv * hd;
    ATT_STAMP(0);
    // ---- early loads (issue order = wait order): RoPE inputs, then the K and V rows to stage
    const float *qg = a.qkv + (int64_t)kvh * G * hd;
    const float *kh = a.qkv + (int64_t)a.H * hd + (int64_t)kvh * hd;
    const float *vh = a.qkv + (int64_t)a.H * hd + kvw + (int64_t)kvh * hd;
    const float *cs = a.rope_cur, *sn = a.rope_cur + half;  // row of *pos (k_advance keeps it)
    // q: thread t takes 4 consecutive pairs (h, e..e+3) of the G*half pairs (npair % 4 == 0)
    const int npair = G * half, nq4 = npair / 4;
    // (only waves holding pairs issue these loads: wave-uniform branches)
    float4 qa[2] = {}, qb[2] = {}, ca[2] = {}, sa[2] = {};
#pragma unroll
    for (int r = 0; r < 2; ++r) {
        const int i4 = tid + r * ATT_THREADS;
        if (i4 - lane < nq4) {
            const int i = (i4 < nq4 ? i4 : 0) * 4;
            const int h = i / half, e = i % half;
            qa[r] = *(const float4 *)(qg + h * hd + e);
            qb[r] = *(const float4 *)(qg + h * hd + e + half);
            ca[r] = *(const float4 *)(cs + e);
            sa[r] = *(const float4 *)(sn + e);
        }
    }
    const int kq4 = half / 4;  // k: 4 pairs per thread for tid < half/4
    const int ik = (tid < kq4 ? tid : 0) * 4;
    float4 ka{}, kb{}, kc4{}, ks4{};
    if (wave * 64 < kq4) {
        ka = *(const float4 *)(kh + ik); kb = *(const float4 *)(kh + ik + half);
        kc4 = *(const float4 *)(cs + ik); ks4 = *(const float4 *)(sn + ik);
    }
    // phase A, first position block of this workgroup: its PS K rows, one coalesced uint4 each
    const int kcw = hd / 8;  // uint4 per K row
    uint4 kst[ATT_STG];
#pragma unroll
    for (int r = 0; r < ATT_STG; ++r) {
        const int idx = tid + r * ATT_THREADS;
        const int row = idx / kcw, c = idx % kcw;
        int j = wg * PS + row;
        j = (idx < PS * kcw && j < a.ctx) ? j : 0;  // rows >= pos are masked; no dependency on pos
        kst[r] = *(const uint4 *)(a.kc + (int64_t)j * kvw + (int64_t)kvh * hd + c * 8);
    }
    // phase B: V rows d of [wg*DS, +DS), positions [0, ATT_VW), one coalesced uint4 each
    constexpr int vcw = ATT_VW / 8;
    uint4 vst[ATT_STG];
    float vsx[ATT_STG];
#pragma unroll
    for (int r = 0; r < ATT_STG; ++r) {
        const int idx = tid + r * ATT_THREADS;
        const int dd = idx / vcw, c = idx % vcw;
        int d = wg * DS + dd;
        d = (idx < DS * vcw && d < hd && wg < nb) ? d : 0;
        vst[r] = *(const uint4 *)(a.vc + ((int64_t)kvh * hd + d) * a.ctx + (c * 8 < a.ctx ? c * 8 : 0));
        vsx[r] = vh[d];  // this token's v of the row (patched into the staged copy)
    }
    const int pa = quad / G < PS ? quad / G : 0, ha = quad % G;
    const bool has_a = quad / G < PS;
    const int db = wg * DS + quad / G, hb = quad % G;
    const bool has_b = wg < nb && quad / G < DS && db < hd;
    const uint16_t *vrow = a.vc + ((int64_t)kvh * hd + (has_b ? db : 0)) * a.ctx;
    const float vx = has_b ? vh[db] : 0.0f;
    ATT_STAMP(6);
    // pos is published with the RoPE row (k_advance / begin): no dependent load
    const int pos = __builtin_amdgcn_readfirstlane(((const int *)a.rope_cur)[hd]);
    const int n_total = pos + 1;
    int n_kv = 32 * (n_total / 32 + 1);  // src/gemma_model.cpp:429
    if (n_kv > a.ctx) n_kv = a.ctx;
    ATT_STAMP(7);

    // LDS: q16 [G][hd], k16 [hd], Ks [PS][hd], Vs [DS][ATT_VW], P16 [G][ctx]
    uint16_t *q16 = (uint16_t *)smem;
    uint16_t *k16 = q16 + (size_t)G * hd;
    uint16_t *Ks = k16 + hd;
    uint16_t *Vs = Ks + (size_t)PS * hd;
    uint16_t *P16 = Vs + (size_t)DS * ATT_VW;

    // RoPE NEOX on q (then * q_scale) and on k; f32 -> f16 (ggml_cpy / MUL_MAT INIT conversions)
    auto rope4 = [&](float4 x0v, float4 x1v, float4 cv, float4 sv, float scale, bool scaled, uint16_t *lo,
                     uint16_t *hi) {
        const float x0s[4] = {x0v.x, x0v.y, x0v.z, x0v.w}, x1s[4] = {x1v.x, x1v.y, x1v.z, x1v.w};
        const float cs4[4] = {cv.x, cv.y, cv.z, cv.w}, sn4[4] = {sv.x, sv.y, sv.z, sv.w};
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
#pragma unroll
    for (int r = 0; r < 2; ++r) {
        const int i4 = tid + r * ATT_THREADS;
        if (i4 < nq4) {
            const int i = i4 * 4, h = i / half, e = i % half;
            rope4(qa[r], qb[r], ca[r], sa[r], a.q_scale, true, q16 + h * hd + e, q16 + h * hd + e + half);
        }
    }
    for (int i4 = tid + 2 * ATT_THREADS; i4 < nq4; i4 += ATT_THREADS) {  // G * hd > 4096 (rare)
        const int i = i4 * 4, h = i / half, e = i % half;
        rope4(*(const float4 *)(qg + h * hd + e), *(const float4 *)(qg + h * hd + e + half), *(const float4 *)(cs + e),
              *(const float4 *)(sn + e), a.q_scale, true, q16 + h * hd + e, q16 + h * hd + e + half);
    }
    if (tid < kq4) rope4(ka, kb, kc4, ks4, 1.0f, false, k16 + ik, k16 + ik + half);
    // stage K and V rows (V patched at `pos`: this token's cache write is not visible in-launch)
#pragma unroll
    for (int r = 0; r < ATT_STG; ++r) {
        const int idx = tid + r * ATT_THREADS;
        if (idx < PS * kcw) *(uint4 *)(Ks + (size_t)idx * 8) = kst[r];
        if (idx < DS * vcw) {
            const int c = idx % vcw;
            uint4 v = vst[r];
            if (pos >= c * 8 && pos < c * 8 + 8) {
                const uint32_t h = f2h(vsx[r]), sh = 16 * ((pos - c * 8) & 1);
                const uint32_t m = ~(0xFFFFu << sh);
                switch ((pos - c * 8) >> 1) {
                    case 0: v.x = (v.x & m) | (h << sh); break;
                    case 1: v.y = (v.y & m) | (h << sh); break;
                    case 2: v.z = (v.z & m) | (h << sh); break;
                    default: v.w = (v.w & m) | (h << sh); break;
                }
            }
            *(uint4 *)(Vs + (size_t)idx * 8) = v;
        }
    }
    __syncthreads();
    ATT_STAMP(1);
    // this token's cache entries (src/gemma_model.cpp:506-517): K row by workgroup 0, V column
    // `pos` by the KQV workgroup owning each dimension
    if (wg == 0)
        for (int i = tid; i < hd; i += ATT_THREADS) a.kc[(int64_t)pos * kvw + (int64_t)kvh * hd + i] = k16[i];
    if (has_b && hb == 0 && t4 == 0) a.vc[((int64_t)kvh * hd + db) * a.ctx + pos] = f2h(vx);

    // ---- phase A: KQ (vec_dot_f16 over hd per kv position) + mask (j > pos -> -inf), scale 1.0
    float *sk_out = a.sbuf + (int64_t)kvh * a.ctx * G;  // [ctx][G]
    for (int blk = wg, pass = 0; blk * PS < n_kv; blk += nwg, ++pass) {
        const int j = blk * PS + pa;
        float acc[8];
#pragma unroll
        for (int y = 0; y < 8; ++y) acc[y] = 0.0f;
        const uint16_t *qh16 = q16 + (size_t)ha * hd + t4 * 8;
        if (pass == 0) {  // staged rows (LDS); row `pos` from this token's k16
            const uint16_t *krow = ((j == pos) ? k16 : Ks + (size_t)pa * hd) + t4 * 8;
            for (int s = 0; s * 32 < hd; ++s)
                f16_step8(acc, *(const uint4 *)(krow + s * 32), *(const uint4 *)(qh16 + s * 32));
        } else {
            const int jc = j < pos ? j : pos;
            if (jc == pos) {
                for (int s = 0; s * 32 < hd; ++s)
                    f16_step8(acc, *(const uint4 *)(k16 + s * 32 + t4 * 8), *(const uint4 *)(qh16 + s * 32));
            } else {
                const uint16_t *krow = a.kc + (int64_t)jc * kvw + (int64_t)kvh * hd + t4 * 8;
                for (int s = 0; s * 32 < hd; ++s)
                    f16_step8(acc, *(const uint4 *)(krow + s * 32), *(const uint4 *)(qh16 + s * 32));
            }
        }
        const float kq = quad_reduce_f16(acc);
        if (t4 == 0 && has_a && j < n_kv) {
            const float w = (j > pos) ? -INFINITY : kq * 1.0f + 0.0f;
            st_sc1(sk_out + (int64_t)j * G + ha, w);
            if (a.dbg_w) a.dbg_w[(int64_t)(kvh * G + ha) * a.ctx + j] = w;
        }
    }
    // publish: every storing wave drains its stores, then one lane arrives
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    ATT_STAMP(2);
    int *cnt = a.sync + kvh * 2;
    if (tid == 0) __hip_atomic_fetch_add(cnt, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (wg >= nb) return;  // no KQV work for this workgroup

    // ---- hand-off: wait for all nwg workgroups of this kv head (bounded spin)
    if (tid == 0) {
        int spins = 0;
        while (ld_sc1_i(cnt) < nwg) {
            __builtin_amdgcn_s_sleep(1);
            if (++spins > (1 << 26)) {  // never on a healthy device: flag and fall through
                if (a.err) *a.err = 1;
                break;
            }
        }
    }
    __syncthreads();
    ATT_STAMP(3);

    // ---- soft_max_ext per head h: one wave reduces a head's scores (DPP, exact)
    for (int h = wave; h < G; h += ATT_THREADS / 64) {
        float mx = -INFINITY;
        float sv[4];
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            const int j = lane + 64 * k;
            sv[k] = j < n_kv ? ld_sc1(sk_out + (int64_t)j * G + h) : -INFINITY;
            mx = fmaxf(mx, sv[k]);
        }
        for (int j = lane + 256; j < n_kv; j += 64) mx = fmaxf(mx, ld_sc1(sk_out + (int64_t)j * G + h));
        mx = wave_max(mx);
        // e values are fp16 in [0,1]: exact multiples of 2^-24, so an integer sum is the exact sum
        // (ggml's double accumulation of them is exact too).  e is parked as f16 in P16.
        unsigned long long isum = 0;
        uint16_t *prow = P16 + (size_t)h * a.ctx;
        for (int j = lane, k = 0; j < n_kv; j += 64, ++k) {
            const float w = k < 4 ? (k == 0 ? sv[0] : k == 1 ? sv[1] : k == 2 ? sv[2] : sv[3])
                                  : ld_sc1(sk_out + (int64_t)j * G + h);
            uint16_t e16 = 0;
            if (w != -INFINITY) e16 = (uint16_t)exp_f16_of(f2h(w - mx));
            prow[j] = e16;
            isum += (unsigned long long)(uint32_t)(h2f(e16) * 16777216.0f);
        }
        const unsigned long long tot = wave_sum_u64(isum);
        const double sum = (double)tot * (1.0 / 16777216.0);
        const float inv = (float)(1.0 / sum);
        if (a.dbg_inv && lane == 0 && wg == 0) a.dbg_inv[kvh * G + h] = inv;
        for (int j = lane; j < n_kv; j += 64) {
            const uint16_t p = f2h(h2f(prow[j]) * inv);
            prow[j] = p;
            if (a.dbg_p && wg == 0) a.dbg_p[(int64_t)(kvh * G + h) * a.ctx + j] = p;
        }
    }
    __syncthreads();
    ATT_STAMP(4);
    // hand-off bookkeeping: the last KQV workgroup to get here resets the counters for the next
    // launch (every other workgroup of this kv head has already passed its poll)
    if (tid == 0) {
        const int done = __hip_atomic_fetch_add(cnt + 1, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        if (done == nb - 1) {
            __hip_atomic_store(cnt, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            __hip_atomic_store(cnt + 1, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
    }

    // ---- KQV: out[h][d] = vec_dot_f16(n_kv, V[kvh][d][0..n_kv), P16[h]); lane t4 = accumulator j
    if (has_b) {
        float acc[8];
#pragma unroll
        for (int y = 0; y < 8; ++y) acc[y] = 0.0f;
        const uint16_t *prow = P16 + (size_t)hb * a.ctx;
        const uint16_t *vs = Vs + (size_t)(db - wg * DS) * ATT_VW;
        for (int st = 0; st < n_kv; st += 32) {
            const int e0 = st + t4 * 8;
            uint4 xv;
            if (st < ATT_VW) {  // staged (and already patched at `pos`)
                xv = *(const uint4 *)(vs + e0);
            } else {
                xv = *(const uint4 *)(vrow + e0);
                if (pos >= e0 && pos < e0 + 8) {  // this token's V: its cache write may not be visible
                    __attribute__((aligned(16))) uint16_t tmp[8];
                    *(uint4 *)tmp = xv;
                    tmp[pos - e0] = f2h(vx);
                    xv = *(const uint4 *)tmp;
                }
            }
            f16_step8(acc, xv, *(const uint4 *)(prow + e0));
        }
        const float o = quad_reduce_f16(acc);
        if (t4 == 0) {
            a.out[(int64_t)(kvh * G + hb) * hd + db] = o;
            if (a.out_act) ((float *)smem)[hb * DS + (db - wg * DS)] = o;  // q16 is dead after KQ
        }
    }
    if (a.out_act) {
        // this slice's Q8_0 blocks of each head's output (DS == 32, aligned: one block per head)
        __syncthreads();
        if (tid < G * 4) {
            const int h = tid >> 2, q = tid & 3;
            const float *o = (const float *)smem + h * DS + q * 8;
            float v[8];
#pragma unroll
            for (int j = 0; j < 8; ++j) v[j] = o[j];
            image_put_quad(a.out_act, nullptr, a.out_da, (int64_t)(kvh * G + h) * (hd / 32) + wg, q, v);
        }
    }
    ATT_STAMP(5);
}

// the per-head form (k_attn_head) lives in attn_impl.h: the fused layer-front kernel runs it too
__global__ void __launch_bounds__(AH_THREADS) k_attn_head(attn_args a) {
    extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
    const int S = a.dsplit, G = a.H / a.Hkv;
    // one inlined copy of the body (a second call site doubled the kernel's code: measured slower,
    // DESIGN.md §10)
    const int hs = blockIdx.x >> 3, h = hs / S, sp = hs % S;
    if ((int)(blockIdx.x & 7) != ((h / G) & 7)) return;  // the G*S workgroups of a kv head share an XCD (speed only)
    attn_head_dev<AH_THREADS, false, AH_KPF, AH_VPF, false>(a, h, smem, nullptr, sp);
}

// ---- exact causal attention for T prompt rows (the reference's prefill graph) -----------------
// Row i of the prefill KQ / soft_max_ext / KQV (src/gemma_model.cpp:467-489 with T tokens) is the
// decode computation at position i: positions j > i are masked to -inf (e = 0), and the KQV terms
// past the row's own padded n_kv multiply exact zeros, so each row runs k_attn_head's arithmetic
// (vec_dot_f16 lane order via v_fma_mix, fp16 exp, integer-exact sum, (float)(1/sum)) over
// n_kv(i) = 32*((i+1)/32+1) positions.  One 1024-thread workgroup per (row, kv head) serves the
// G <= 8 query heads of that kv head: quad q -> KQ position q (+ 256 per pass) and KQV dim q, each
// for all G heads, so every K / V row is loaded once per row and 8 steps share one round trip
// (the head-major mapping of round 1 paid a round trip per 256/G positions).  Rows are issued
// longest first.  q16 / caches come from k_rope_kv_prefill (same RoPE/f16 arithmetic).
#ifndef GHIP_AR_THREADS
#define GHIP_AR_THREADS 512
#endif
// 512 threads and P16 written over S in place (LDS G*n_kv*4 + G*hd*2 B): two row workgroups per CU,
// so one's loads overlap the other's fma chains (1024 threads, separate P16: one per CU)
constexpr int AR_THREADS = GHIP_AR_THREADS;
constexpr bool AR_ALIAS = AR_THREADS <= 512;

__global__ void __launch_bounds__(AR_THREADS) k_attn_rows(attnp_args a) {
    extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
    const int tid = threadIdx.x, t4 = tid & 3, quad = tid >> 2, lane = tid & 63, wave = tid >> 6;
    const int G = a.H / a.Hkv, hd = a.hd, kvw = a.Hkv * hd, nkp = a.n_kv;
    const int kvh = blockIdx.x % a.Hkv, i = a.T - 1 - (int)(blockIdx.x / a.Hkv);
    float *S = (float *)smem;                      // [G][nkp]
    // P16 row gg: over S row gg (in place: the softmax's last pass reads S[j] before any lane of the
    // wave writes P16[j], which lies inside S[j/2], already read) or after S
    uint16_t *P16 = AR_ALIAS ? (uint16_t *)S : (uint16_t *)(S + (size_t)G * nkp);
    const int p16s = AR_ALIAS ? 2 * nkp : nkp;     // P16 row stride (halfs)
    uint16_t *Q16 = (uint16_t *)(S + (size_t)G * nkp) + (AR_ALIAS ? 0 : (size_t)G * nkp);  // [G][hd]
    int n_kv = 32 * ((i + 1) / 32 + 1);
    if (n_kv > nkp) n_kv = nkp;
    for (int k = tid; k < G * hd / 8; k += AR_THREADS) {
        const int gg = k / (hd / 8), o = (k % (hd / 8)) * 8;
        *(uint4 *)(Q16 + gg * hd + o) = *(const uint4 *)(a.q16 + ((int64_t)i * a.H + kvh * G + gg) * hd + o);
    }
    __syncthreads();
    // KQ + mask (scale 1.0, mask 0 / -inf): quad -> one position per pass (256 per pass) for all G
    // heads, so each K row is loaded once per pass (8 x 16 B per lane, one round trip) and every
    // (head, position) dot is the same 32-accumulator vec_dot_f16 chain against that head's q
    for (int j0 = 0; j0 < n_kv; j0 += AR_THREADS / 4) {
        const int j = j0 + quad;
        const int jl = j <= i ? j : i;  // masked positions load a valid row (result unused)
        const uint16_t *krow = a.kc + (int64_t)jl * kvw + (int64_t)kvh * hd + t4 * 8;
        uint4 kv[8];
#pragma unroll
        for (int s = 0; s < 8; ++s) kv[s] = *(const uint4 *)(krow + (s * 32 < hd ? s * 32 : 0));
#pragma unroll
        for (int gg = 0; gg < 8; ++gg) {
            if (gg >= G) break;
            float acc[8];
#pragma unroll
            for (int y = 0; y < 8; ++y) acc[y] = 0.0f;
#pragma unroll
            for (int s = 0; s < 8; ++s)
                if (s * 32 < hd) f16_step8(acc, kv[s], *(const uint4 *)(Q16 + gg * hd + s * 32 + t4 * 8));
            const float kq = quad_reduce_f16(acc);
            if (t4 == 0 && j < n_kv) S[gg * nkp + j] = (j > i) ? -INFINITY : kq * 1.0f + 0.0f;
        }
    }
    __syncthreads();
    // soft_max_ext per head row: wave w takes heads w, w+16, ...
    for (int gg = wave; gg < G; gg += AR_THREADS / 64) {
        const float *Sr = S + gg * nkp;
        float mx = -INFINITY;
        for (int j = lane; j < n_kv; j += 64) mx = fmaxf(mx, Sr[j]);
        mx = wave_max(mx);
        unsigned long long isum = 0;
        for (int j = lane; j < n_kv; j += 64) {
            const float w = Sr[j];
            const float e = w != -INFINITY ? h2f(exp_f16_of(f2h(w - mx))) : 0.0f;
            isum += (unsigned long long)(uint32_t)(e * 16777216.0f);  // e*2^24 <= 2^24: exact in u32 (one v_cvt_u32_f32)
        }
        const unsigned long long tot = wave_sum_u64(isum);
        const double sum = (double)tot * (1.0 / 16777216.0);
        const float inv = (float)(1.0 / sum);
        for (int j = lane; j < n_kv; j += 64) {
            const float w = Sr[j];
            const float e = w != -INFINITY ? h2f(exp_f16_of(f2h(w - mx))) : 0.0f;
            P16[gg * p16s + j] = (uint16_t)f2h(e * inv);
        }
    }
    __syncthreads();
    // KQV: out[i][h][d] = vec_dot_f16(n_kv, V[kvh][d][0..n_kv), P16[h]): quad -> output dim d for
    // all G heads, so each V row is loaded once (8 steps per round trip) and multiplied against each
    // head's P16 row; each (head, dim) keeps vec_dot_f16's chain in step order
    for (int d = quad; d < hd; d += AR_THREADS / 4) {
        float acc[8][8];
#pragma unroll
        for (int gg = 0; gg < 8; ++gg)
#pragma unroll
            for (int y = 0; y < 8; ++y) acc[gg][y] = 0.0f;
        const uint16_t *vr = a.vc + ((int64_t)kvh * hd + d) * a.ctx + t4 * 8;
        for (int st0 = 0; st0 < n_kv; st0 += 256) {
            uint4 vv[8];
#pragma unroll
            for (int u = 0; u < 8; ++u) vv[u] = *(const uint4 *)(vr + (st0 + 32 * u < n_kv ? st0 + 32 * u : 0));
#pragma unroll
            for (int u = 0; u < 8; ++u) {
                if (st0 + 32 * u >= n_kv) break;
#pragma unroll
                for (int gg = 0; gg < 8; ++gg) {
                    if (gg >= G) break;
                    f16_step8(acc[gg], vv[u], *(const uint4 *)(P16 + gg * p16s + st0 + 32 * u + t4 * 8));
                }
            }
        }
#pragma unroll
        for (int gg = 0; gg < 8; ++gg) {
            if (gg >= G) break;
            const float o = quad_reduce_f16(acc[gg]);
            if (t4 == 0) a.out[(int64_t)i * a.ldo + (int64_t)(kvh * G + gg) * hd + d] = o;
        }
    }
}

// streaming read for the measured HBM roofline: 8 x 16 B in flight per lane, grid-stride
typedef unsigned v4u_t __attribute__((ext_vector_type(4)));
__global__ void __launch_bounds__(256) k_stream_read(const uint4 *src_, uint64_t n16, unsigned *sink) {
    const v4u_t *src = (const v4u_t *)src_;
    const uint64_t nth = (uint64_t)gridDim.x * blockDim.x;
    uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    uint32_t acc = 0;
    for (; i + 7 * nth < n16; i += 8 * nth) {
        v4u_t v[8];
#pragma unroll
        for (int u = 0; u < 8; ++u) v[u] = __builtin_nontemporal_load(src + i + u * nth);
#pragma unroll
        for (int u = 0; u < 8; ++u) acc ^= v[u].x ^ v[u].y ^ v[u].z ^ v[u].w;
    }
    for (; i < n16; i += nth) {
        const v4u_t v = src[i];
        acc ^= v.x ^ v.y ^ v.z ^ v.w;
    }
    if (acc == 0x9E3779B9u) *sink = acc;  // never true for the memset pattern: keeps the loads
}

// streaming read by LDS-DMA (global_load_lds_dwordx4 nt: no VGPR destination, so each wave keeps
// 16 KiB in flight): MI355X_MICROARCH's ldsdma-fill row measures 6.5-6.8 TB/s chip-wide this way, the
// better yardstick for "measured HBM read".  Each wave instruction moves one contiguous 1 KiB chunk
// into the wave's ring slot (never read: only the HBM -> CU stream is timed).
constexpr int SL_SLOTS = 16;
__global__ void __launch_bounds__(256) k_stream_lds(const uint4 *src, uint64_t n16) {
    __shared__ __attribute__((aligned(16))) uint8_t ring[4 * SL_SLOTS * 1024];
    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const uint64_t nw = (uint64_t)gridDim.x * 4, nchunks = n16 / 64;
    int slot = 0;
    for (uint64_t c = (uint64_t)blockIdx.x * 4 + wave; c < nchunks; c += nw) {
        const uint32_t lds = __builtin_amdgcn_readfirstlane((uint32_t)(uintptr_t)(ring + (wave * SL_SLOTS + slot) * 1024));
        const uint4 *g = src + c * 64 + lane;
        unsigned keep;
        asm volatile(
            "s_mov_b32 %0, m0\n\t"
            "s_mov_b32 m0, %2\n\t"
            "s_nop 0\n\t"
            "global_load_lds_dwordx4 %1, off nt\n\t"
            "s_mov_b32 m0, %0"
            : "=&s"(keep)
            : "v"(g), "s"(lds)
            : "memory");
        slot = (slot + 1) & (SL_SLOTS - 1);
        asm volatile("s_waitcnt vmcnt(15)" ::: "memory");  // the slot about to be reused has landed
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
}

__global__ void k_exp_f16_all(uint16_t *out) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i < 65536) out[i] = (uint16_t)exp_f16_of((uint32_t)i);
}

// TP: this rank's per-workgroup keys -> one key whose index is global (local + row_base); the order
// of keys is preserved (larger value first, then smaller global index), so the merged argmax is
// the single-GPU one
__global__ void __launch_bounds__(256) k_reduce_keys(const unsigned long long *keys, int n, int64_t row_base,
                                                     unsigned long long *out) {
    __shared__ unsigned long long red[4];
    unsigned long long best = 0;
    for (int i = threadIdx.x; i < n; i += 256) best = keys[i] > best ? keys[i] : best;
#pragma unroll
    for (int off = 32; off >= 1; off >>= 1) {
        const unsigned long long o = __shfl_xor(best, off);
        best = o > best ? o : best;
    }
    if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = best;
    __syncthreads();
    if (threadIdx.x != 0) return;
    for (int w = 1; w < 4; ++w) best = red[w] > best ? red[w] : best;
    const uint32_t local = 0xFFFFFFFFu - (uint32_t)(best & 0xFFFFFFFFull);
    *out = (best & 0xFFFFFFFF00000000ull) | (unsigned long long)(0xFFFFFFFFu - (uint32_t)(local + row_base));
}

__global__ void __launch_bounds__(256) k_advance(const unsigned long long *keys, int n_parts, int *token, int *pos,
                                                 int *hist, int hist_cap, const int *n_fixed, rope_row r) {
    __shared__ unsigned long long red[4];
    // the next position does not depend on the argmax: every thread reads *pos first (one line), so
    // the RoPE row copy of position p overlaps the key loads instead of waiting for the reduction and
    // a second dependent load of *pos (three serial memory round trips -> one; thread 0 writes *pos
    // only after the barrier below, which every read precedes)
    const int p = *pos + 1;
    const int fixed = hist ? *n_fixed : 0;
    if (r.cur && p < r.ctx) {  // the RoPE row of the next position, at a fixed address (attention loads it without *pos)
        for (int i = threadIdx.x; i < r.half; i += 256) {
            r.cur[i] = r.cos[(int64_t)p * r.half + i];
            r.cur[r.half + i] = r.sin[(int64_t)p * r.half + i];
        }
        if (threadIdx.x == 0) ((int *)r.cur)[2 * r.half] = p;
    }
    unsigned long long best = 0;
    for (int i = threadIdx.x; i < n_parts; i += 256) best = keys[i] > best ? keys[i] : best;
#pragma unroll
    for (int off = 32; off >= 1; off >>= 1) {
        const unsigned long long o = __shfl_xor(best, off);
        best = o > best ? o : best;
    }
    if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = best;
    __syncthreads();
    if (threadIdx.x == 0) {
        for (int w = 1; w < 4; ++w) best = red[w] > best ? red[w] : best;
        // strict '>' argmax, first max wins (src/gemma_model.cpp:538-543): the key's low word is ~index
        const int idx = (int)(0xFFFFFFFFu - (uint32_t)(best & 0xFFFFFFFFull));
        *token = idx;
        if (hist && p < hist_cap && p >= fixed) hist[p] = idx;  // never overwrite the prompt
        *pos = p;
        if (r.epoch) ++*r.epoch;  // a new token: fresh granule tags for the persistent launch
    }
}

// host-fed position (the ggml executor's engine path): hist[p] = token, *pos = p, *n_fixed past the
// history (k_advance leaves hist alone), the RoPE row of p — kernel arguments instead of four
// pageable host copies
__global__ void __launch_bounds__(256) k_set_position(int token, int p, int *pos, int *hist, int *n_fixed, int fixed,
                                                      rope_row r) {
    if (threadIdx.x == 0) {
        hist[p] = token;
        *pos = p;
        *n_fixed = fixed;
        ((int *)r.cur)[2 * r.half] = p;
        if (r.epoch) ++*r.epoch;
    }
    for (int i = threadIdx.x; i < r.half; i += 256) {
        r.cur[i] = r.cos[(int64_t)p * r.half + i];
        r.cur[r.half + i] = r.sin[(int64_t)p * r.half + i];
    }
}

// C-ABI F16 mul_mat (KQ/KQV shapes): one thread per (row, col), vec_dot_f16 order
__global__ void k_mul_mat_f16(const uint16_t *src0, int64_t nb01e, int64_t ne01, const uint16_t *src1, int64_t rse,
                              int64_t ncols, int64_t K, float *dst) {
    const int64_t gid = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (gid >= ne01 * ncols) return;
    const int64_t c = gid / ne01, r = gid % ne01;
    const uint16_t *x = src0 + r * nb01e, *y = src1 + c * rse;
    float acc[4][8];
    for (int i = 0; i < 4; ++i)
        for (int j = 0; j < 8; ++j) acc[i][j] = 0.0f;
    const int64_t np = K & ~(int64_t)31;
    for (int64_t i = 0; i < np; i += 32)
        for (int j = 0; j < 4; ++j)
            for (int l = 0; l < 8; ++l) {
                const int64_t e = i + j * 8 + l;
                acc[j][l] = __builtin_fmaf(h2f(x[e]), h2f(y[e]), acc[j][l]);
            }
    double sumf = reduce_f16_acc(acc);
    for (int64_t i = np; i < K; ++i) sumf += (double)(h2f(x[i]) * h2f(y[i]));
    dst[c * ne01 + r] = (float)sumf;
}

}  // namespace

int launch_repack(const tiled_mat &m, const uint8_t *src, int64_t row_bytes, hipStream_t s) {
    const int64_t n = m.n_rt * m.n_bt * 64;
    const int grid = (int)((n + 255) / 256);
    if (m.type == T_Q4_0) hipLaunchKernelGGL(k_repack<T_Q4_0>, dim3(grid), dim3(256), 0, s, m, src, row_bytes);
    else hipLaunchKernelGGL(k_repack<T_Q8_0>, dim3(grid), dim3(256), 0, s, m, src, row_bytes);
    GHIP_CHECK(hipGetLastError());
    return 0;
}

int launch_untile(const tiled_mat &m, uint8_t *dst, hipStream_t s) {
    const int64_t n = m.rows * m.nb;
    const int grid = (int)((n + 255) / 256);
    if (m.type == T_Q4_0) hipLaunchKernelGGL(k_untile<T_Q4_0>, dim3(grid), dim3(256), 0, s, m, dst);
    else hipLaunchKernelGGL(k_untile<T_Q8_0>, dim3(grid), dim3(256), 0, s, m, dst);
    GHIP_CHECK(hipGetLastError());
    return 0;
}

int launch_synth_tiled(const tiled_mat &m, uint64_t key, float scale, int64_t row_off, hipStream_t s) {
    const int bpu = m.type == T_Q4_0 ? 2 : 1;
    const int bt = m.type == T_Q4_0 ? 8 : 4;
    const int64_t n = m.n_rt * 8 * (m.n_bt * bt / bpu);
    const int grid = (int)((n + 255) / 256);
    if (m.type == T_Q4_0) hipLaunchKernelGGL(k_synth_tiled<T_Q4_0>, dim3(grid), dim3(256), 0, s, m, key, scale, row_off);
    else hipLaunchKernelGGL(k_synth_tiled<T_Q8_0>, dim3(grid), dim3(256), 0, s, m, key, scale, row_off);
    GHIP_CHECK(hipGetLastError());
    return 0;
}

int launch_synth_norm(float *dst, int64_t n, uint64_t key, float scale, hipStream_t s) {
    hipLaunchKernelGGL(k_synth_norm, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s, dst, n, key, scale);
    GHIP_CHECK(hipGetLastError());
    return 0;
}

int launch_embed(const uint8_t *qs, const uint8_t *sc, int wtype, int64_t n_bt, const int *token, float scale,
                 float *out, int64_t E, hipStream_t s) {
    if (wtype == T_Q4_0)
        hipLaunchKernelGGL(k_embed<T_Q4_0>, dim3((unsigned)((E + 255) / 256)), dim3(256), 0, s, qs, sc, n_bt, token,
                           scale, out, E);
    else
        hipLaunchKernelGGL(k_embed<T_Q8_0>, dim3((unsigned)((E + 255) / 256)), dim3(256), 0, s, qs, sc, n_bt, token,
                           scale, out, E);
    GHIP_CHECK(hipGetLastError());
    return 0;
}

attn_geom attn_geometry(int H, int Hkv, int hd, int ctx) {
    attn_geom g{};
    if (Hkv <= 0 || H % Hkv) return g;
    const int G = H / Hkv;
    if (G > ATT_QUADS || ATT_QUADS % G || hd % 8 || (G * hd / 2) % 4 || (hd / 2) / 4 > ATT_THREADS) return g;
    const attn_split sp = attn_split_of(G, hd);
    const int PS = sp.ps, DS = sp.ds;
    if (PS < 1 || DS < 1) return g;
    const int nb = (hd + DS - 1) / DS;
    if (nb * Hkv > ATT_MAXWG) return g;
    const int na = (ctx + PS - 1) / PS;
    g.nwg = std::max(nb, std::min(na, std::min(32, ATT_MAXWG / Hkv)));
    g.grid = 8 * g.nwg * ((Hkv + 7) / 8);  // XCD-colocated groups (idle slots exit at once)
    g.lds = (size_t)G * hd * 2 + (size_t)hd * 2 + (size_t)PS * hd * 2 + (size_t)DS * ATT_VW * 2 + (size_t)G * ctx * 2;
    g.sbuf_floats = (size_t)Hkv * ctx * G;
    g.sync_ints = (size_t)Hkv * 2;
    g.img = DS == 32 && hd % 32 == 0;
    return g;
}

int launch_attn_rows(const attnp_args &a, hipStream_t s) {
    const int G = a.Hkv > 0 ? a.H / a.Hkv : 0;
    const size_t lds = (size_t)G * a.n_kv * (AR_ALIAS ? 4 : 6) + (size_t)G * a.hd * 2;
    if (G <= 0 || G > 8 || a.H % a.Hkv || (AR_THREADS / 4) % G || a.hd % 32 || a.hd > 256 || a.ctx % 32 || a.n_kv % 32 ||
        a.n_kv > a.ctx || a.T <= 0 || a.T > a.n_kv || lds > 160 * 1024) {
        set_error("attn_rows: unsupported shape (head_dim <= 256, G <= 8, 256 % G == 0, G*(n_kv*6 + hd*2) B of LDS <= 160 KiB)");
        return -1;
    }
    GHIP_CHECK(hipFuncSetAttribute((const void *)k_attn_rows, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
    hipLaunchKernelGGL(k_attn_rows, dim3((unsigned)(a.T * a.Hkv)), dim3(AR_THREADS), lds, s, a);
    GHIP_CHECK(hipGetLastError());
    return 0;
}

int launch_attn_decode(const attn_args &a, hipStream_t s) {
    if (a.mode == ATTN_PER_HEAD) {
        if (a.hd % 32 != 0 || a.hd > 256 || a.ctx % 32 != 0 || a.H % a.Hkv != 0 || !a.rope_cur ||
            (a.out_q8k && (a.hd != 256 || a.dsplit != 1)) || a.dsplit < 1 || a.hd % (32 * a.dsplit) ||
            4 * (a.hd / a.dsplit) > AH_THREADS) {
            set_error("attn_decode: unsupported shape for the per-head form");
            return -1;
        }
        size_t lds = ((2 * (size_t)a.hd * 2 + 15) & ~(size_t)15) + (size_t)a.ctx * 4 + (size_t)a.ctx * 2 + 16;
        if (lds > 160 * 1024) {
            set_error("attn_decode: context too long for the LDS image");
            return -1;
        }
        // (V rows by LDS-DMA, and the heads spread over the XCDs, measured neutral / slower: removed,
        // DESIGN.md §10)
        if (lds > 64 * 1024)
            GHIP_CHECK(hipFuncSetAttribute((const void *)k_attn_head, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
        hipLaunchKernelGGL(k_attn_head, dim3(8 * a.H * a.dsplit), dim3(AH_THREADS), lds, s, a);
        GHIP_CHECK(hipGetLastError());
        return 0;
    }
    const attn_geom g = attn_geometry(a.H, a.Hkv, a.hd, a.ctx);
    if (a.hd % 32 != 0 || a.hd > 512 || a.ctx % 32 != 0 || g.nwg == 0 || a.nwg != g.nwg || !a.sbuf || !a.sync ||
        (a.out_act && attn_split_of(a.H / a.Hkv, a.hd).ds != 32) || a.out_q8k) {
        set_error("attn_decode: unsupported shape or missing scratch");
        return -1;
    }
    // every workgroup of a kv group must be resident at once (in-kernel hand-off)
    if (g.nwg * a.Hkv > ATT_MAXWG) {
        set_error("attn_decode: too many workgroups for the in-kernel hand-off");
        return -1;
    }
    if (g.lds > 160 * 1024) {
        set_error("attn_decode: context too long for the LDS image");
        return -1;
    }
    if (g.lds > 64 * 1024)
        GHIP_CHECK(hipFuncSetAttribute((const void *)k_attn_decode, hipFuncAttributeMaxDynamicSharedMemorySize, (int)g.lds));
    hipLaunchKernelGGL(k_attn_decode, dim3(g.grid), dim3(ATT_THREADS), g.lds, s, a);
    GHIP_CHECK(hipGetLastError());
    return 0;
}

int launch_stream_read(const void *buf, size_t bytes, unsigned *sink, hipStream_t s, int variant) {
    if (variant == 1)
        hipLaunchKernelGGL(k_stream_lds, dim3(256 * 2), dim3(256), 0, s, (const uint4 *)buf, (uint64_t)(bytes / 16));
    else
        hipLaunchKernelGGL(k_stream_read, dim3(256 * 16), dim3(256), 0, s, (const uint4 *)buf, (uint64_t)(bytes / 16), sink);
    GHIP_CHECK(hipGetLastError());
    return 0;
}

int launch_exp_f16_all(uint16_t *out, hipStream_t s) {
    hipLaunchKernelGGL(k_exp_f16_all, dim3(256), dim3(256), 0, s, out);
    GHIP_CHECK(hipGetLastError());
    return 0;
}

int launch_reduce_keys(const unsigned long long *keys, int n, int64_t row_base, unsigned long long *out, hipStream_t s) {
    hipLaunchKernelGGL(k_reduce_keys, dim3(1), dim3(256), 0, s, keys, n, row_base, out);
    GHIP_CHECK(hipGetLastError());
    return 0;
}


int launch_advance(const unsigned long long *keys, int n_parts, int *token, int *pos, int *hist, int hist_cap,
                   const int *n_fixed, const rope_row &r, hipStream_t s) {
    hipLaunchKernelGGL(k_advance, dim3(1), dim3(256), 0, s, keys, n_parts, token, pos, hist, hist_cap, n_fixed, r);
    GHIP_CHECK(hipGetLastError());
    return 0;
}

int launch_set_position(int token, int p, int *pos, int *hist, int *n_fixed, int fixed, const rope_row &r, hipStream_t s) {
    hipLaunchKernelGGL(k_set_position, dim3(1), dim3(256), 0, s, token, p, pos, hist, n_fixed, fixed, r);
    GHIP_CHECK(hipGetLastError());
    return 0;
}

int launch_mul_mat_f16(const uint16_t *src0, int64_t nb01e, int64_t ne01, const uint16_t *src1, int64_t rse,
                       int64_t ncols, int64_t K, float *dst, hipStream_t s) {
    const int64_t n = ne01 * ncols;
    hipLaunchKernelGGL(k_mul_mat_f16, dim3((unsigned)((n + 127) / 128)), dim3(128), 0, s, src0, nb01e, ne01, src1, rse,
                       ncols, K, dst);
    GHIP_CHECK(hipGetLastError());
    return 0;
}

}  // namespace ghip
