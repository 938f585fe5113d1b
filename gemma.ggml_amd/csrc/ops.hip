// ops.hip — weight preparation and the small decode-step ops around the matvec (gfx950).
//
//  * k_repack / k_untile: ggml row-major Q4_0/Q8_0 blocks <-> the tiled HBM layout (common.h).
//  * k_synth_*: the synthetic-weight generator (same integer stream and reference quantizers as
//    oracle/gemma_cpu.cpp; DESIGN.md §Synthetic weights), writing straight into the tiled layout.
//  * k_attn_decode: RoPE-NEOX (src/gemma_model.cpp:698-716) + q scale (:708) + KV store (:499-518)
//    + KQ (:474) + soft_max_ext (:476) + KQV (:485) + permute/cont (:487-489) for one token, with
//    ggml's AVX/F16C vec_dot_f16 order and the fp16 exp table (A.6).
//  * k_embed, k_advance (greedy token feedback), k_mul_mat_f16 (C-ABI F16 path).
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

constexpr int ATT_THREADS = 1024;
constexpr int ATT_DCHUNK = 256;  // KQV outputs per workgroup: grid = (H, hd / 256): one pass of 256 quads
constexpr int ATT_KPF = 8;      // K steps (of 32 elements) prefetched per thread: hd <= 256
constexpr int ATT_VPF = 8;      // V steps (of 32 positions) prefetched per thread: n_kv <= 256

// ggml_vec_dot_f16 with accumulator row j = t4 held by lane t4 of a quad: fold the
// quad exactly as sum0+=sum2, sum1+=sum3, sum0+=sum1 (xor-2 then xor-1), then halves and hadds.
__device__ __forceinline__ float quad_reduce_f16(const float acc[8], int t4) {
    float x0[8];
#pragma unroll
    for (int l = 0; l < 8; ++l) x0[l] = quad_fold_dpp(acc[l]);
    float t0[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) t0[i] = x0[i] + x0[i + 4];
    const float h0 = t0[0] + t0[1], h1 = t0[2] + t0[3];
    (void)t4;
    return h0 + h1;
}

__device__ __forceinline__ void f16_step8(float acc[8], uint4 xv, uint4 yv) {
    const uint32_t xs[4] = {xv.x, xv.y, xv.z, xv.w}, ys[4] = {yv.x, yv.y, yv.z, yv.w};
#pragma unroll
    for (int w = 0; w < 4; ++w) {
        acc[2 * w] = __builtin_fmaf(h2f(xs[w]), h2f(ys[w]), acc[2 * w]);
        acc[2 * w + 1] = __builtin_fmaf(h2f(xs[w] >> 16), h2f(ys[w] >> 16), acc[2 * w + 1]);
    }
}

// One token's attention for head h = blockIdx.x, KQV outputs [64*blockIdx.y, +64).  Every
// workgroup recomputes the (cheap) RoPE, KQ and softmax of its head.  Quads of lanes own one KQ
// position (or one KQV output): lane t4 runs accumulator row j = t4 of the AVX/F16C loop.  The
// K rows and V rows of the first pass are requested at kernel entry, before RoPE.
__global__ void __launch_bounds__(ATT_THREADS) k_attn_decode(attn_args a) {
    extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
    const int hd = a.hd, half = hd / 2, tid = threadIdx.x, t4 = tid & 3, quad = tid >> 2;
    const int h = blockIdx.x, ds = blockIdx.y, grp = a.H / a.Hkv, kvh = h / grp;
    if (a.dbg_t && tid == 0) a.dbg_t[(blockIdx.x * gridDim.y + blockIdx.y) * 8 + 0] = __builtin_amdgcn_s_memrealtime();
    const int pos = *a.pos;
    const int n_total = pos + 1;
    int n_kv = 32 * (n_total / 32 + 1);                    // src/gemma_model.cpp:429
    if (n_kv > a.ctx) n_kv = a.ctx;
    const int kvw = a.Hkv * hd;
    const int nq = blockDim.x >> 2;                      // quads per workgroup (64)
    // ---- early loads: first KQ pass (position `quad`) and the first V steps of output d
    const int d0 = ds * ATT_DCHUNK + quad;
    const uint16_t *vrow = a.vc + ((int64_t)kvh * hd + (d0 < hd ? d0 : 0)) * a.ctx;
    uint4 kpre[ATT_KPF], vpre[ATT_VPF];
    {
        const int j = quad < a.ctx ? quad : 0;           // no dependency on *pos: rows >= pos are masked
        const uint16_t *krow = a.kc + (int64_t)j * kvw + (int64_t)kvh * hd + t4 * 8;
#pragma unroll
        for (int s = 0; s < ATT_KPF; ++s) kpre[s] = *(const uint4 *)(krow + (s * 32 < hd ? s * 32 : 0));
#pragma unroll
        for (int s = 0; s < ATT_VPF; ++s) vpre[s] = *(const uint4 *)(vrow + (s * 32 < a.ctx ? s * 32 : 0) + t4 * 8);
    }
    uint16_t *q16 = (uint16_t *)smem;                    // hd
    uint16_t *k16 = q16 + hd;                            // hd (this token's k, post-rope)
    uint16_t *v16 = k16 + hd;                            // hd (this token's v)
    float *S = (float *)(smem + ((3 * hd * 2 + 15) & ~15));  // ctx
    uint16_t *P16 = (uint16_t *)(S + a.ctx);             // ctx

    // RoPE NEOX on q (then * q_scale) and on k; f32 -> f16 (ggml_cpy / MUL_MAT INIT conversions)
    const float *cs = a.rope_cos + (int64_t)pos * half, *sn = a.rope_sin + (int64_t)pos * half;
    const float *qh = a.qkv + (int64_t)h * hd;
    const float *kh = a.qkv + (int64_t)a.H * hd + (int64_t)kvh * hd;
    const float *vh = a.qkv + (int64_t)a.H * hd + kvw + (int64_t)kvh * hd;
    for (int i = tid; i < half; i += blockDim.x) {
        const float c = cs[i], s = sn[i];
        {
            const float x0 = qh[i], x1 = qh[i + half];
            const float p0 = x0 * c, p1 = x1 * s, p2 = x0 * s, p3 = x1 * c;
            const float r0 = p0 - p1, r1 = p2 + p3;
            q16[i] = f2h(r0 * a.q_scale);
            q16[i + half] = f2h(r1 * a.q_scale);
        }
        {
            const float x0 = kh[i], x1 = kh[i + half];
            const float p0 = x0 * c, p1 = x1 * s, p2 = x0 * s, p3 = x1 * c;
            k16[i] = f2h(p0 - p1);
            k16[i + half] = f2h(p2 + p3);
        }
    }
    for (int i = tid; i < hd; i += blockDim.x) v16[i] = f2h(vh[i]);
    __syncthreads();
    if (a.dbg_t && tid == 0) a.dbg_t[(blockIdx.x * gridDim.y + blockIdx.y) * 8 + 1] = __builtin_amdgcn_s_memrealtime();
    if (h % grp == 0) {  // one writer per kv head: K row `pos`, V column `pos` (src/gemma_model.cpp:506-517)
        for (int i = ds * ATT_DCHUNK + tid; i < (ds + 1) * ATT_DCHUNK && i < hd; i += blockDim.x) {
            a.kc[(int64_t)pos * kvw + (int64_t)kvh * hd + i] = k16[i];
            a.vc[((int64_t)kvh * hd + i) * a.ctx + pos] = v16[i];
        }
    }
    // ---- KQ (vec_dot_f16 over hd per kv position) + mask (j > pos -> -inf), scale 1.0
    for (int j0 = 0; j0 < n_kv; j0 += nq) {
        const int j = j0 + quad;
        float acc[8];
#pragma unroll
        for (int y = 0; y < 8; ++y) acc[y] = 0.0f;
        if (j0 == 0) {
#pragma unroll
            for (int s = 0; s < ATT_KPF; ++s)
                if (s * 32 < hd) {
                    const uint4 kv = (j == pos) ? *(const uint4 *)(k16 + s * 32 + t4 * 8) : kpre[s];
                    f16_step8(acc, kv, *(const uint4 *)(q16 + s * 32 + t4 * 8));
                }
            for (int s = ATT_KPF; s * 32 < hd; ++s) {
                const uint16_t *krow = (j == pos) ? k16 : a.kc + (int64_t)j * kvw + (int64_t)kvh * hd;
                f16_step8(acc, *(const uint4 *)(krow + s * 32 + t4 * 8), *(const uint4 *)(q16 + s * 32 + t4 * 8));
            }
        } else {
            const int jc = j < pos ? j : pos;
            const uint16_t *krow = (jc == pos) ? k16 : a.kc + (int64_t)jc * kvw + (int64_t)kvh * hd;
            for (int s = 0; s * 32 < hd; ++s)
                f16_step8(acc, *(const uint4 *)(krow + s * 32 + t4 * 8), *(const uint4 *)(q16 + s * 32 + t4 * 8));
        }
        const float kq = quad_reduce_f16(acc, t4);
        if (t4 == 0 && j < n_kv) {
            const float w = (j > pos) ? -INFINITY : kq * 1.0f + 0.0f;
            S[j] = w;
            if (a.dbg_w && ds == 0) a.dbg_w[(int64_t)h * a.ctx + j] = w;
        }
    }
    __syncthreads();
    if (a.dbg_t && tid == 0) a.dbg_t[(blockIdx.x * gridDim.y + blockIdx.y) * 8 + 2] = __builtin_amdgcn_s_memrealtime();
    // ---- soft_max_ext: max; e = table_exp[f16(w - max)]; exact sum; e * (float)(1/sum)
    // Every wave reduces the whole row itself (DPP, no LDS round trip) and writes P16 for its own
    // slice j = 64*wave + lane (+ blockDim.x*m): one barrier for the softmax instead of three.
    const int lane = tid & 63, wave = tid >> 6;
    float mx = -INFINITY;
    for (int j = lane; j < n_kv; j += 64) mx = fmaxf(mx, S[j]);
    mx = wave_max(mx);
    if (a.dbg_t && tid == 0) a.dbg_t[(blockIdx.x * gridDim.y + blockIdx.y) * 8 + 3] = __builtin_amdgcn_s_memrealtime();
    // e values are fp16 in [0,1]: exact multiples of 2^-24, so an integer sum is the exact sum
    // (ggml's double accumulation of them is exact too).
    unsigned long long isum = 0;
    float mine[4] = {0.0f, 0.0f, 0.0f, 0.0f};  // e of this wave's own slice (n_kv <= 4 * blockDim.x)
    for (int j = lane, k = 0; j < n_kv; j += 64, ++k) {
        const float w = S[j];
        float e = 0.0f;
        if (w != -INFINITY) e = h2f(a.exp_tab[f2h(w - mx)]);
        isum += (unsigned long long)(e * 16777216.0f);
        const int r = k - wave;  // slot of j = 64*wave + lane + blockDim.x*m
        if (r >= 0 && (r & ((int)(blockDim.x >> 6) - 1)) == 0) {
            const int m = r / (int)(blockDim.x >> 6);
            if (m == 0) mine[0] = e; else if (m == 1) mine[1] = e; else if (m == 2) mine[2] = e; else mine[3] = e;
        }
    }
    const unsigned long long tot = wave_sum_u64(isum);
    if (a.dbg_t && tid == 0) a.dbg_t[(blockIdx.x * gridDim.y + blockIdx.y) * 8 + 4] = __builtin_amdgcn_s_memrealtime();
    const double sum = (double)tot * (1.0 / 16777216.0);
    const float inv = (float)(1.0 / sum);
    if (a.dbg_inv && tid == 0 && ds == 0) a.dbg_inv[h] = inv;
    for (int j = tid, m = 0; j < n_kv; j += blockDim.x, ++m) {
        float e;
        if (m < 4) {
            e = m == 0 ? mine[0] : m == 1 ? mine[1] : m == 2 ? mine[2] : mine[3];
        } else {  // long rows: recompute (same table lookup, same value)
            const float w = S[j];
            e = w != -INFINITY ? h2f(a.exp_tab[f2h(w - mx)]) : 0.0f;
        }
        P16[j] = f2h(e * inv);
        if (a.dbg_p && ds == 0) a.dbg_p[(int64_t)h * a.ctx + j] = P16[j];
    }
    __syncthreads();
    if (a.dbg_t && tid == 0) a.dbg_t[(blockIdx.x * gridDim.y + blockIdx.y) * 8 + 5] = __builtin_amdgcn_s_memrealtime();
    // ---- KQV: out[d] = vec_dot_f16(n_kv, V[kvh][d][0..n_kv), P16); lane t4 runs accumulator j = t4
    for (int d = d0; d < (ds + 1) * ATT_DCHUNK && d < hd; d += nq) {
        float acc[8];
#pragma unroll
        for (int y = 0; y < 8; ++y) acc[y] = 0.0f;
        const uint16_t *vr = a.vc + ((int64_t)kvh * hd + d) * a.ctx;
        for (int st = 0, s = 0; st < n_kv; st += 32, ++s) {
            const int e0 = st + t4 * 8;
            uint4 xv;
            if (d == d0 && s < ATT_VPF) {
                // statically-indexed pick from the early loads
                xv = vpre[0];
#pragma unroll
                for (int k = 1; k < ATT_VPF; ++k)
                    if (s == k) xv = vpre[k];
            } else {
                xv = *(const uint4 *)(vr + e0);
            }
            if (pos >= e0 && pos < e0 + 8) {  // this token's V: only the LDS copy is safe to read
                __attribute__((aligned(16))) uint16_t tmp[8];
                *(uint4 *)tmp = xv;
                tmp[pos - e0] = v16[d];
                xv = *(const uint4 *)tmp;
            }
            f16_step8(acc, xv, *(const uint4 *)(P16 + e0));
        }
        const float o = quad_reduce_f16(acc, t4);
        if (t4 == 0) a.out[(int64_t)h * hd + d] = o;
    }
    if (a.dbg_t && tid == 0) a.dbg_t[(blockIdx.x * gridDim.y + blockIdx.y) * 8 + 6] = __builtin_amdgcn_s_memrealtime();
}

__global__ void __launch_bounds__(256) k_advance(const unsigned long long *keys, int n_parts, int *token, int *pos,
                                                 int *hist, int hist_cap, const int *n_fixed) {
    __shared__ unsigned long long red[4];
    unsigned long long best = 0;
    for (int i = threadIdx.x; i < n_parts; i += blockDim.x) best = keys[i] > best ? keys[i] : best;
#pragma unroll
    for (int off = 32; off >= 1; off >>= 1) {
        const unsigned long long o = __shfl_xor(best, off);
        best = o > best ? o : best;
    }
    if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = best;
    __syncthreads();
    if (threadIdx.x != 0) return;
    for (int w = 1; w < (int)(blockDim.x >> 6); ++w) best = red[w] > best ? red[w] : best;
    // strict '>' argmax, first max wins (src/gemma_model.cpp:538-543): the key's low word is ~index
    const int idx = (int)(0xFFFFFFFFu - (uint32_t)(best & 0xFFFFFFFFull));
    const int p = *pos + 1;
    *token = idx;
    if (hist && p < hist_cap && p >= *n_fixed) hist[p] = idx;  // never overwrite the prompt
    *pos = p;
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

int launch_attn_decode(const attn_args &a, hipStream_t s) {
    if (a.hd % 32 != 0 || a.hd > 512 || a.ctx % 32 != 0 || a.H % a.Hkv != 0) {
        set_error("attn_decode: unsupported shape");
        return -1;
    }
    const size_t lds = ((3 * (size_t)a.hd * 2 + 15) & ~(size_t)15) + (size_t)a.ctx * 4 + (size_t)a.ctx * 2 + 16 + 64 +
                       64 + 8 + 128;  // red: 16 floats, align, 16 u64
    if (lds > 160 * 1024) {
        set_error("attn_decode: context too long for the LDS image");
        return -1;
    }
    if (lds > 64 * 1024)
        GHIP_CHECK(hipFuncSetAttribute((const void *)k_attn_decode, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
    hipLaunchKernelGGL(k_attn_decode, dim3(a.H, (a.hd + ATT_DCHUNK - 1) / ATT_DCHUNK), dim3(ATT_THREADS), lds, s, a);
    GHIP_CHECK(hipGetLastError());
    return 0;
}

int launch_advance(const unsigned long long *keys, int n_parts, int *token, int *pos, int *hist, int hist_cap,
                   const int *n_fixed, hipStream_t s) {
    hipLaunchKernelGGL(k_advance, dim3(1), dim3(256), 0, s, keys, n_parts, token, pos, hist, hist_cap, n_fixed);
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
