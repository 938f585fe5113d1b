// matvec.hip — the decode hot path: fused Q4_0/Q8_0 dequant x Q8_0-activation matvec for gfx950.
//
// Replaces, for one MUL_MAT node, the reference's INIT (src1 -> Q8_0, ggml [ext]) plus
// `mul_mat` (src/hpc.cpp:216-273) whose per-(row,col) `vec_dot` (src/hpc.cpp:35-36) is
// ggml_vec_dot_q4_0_q8_0 / q8_0_q8_0.
//
// Bit-exactness: ggml's AVX2 vec_dot keeps 8 fp32 lanes per row; lane l accumulates
// fmaf(d_w*d_a, (float)isum(elements 4l..4l+3), acc_l) block after block and the lanes are
// folded as ((a0+a4)+(a2+a6))+((a1+a5)+(a3+a7)).  Here one GPU thread *is* one of
// those lanes: a wave = 8 rows x 8 lanes, each thread runs its lane's fma chain in block order,
// the integer part is one v_dot4_i32_i8 per block (exact), and the fold is a xor-4/2/1
// butterfly — so results equal the ordered CPU restatement bit for bit.
//
// Memory: weights are read once, 16 B per thread per 8-block tile (1 KiB coalesced per wave;
// DESIGN.md §HBM layout); the activation is quantized once per workgroup in the prologue
// (optionally fused with RMSNorm and the embedding lookup) and staged in LDS.
// K-split (KS > 1): the waves of a workgroup each take a contiguous K segment of the same 8 rows;
// waves 1..KS-1 stash their exact (d, isum) terms in LDS and the fma chain is carried across the
// segments in order (wave w continues wave w-1's accumulator), which keeps the AVX2 order.
#include "device_util.h"
#include "kernels.h"

namespace ghip {
namespace {

__device__ __forceinline__ int sdot4(uint32_t a, uint32_t b, int c) {
    return __builtin_amdgcn_sdot4((int)a, (int)b, c, false);
}

// ---- LDS image --------------------------------------------------------------------------------
// act: Q4_0 -> uint4 [n_bt*4 pairs][8 lanes] = {a_b, -8*sum(a_b), a_b+1, -8*sum(a_b+1)}
//      Q8_0 -> uint4 [n_bt][8 lanes]        = {a_b0, a_b1, a_b2, a_b3}
// da:  float [n_bt*BT] (fp32 of the fp16 activation scale)
struct lds_map {
    size_t act, da, stash_s, stash_d, xfer, red, total;
};
template <int WT>
__host__ __device__ inline lds_map make_lds_map(int ks, int64_t n_bt, int64_t seg_tiles) {
    constexpr int BT = wfmt<WT>::BT;
    lds_map m;
    m.act = 0;
    const size_t act_bytes = WT == T_Q4_0 ? (size_t)n_bt * 4 * 8 * 16 : (size_t)n_bt * 8 * 16;
    m.da = act_bytes;
    size_t off = m.da + (size_t)n_bt * BT * 4;
    off = (off + 15) & ~(size_t)15;
    const size_t seg_blocks = (size_t)seg_tiles * BT;
    const size_t s_elem = WT == T_Q4_0 ? 2 : 4;
    m.stash_s = off;
    off += (ks > 1 ? (size_t)(ks - 1) * seg_blocks * 64 * s_elem : 0);
    off = (off + 15) & ~(size_t)15;
    m.stash_d = off;
    off += (ks > 1 ? (size_t)(ks - 1) * seg_blocks * 8 * 4 : 0);
    m.xfer = off;
    off += 2 * 64 * 4;
    m.red = off;
    off += 64 * 8;
    m.total = off;
    return m;
}

// ---- prologue: build the Q8_0 activation image in LDS (quantize_row_q8_0) ------
// Writes block b (32 values v[0..31]) in the layout above.  amax, d = amax/127 (fp16 RNE),
// id = amax ? 127/amax : 0, q = rint(v*id) — identical to oracle orc_quantize_row_q8_0.
template <int WT>
__device__ __forceinline__ void put_block(uint8_t *smem, const lds_map &m, int64_t b, const float *v) {
    float amax = 0.0f;
#pragma unroll
    for (int j = 0; j < 32; ++j) amax = fmaxf(amax, fabsf(v[j]));
    const float d = amax / 127.f;
    const uint32_t d16 = f2h(d);
    const float id = (amax != 0.0f) ? 127.f / amax : 0.0f;
    uint32_t *act = (uint32_t *)(smem + m.act);
#pragma unroll
    for (int l = 0; l < 8; ++l) {
        int q[4];
#pragma unroll
        for (int k = 0; k < 4; ++k) q[k] = (int)__builtin_rintf(v[4 * l + k] * id);
        const uint32_t packed = (uint32_t)(q[0] & 0xFF) | ((uint32_t)(q[1] & 0xFF) << 8) |
                                ((uint32_t)(q[2] & 0xFF) << 16) | ((uint32_t)(q[3] & 0xFF) << 24);
        if (WT == T_Q4_0) {
            const int nsa = -8 * (q[0] + q[1] + q[2] + q[3]);
            const int64_t base = ((b >> 1) * 8 + l) * 4 + (b & 1) * 2;
            act[base] = packed;
            act[base + 1] = (uint32_t)nsa;
        } else {
            act[((b >> 2) * 8 + l) * 4 + (b & 3)] = packed;
        }
    }
    ((float *)(smem + m.da))[b] = h2f(d16);
}

template <int WT>
__device__ __forceinline__ void put_block_q8(uint8_t *smem, const lds_map &m, int64_t b, const block_q8_0 *blk) {
    const uint8_t *p = (const uint8_t *)blk;
    const uint32_t d16 = (uint32_t)p[0] | ((uint32_t)p[1] << 8);
    uint32_t *act = (uint32_t *)(smem + m.act);
#pragma unroll
    for (int l = 0; l < 8; ++l) {
        int q[4];
#pragma unroll
        for (int k = 0; k < 4; ++k) q[k] = (int)(int8_t)p[2 + 4 * l + k];
        const uint32_t packed = (uint32_t)(q[0] & 0xFF) | ((uint32_t)(q[1] & 0xFF) << 8) |
                                ((uint32_t)(q[2] & 0xFF) << 16) | ((uint32_t)(q[3] & 0xFF) << 24);
        if (WT == T_Q4_0) {
            const int64_t base = ((b >> 1) * 8 + l) * 4 + (b & 1) * 2;
            act[base] = packed;
            act[base + 1] = (uint32_t)(-8 * (q[0] + q[1] + q[2] + q[3]));
        } else {
            act[((b >> 2) * 8 + l) * 4 + (b & 3)] = packed;
        }
    }
    ((float *)(smem + m.da))[b] = h2f(d16);
}

// embedding row element: tiled Q4_0/Q8_0 row `row`, block b, element e (ggml order)
template <int EWT>
__device__ __forceinline__ float emb_value(const uint8_t *qs, const uint8_t *sc, int64_t n_bt, int64_t row, int64_t b,
                                           int e) {
    constexpr int BT = wfmt<EWT>::BT;
    const int64_t rt = row >> 3, rr = row & 7, bt = b / BT, bi = b % BT;
    const int64_t tile = rt * n_bt + bt;
    const int l = e >> 2, k = e & 3;
    const uint16_t d16 = ((const uint16_t *)(sc + tile * 8 * wfmt<EWT>::SCALE_BYTES + rr * wfmt<EWT>::SCALE_BYTES))[bi];
    const uint8_t *t = qs + tile * 1024 + (rr * 8 + l) * 16;
    int q;
    if (EWT == T_Q4_0) {
        const uint8_t byte = t[(bi >> 1) * 4 + k];
        q = (int)((bi & 1) ? (byte >> 4) : (byte & 15)) - 8;
    } else {
        q = (int)(int8_t)t[bi * 4 + k];
    }
    return (float)q * pin(h2f(d16));  // pinned: keep a true v_mul_f32 (sign of zero as on the CPU)
}

template <int WT, int PRO>
__device__ void build_activation(const mv_args &a, int col, uint8_t *smem, const lds_map &m) {
    constexpr int BT = wfmt<WT>::BT;
    const int tid = threadIdx.x, nth = blockDim.x;
    const int64_t nb = a.nb, nb_pad = a.n_bt * BT;
    // zero the padded tail blocks (their d = 0 makes every chain step an exact no-op)
    for (int64_t b = nb + tid; b < nb_pad; b += nth) {
        float z[32];
#pragma unroll
        for (int j = 0; j < 32; ++j) z[j] = 0.0f;
        put_block<WT>(smem, m, b, z);
    }
    if (PRO == PRO_Q8) {
        const block_q8_0 *xb = (const block_q8_0 *)((const uint8_t *)a.x + (int64_t)col * a.x_col_stride);
        for (int64_t b = tid; b < nb; b += nth) put_block_q8<WT>(smem, m, b, xb + b);
        return;
    }
    // f32 source (PRO_F32 / PRO_NORM) or dequantized embedding row (PRO_EMBED)
    const float *x = (const float *)((const uint8_t *)a.x + (int64_t)col * a.x_col_stride);
    int64_t tok = 0;
    if (PRO == PRO_EMBED) tok = ((const int *)a.x)[*a.tok_pos];
    auto load = [&](int64_t i) -> float {
        if (PRO == PRO_EMBED) {
            const float v = emb_value<WT>(a.emb_qs, a.emb_sc, a.emb_n_bt, tok, i >> 5, (int)(i & 31));
            return v * a.emb_scale;   // ggml_get_rows then ggml_scale (src/gemma_model.cpp:677-679)
        }
        return x[i];
    };
    float scale = 1.0f;
    if (PRO == PRO_NORM || PRO == PRO_EMBED) {
        // rms_norm: double sum of fp32 squares, fixed-order tree
        double part = 0.0;
        for (int64_t i = tid; i < nb * 32; i += nth) {
            const float v = load(i);
            const float sq = v * v;
            part += (double)sq;
        }
        double *red = (double *)(smem + m.red);
#pragma unroll
        for (int off = 32; off >= 1; off >>= 1) part += __shfl_xor(part, off);
        if ((tid & 63) == 0) red[tid >> 6] = part;
        __syncthreads();
        double sum = 0.0;
        for (int w = 0; w < nth / 64; ++w) sum += red[w];
        const float mean = (float)(sum / (double)(nb * 32));
        scale = 1.0f / sqrtf(mean + a.eps);
        __syncthreads();
        if (PRO == PRO_EMBED && a.emb_out && blockIdx.x == 0 && col == 0)
            for (int64_t i = tid; i < nb * 32; i += nth) a.emb_out[i] = load(i);
    }
    for (int64_t b = tid; b < nb; b += nth) {
        float v[32];
#pragma unroll
        for (int j = 0; j < 32; ++j) {
            float t = load(b * 32 + j);
            if (PRO == PRO_NORM || PRO == PRO_EMBED) {
                t = t * scale;            // rms_norm output
                t = t * a.norm_w[b * 32 + j];  // ggml_mul by the norm weight
            }
            v[j] = t;
        }
        put_block<WT>(smem, m, b, v);
    }
}

// ---- one 8-row x BT-block tile for this thread's (row rr, lane l) ----------------------------
// STASH: write the exact (d, isum) terms instead of accumulating (K-split waves 1..KS-1)
template <int WT, bool STASH>
__device__ __forceinline__ float tile_dot(uint4 q, uint4 scv, const uint8_t *smem, const lds_map &m, int64_t bt, int l,
                                          float acc, int16_t *st_s, int32_t *st_s32, float *st_d, int j0, int rr,
                                          int lane) {
    const float *da = (const float *)(smem + m.da);
    const uint32_t qv[4] = {q.x, q.y, q.z, q.w};
    if (WT == T_Q4_0) {
        const uint4 *act = (const uint4 *)(smem + m.act);
        const float4 DA0 = *(const float4 *)(da + bt * 8), DA1 = *(const float4 *)(da + bt * 8 + 4);
        const float dav[8] = {DA0.x, DA0.y, DA0.z, DA0.w, DA1.x, DA1.y, DA1.z, DA1.w};
        const uint32_t sv[4] = {scv.x, scv.y, scv.z, scv.w};
#pragma unroll
        for (int p = 0; p < 4; ++p) {
            const uint4 A = act[(bt * 4 + p) * 8 + l];
            const uint32_t lo = qv[p] & 0x0F0F0F0Fu, hi = (qv[p] >> 4) & 0x0F0F0F0Fu;
            const int s0 = sdot4(lo, A.x, (int)A.y);
            const int s1 = sdot4(hi, A.z, (int)A.w);
            const float d0 = h2f(sv[p]) * dav[2 * p];
            const float d1 = h2f(sv[p] >> 16) * dav[2 * p + 1];
            if (STASH) {
                st_s[(j0 + 2 * p) * 64 + lane] = (int16_t)s0;
                st_s[(j0 + 2 * p + 1) * 64 + lane] = (int16_t)s1;
                if (l == 0) {
                    st_d[(j0 + 2 * p) * 8 + rr] = d0;
                    st_d[(j0 + 2 * p + 1) * 8 + rr] = d1;
                }
            } else {
                acc = __builtin_fmaf(d0, (float)s0, acc);
                acc = __builtin_fmaf(d1, (float)s1, acc);
            }
        }
    } else {
        const uint4 A = ((const uint4 *)(smem + m.act))[bt * 8 + l];
        const uint32_t av[4] = {A.x, A.y, A.z, A.w};
        const float4 DA = *(const float4 *)(da + bt * 4);
        const float dav[4] = {DA.x, DA.y, DA.z, DA.w};
        const uint32_t sv[4] = {scv.x & 0xFFFF, scv.x >> 16, scv.y & 0xFFFF, scv.y >> 16};
#pragma unroll
        for (int p = 0; p < 4; ++p) {
            const int s = sdot4(qv[p], av[p], 0);
            const float d = h2f(sv[p]) * dav[p];
            if (STASH) {
                st_s32[(j0 + p) * 64 + lane] = s;
                if (l == 0) st_d[(j0 + p) * 8 + rr] = d;
            } else {
                acc = __builtin_fmaf(d, (float)s, acc);
            }
        }
    }
    return acc;
}

template <int WT>
__device__ __forceinline__ uint4 load_scale(const uint8_t *sc, int64_t tile, int rr) {
    if (WT == T_Q4_0) return ((const uint4 *)sc)[tile * 8 + rr];
    const uint2 v = ((const uint2 *)sc)[tile * 8 + rr];
    return make_uint4(v.x, v.y, 0, 0);
}

// chain over block tiles [bt0, bt1) of row tile rt, 4-deep register prefetch
template <int WT, bool STASH>
__device__ __forceinline__ float run_chain(const uint8_t *qs, const uint8_t *sc, int64_t n_bt, int64_t rt, int64_t bt0,
                                           int64_t bt1, const uint8_t *smem, const lds_map &m, float acc, int lane,
                                           int16_t *st_s, int32_t *st_s32, float *st_d) {
    constexpr int BT = wfmt<WT>::BT;
    constexpr int U = 4;
    const int rr = lane >> 3, l = lane & 7;
    const int64_t base = rt * n_bt + bt0;
    const uint4 *q = (const uint4 *)qs + base * 64 + lane;
    const int n = (int)(bt1 - bt0);
    uint4 qb[U], sb[U];
#pragma unroll
    for (int u = 0; u < U; ++u)
        if (u < n) {
            qb[u] = q[(int64_t)u * 64];
            sb[u] = load_scale<WT>(sc, base + u, rr);
        }
    for (int i = 0; i < n; i += U) {
#pragma unroll
        for (int u = 0; u < U; ++u) {
            if (i + u < n) {
                const uint4 qc = qb[u], scc = sb[u];
                if (i + u + U < n) {
                    qb[u] = q[(int64_t)(i + u + U) * 64];
                    sb[u] = load_scale<WT>(sc, base + i + u + U, rr);
                }
                acc = tile_dot<WT, STASH>(qc, scc, smem, m, bt0 + i + u, l, acc, st_s, st_s32, st_d, (i + u) * BT, rr,
                                          lane);
            }
        }
    }
    return acc;
}

// ordered fold of the 8 lanes (hsum_float_8): xor 4, then 2, then 1
__device__ __forceinline__ float fold8(float v) {
    v = v + __shfl_xor(v, 4);
    v = v + __shfl_xor(v, 2);
    v = v + __shfl_xor(v, 1);
    return v;
}

__device__ __forceinline__ unsigned long long argmax_key(float v, int64_t idx) {
    uint32_t u = __builtin_bit_cast(uint32_t, v);
    u = (u & 0x80000000u) ? ~u : (u | 0x80000000u);
    return ((unsigned long long)u << 32) | (unsigned long long)(0xFFFFFFFFu - (uint32_t)idx);
}

__device__ __forceinline__ float gelu_tab(const mv_args &a, float x) {
    if (a.gelu_clamp && x <= -10.0f) return 0.0f;
    if (a.gelu_clamp && x >= 10.0f) return x;
    return h2f(a.gelu_tab[f2h(x)]);
}

template <int EPI>
__device__ __forceinline__ void epilogue(const mv_args &a, int col, int64_t row, float v, float vb,
                                         unsigned long long &best) {
    if (row >= a.rows) return;
    float *y = a.y + (int64_t)col * a.y_col_stride;
    if (EPI == EPI_STORE) y[row] = v;
    if (EPI == EPI_ADD) y[row] = v + a.resid[(int64_t)col * a.y_col_stride + row];
    if (EPI == EPI_GELU_MUL) y[row] = gelu_tab(a, v) * vb;
    if (EPI == EPI_ARGMAX) {
        y[row] = v;
        const unsigned long long k = argmax_key(v, row);
        best = k > best ? k : best;
    }
}

template <int WT, int KS, int PRO, int EPI>
__global__ void __launch_bounds__(512) k_matvec(mv_args a) {
    extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
    constexpr int BT = wfmt<WT>::BT;
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int col = blockIdx.y;
    const int64_t seg_tiles = KS > 1 ? a.n_bt / KS : a.n_bt;
    const lds_map m = make_lds_map<WT>(KS, a.n_bt, seg_tiles);
    build_activation<WT, PRO>(a, col, smem, m);
    __syncthreads();
    unsigned long long best = 0;
    const int rr = lane >> 3;

    if (KS == 1) {
        const int nw = blockDim.x >> 6;
        for (int64_t rt = (int64_t)blockIdx.x * nw + wave; rt < a.n_rt; rt += (int64_t)gridDim.x * nw) {
            float acc = run_chain<WT, false>(a.qs, a.sc, a.n_bt, rt, 0, a.n_bt, smem, m, 0.0f, lane, nullptr, nullptr,
                                             nullptr);
            const float v = fold8(acc);
            float vb = 0.0f;
            if (EPI == EPI_GELU_MUL) {
                float accb = run_chain<WT, false>(a.qs2, a.sc2, a.n_bt, rt, 0, a.n_bt, smem, m, 0.0f, lane, nullptr,
                                                  nullptr, nullptr);
                vb = fold8(accb);
            }
            if ((lane & 7) == 0) epilogue<EPI>(a, col, rt * 8 + rr, v, vb, best);
        }
    } else {
        float *xfer = (float *)(smem + m.xfer);
        int16_t *st_s16 = (int16_t *)(smem + m.stash_s);
        int32_t *st_s32 = (int32_t *)(smem + m.stash_s);
        float *st_d = (float *)(smem + m.stash_d);
        const int seg_blocks = (int)(seg_tiles * BT);
        int16_t *my_s16 = st_s16 + (size_t)(wave > 0 ? wave - 1 : 0) * seg_blocks * 64;
        int32_t *my_s32 = st_s32 + (size_t)(wave > 0 ? wave - 1 : 0) * seg_blocks * 64;
        float *my_d = st_d + (size_t)(wave > 0 ? wave - 1 : 0) * seg_blocks * 8;
        for (int64_t rt = blockIdx.x; rt < a.n_rt; rt += gridDim.x) {
            const int64_t bt0 = wave * seg_tiles, bt1 = bt0 + seg_tiles;
            float acc = 0.0f;
            if (wave == 0)
                acc = run_chain<WT, false>(a.qs, a.sc, a.n_bt, rt, bt0, bt1, smem, m, 0.0f, lane, nullptr, nullptr,
                                           nullptr);
            else
                run_chain<WT, true>(a.qs, a.sc, a.n_bt, rt, bt0, bt1, smem, m, 0.0f, lane, my_s16, my_s32, my_d);
            __syncthreads();
            // ordered carry: wave w continues wave w-1's accumulator over its stashed terms
            for (int w = 1; w < KS; ++w) {
                if (wave == w - 1) xfer[(w & 1) * 64 + lane] = acc;
                __syncthreads();
                if (wave == w) {
                    acc = xfer[(w & 1) * 64 + lane];
#pragma unroll 8
                    for (int j = 0; j < seg_blocks; ++j) {
                        const float d = my_d[j * 8 + rr];
                        const float s = WT == T_Q4_0 ? (float)my_s16[j * 64 + lane] : (float)my_s32[j * 64 + lane];
                        acc = __builtin_fmaf(d, s, acc);
                    }
                }
            }
            if (wave == KS - 1) {
                const float v = fold8(acc);
                if ((lane & 7) == 0) epilogue<EPI>(a, col, rt * 8 + rr, v, 0.0f, best);
            }
            __syncthreads();
        }
    }
    if (EPI == EPI_ARGMAX) {
        // wave-level max then one atomic per wave (first max wins via the index complement)
#pragma unroll
        for (int off = 32; off >= 1; off >>= 1) {
            const unsigned long long o = __shfl_xor(best, off);
            best = o > best ? o : best;
        }
        if (lane == 0 && best != 0) atomicMax(a.argmax_key, best);
    }
}

template <int WT, int KS, int PRO, int EPI>
int launch_t(const mv_args &a, int grid_x, hipStream_t s) {
    const int64_t seg = KS > 1 ? a.n_bt / KS : a.n_bt;
    const lds_map m = make_lds_map<WT>(KS, a.n_bt, seg);
    const int threads = KS > 1 ? 64 * KS : 256;
    if (KS > 1 && a.n_bt % KS != 0) {
        set_error("matvec: n_bt not divisible by KS");
        return -1;
    }
    if (m.total > 160 * 1024) {
        set_error("matvec: LDS image too large");
        return -1;
    }
    if (m.total > 64 * 1024)
        GHIP_CHECK(hipFuncSetAttribute((const void *)k_matvec<WT, KS, PRO, EPI>,
                                       hipFuncAttributeMaxDynamicSharedMemorySize, (int)m.total));
    hipLaunchKernelGGL((k_matvec<WT, KS, PRO, EPI>), dim3(grid_x, a.ncols), dim3(threads), m.total, s, a);
    GHIP_CHECK(hipGetLastError());
    return 0;
}

template <int WT, int KS, int PRO>
int dispatch_epi(int epi, const mv_args &a, int g, hipStream_t s) {
    switch (epi) {
        case EPI_STORE: return launch_t<WT, KS, PRO, EPI_STORE>(a, g, s);
        case EPI_ADD: return launch_t<WT, KS, PRO, EPI_ADD>(a, g, s);
        case EPI_GELU_MUL: return KS == 1 ? launch_t<WT, 1, PRO, EPI_GELU_MUL>(a, g, s) : -1;
        case EPI_ARGMAX: return launch_t<WT, KS, PRO, EPI_ARGMAX>(a, g, s);
    }
    return -1;
}

template <int WT, int KS>
int dispatch_pro(int pro, int epi, const mv_args &a, int g, hipStream_t s) {
    switch (pro) {
        case PRO_F32: return dispatch_epi<WT, KS, PRO_F32>(epi, a, g, s);
        case PRO_NORM: return dispatch_epi<WT, KS, PRO_NORM>(epi, a, g, s);
        case PRO_Q8: return dispatch_epi<WT, KS, PRO_Q8>(epi, a, g, s);
        case PRO_EMBED: return dispatch_epi<WT, KS, PRO_EMBED>(epi, a, g, s);
    }
    return -1;
}

template <int WT>
int dispatch_ks(int ks, int pro, int epi, const mv_args &a, int g, hipStream_t s) {
    switch (ks) {
        case 1: return dispatch_pro<WT, 1>(pro, epi, a, g, s);
        case 2: return dispatch_pro<WT, 2>(pro, epi, a, g, s);
        case 4: return dispatch_pro<WT, 4>(pro, epi, a, g, s);
        case 8: return dispatch_pro<WT, 8>(pro, epi, a, g, s);
    }
    set_error("matvec: unsupported KS");
    return -1;
}

}  // namespace

size_t matvec_lds_bytes(int wtype, int ks, int64_t n_bt, int64_t seg) {
    return wtype == T_Q4_0 ? make_lds_map<T_Q4_0>(ks, n_bt, seg).total : make_lds_map<T_Q8_0>(ks, n_bt, seg).total;
}

int launch_matvec(int wtype, int ks, int pro, int epi, const mv_args &a, int grid_x, hipStream_t s) {
    if (a.n_rt <= 0 || a.n_bt <= 0) return 0;
    if (grid_x <= 0) {
        set_error("matvec: grid_x <= 0");
        return -1;
    }
    int r = -1;
    if (wtype == T_Q4_0) r = dispatch_ks<T_Q4_0>(ks, pro, epi, a, grid_x, s);
    else if (wtype == T_Q8_0) r = dispatch_ks<T_Q8_0>(ks, pro, epi, a, grid_x, s);
    else set_error("matvec: unsupported weight type");
    if (r != 0 && last_error().empty()) set_error("matvec: bad (ks, pro, epi) combination");
    return r;
}

}  // namespace ghip
