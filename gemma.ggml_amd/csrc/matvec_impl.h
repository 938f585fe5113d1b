// matvec_impl.h — the decode hot path: fused Q4_0/Q8_0 dequant x Q8_0-activation matvec for gfx950.
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
// DESIGN.md §HBM layout) through a U-deep register ring that is filled BEFORE the activation
// prologue, so the first HBM round trip overlaps the (per-workgroup) RMSNorm + quantization of
// the activation into LDS.  A wave streams its tiles continuously across row-tile boundaries.
// K-split (KS > 1): the waves of a workgroup each take a contiguous K segment of the same 8 rows;
// waves 1..KS-1 stash their exact (d, isum) terms in LDS and the fma chain is carried across the
// segments in order (wave w continues wave w-1's accumulator), which keeps the AVX2 order.
#pragma once

#include "device_util.h"
#include "kernels.h"

namespace ghip {
namespace {

typedef uint32_t v4u_nt __attribute__((ext_vector_type(4)));
typedef uint32_t v2u_nt __attribute__((ext_vector_type(2)));
#ifndef GHIP_MV_NT
#define GHIP_MV_NT 1  // weight loads non-temporal (0: plain loads, an A/B switch)
#endif
__device__ __forceinline__ uint4 ld_nt16(const uint8_t *p) {
    if constexpr (!GHIP_MV_NT) return *(const uint4 *)p;
    const v4u_nt v = __builtin_nontemporal_load((const v4u_nt *)p);
    return make_uint4(v.x, v.y, v.z, v.w);
}
__device__ __forceinline__ uint2 ld_nt8(const uint8_t *p) {
    if constexpr (!GHIP_MV_NT) return *(const uint2 *)p;
    const v2u_nt v = __builtin_nontemporal_load((const v2u_nt *)p);
    return make_uint2(v.x, v.y);
}
#ifndef GHIP_MV_SCNT
#define GHIP_MV_SCNT 1  // the scale loads' policy on its own (0: plain, an A/B switch)
#endif
__device__ __forceinline__ uint4 ld_sc16(const uint8_t *p) {
    if constexpr (!GHIP_MV_SCNT) return *(const uint4 *)p;
    return ld_nt16(p);
}
__device__ __forceinline__ uint2 ld_sc8(const uint8_t *p) {
    if constexpr (!GHIP_MV_SCNT) return *(const uint2 *)p;
    return ld_nt8(p);
}

__device__ __forceinline__ int sdot4(uint32_t a, uint32_t b, int c) {
    return __builtin_amdgcn_sdot4((int)a, (int)b, c, false);
}

// ---- LDS image --------------------------------------------------------------------------------
// act: uint4 [nb_pad/4][8 lanes] = {a_b, a_b+1, a_b+2, a_b+3} (4 int8 of lane l per block)
// ns:  uint4 [nb_pad/4][8 lanes] = -8*sum(a) per (block, lane) (Q4_0 only, when NSA; otherwise
//      recomputed with one more v_dot4 to save LDS)
// da:  float [nb_pad] (fp32 of the fp16 activation scale)
// stash (KS > 1): s [64 lanes][SBP], d float [8 rows][SBPD]; a lane's (or row's) segments
//      1..KS-1 are contiguous, so the carry chain reads one linear run (SBP = (KS-1)*seg + pad).
//      s is int16 for Q4_0 (|sum of 4 (nib-8)*a| <= 4*8*127 = 4064: exact, half the LDS and half
//      the carrier's reads) and fp32 for Q8_0 (|sum| up to 4*127*128 needs 17 bits)
constexpr int STASH_PAD = 4;
struct lds_map {
    size_t act, ns, da, stash_s, stash_d, red, ybuf, total;
    int sbp, sbpd;  // s stride in elements (int16 or float), d stride in floats
};
template <int WT, bool NSA>
__host__ __device__ inline lds_map make_lds_map(int ks, int64_t n_bt, int64_t seg_tiles, int64_t ygroups = 0) {
    constexpr int BT = wfmt<WT>::BT;
    lds_map m;
    const size_t nb_pad = (size_t)n_bt * BT;
    m.act = 0;
    size_t off = nb_pad / 4 * 8 * 16;
    m.ns = off;
    if (WT == T_Q4_0 && NSA) off += nb_pad / 4 * 8 * 16;
    m.da = off;
    off += nb_pad * 4;
    off = (off + 15) & ~(size_t)15;
    constexpr int SW = WT == T_Q4_0 ? 2 : 4;  // bytes per stashed s
    m.sbp = ks > 1 ? (int)((ks - 1) * seg_tiles * BT) + STASH_PAD * 4 / SW : 0;
    m.sbpd = ks > 1 ? (int)((ks - 1) * seg_tiles * BT) + STASH_PAD : 0;
    m.stash_s = off;
    off += (size_t)64 * m.sbp * SW;
    m.stash_d = off;
    off += (size_t)8 * m.sbpd * 4;
    m.red = off;
    off += 64 * 8;
    m.ybuf = off;  // EPI_GELU_MUL image output: 32 values per row-tile group of this workgroup
    off += (size_t)ygroups * 32 * 4;
    m.total = off;
    return m;
}

// ---- prologue: build the Q8_0 activation image in LDS (quantize_row_q8_0) ------
// A quad of threads owns one block: thread q holds elements 8q..8q+7 (= AVX2 lanes 2q, 2q+1).
// amax = max|v|; d = amax/127 (fp16 RNE); id = amax ? 127/amax : 0; q = rint(v*id) — identical
// to oracle orc_quantize_row_q8_0.
template <int WT, bool NSA>
__device__ __forceinline__ void put_quad(uint8_t *smem, const lds_map &m, int64_t b, int q, const float v[8]) {
    image_put_quad((uint32_t *)(smem + m.act), (WT == T_Q4_0 && NSA) ? (uint32_t *)(smem + m.ns) : nullptr,
                   (float *)(smem + m.da), b, q, v);
}

template <int WT, bool NSA>
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
        const int64_t idx = ((b >> 2) * 8 + l) * 4 + (b & 3);
        act[idx] = packed;
        if (WT == T_Q4_0 && NSA) ((uint32_t *)(smem + m.ns))[idx] = (uint32_t)(-8 * (q[0] + q[1] + q[2] + q[3]));
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
__device__ __forceinline__ void load8(const mv_args &a, const float *x, int64_t tok, int64_t i0, float v[8]) {
    if (PRO == PRO_EMBED) {
#pragma unroll
        for (int j = 0; j < 8; ++j) {
            const int64_t i = i0 + j;
            // ggml_get_rows then ggml_scale (src/gemma_model.cpp:677-679)
            v[j] = emb_value<WT>(a.emb_qs, a.emb_sc, a.emb_n_bt, tok, i >> 5, (int)(i & 31)) * a.emb_scale;
        }
    } else {
        const float4 u = *(const float4 *)(x + i0), w = *(const float4 *)(x + i0 + 4);
        v[0] = u.x; v[1] = u.y; v[2] = u.z; v[3] = u.w; v[4] = w.x; v[5] = w.y; v[6] = w.z; v[7] = w.w;
    }
}

// Activation values for the first R blocks of each quad, loaded into registers BEFORE the weight
// ring is filled (vmcnt retires in issue order: loads issued after the ring would wait for it).
template <int R>
struct act_regs {
    float x[R][8];
    float w[R][8];
};

// PRO_IMG: the image is nb*2 uint4 of act then nb/4 uint4 of da; thread t holds items t + i*nth
// (i < 2R) in the act_regs storage, loaded before the weight ring
__device__ __forceinline__ const uint4 *img_item(const mv_args &a, int64_t i) {
    const int64_t n_act = a.nb * 2;
    return i < n_act ? (const uint4 *)a.x + i : (const uint4 *)a.x_da + (i - n_act);
}

// NTH: the launch's thread count as a constant.  blockDim.x would be read from the implicit kernel
// arguments with a global load the prologue then waits for (one HBM round trip, ~1 us, before the
// first weight load could issue).
template <int WT, int PRO, int R, int NTH>
__device__ __forceinline__ void prefetch_activation(const mv_args &a, int col, act_regs<R> &r) {
    if (PRO == PRO_IMG) {
        const int64_t T = a.nb * 2 + a.nb / 4;
        const int tid = threadIdx.x, nth = NTH;
#pragma unroll
        for (int i = 0; i < 2 * R; ++i) {
            int64_t it = tid + (int64_t)i * nth;
            it = it < T ? it : T - 1;  // clamp instead of branching around the load
            const uint4 v = *img_item(a, it);
            float *dst = (i & 1) ? &r.w[i >> 1][0] : &r.x[i >> 1][0];
            dst[0] = __builtin_bit_cast(float, v.x); dst[1] = __builtin_bit_cast(float, v.y);
            dst[2] = __builtin_bit_cast(float, v.z); dst[3] = __builtin_bit_cast(float, v.w);
        }
        return;
    }
    if (PRO != PRO_F32 && PRO != PRO_NORM) return;
    const int tid = threadIdx.x, q = tid & 3, nquads = NTH >> 2;
    const float *x = (const float *)((const uint8_t *)a.x + (int64_t)col * a.x_col_stride);
#pragma unroll
    for (int i = 0; i < R; ++i) {
        const int64_t b = (tid >> 2) + (int64_t)i * nquads;
        const int64_t bb = b < a.nb ? b : 0;  // clamp instead of branching around the load
        load8<WT, PRO_F32>(a, x, 0, bb * 32 + q * 8, r.x[i]);
        if (PRO == PRO_NORM) {
            const float4 w0 = *(const float4 *)(a.norm_w + bb * 32 + q * 8);
            const float4 w1 = *(const float4 *)(a.norm_w + bb * 32 + q * 8 + 4);
            r.w[i][0] = w0.x; r.w[i][1] = w0.y; r.w[i][2] = w0.z; r.w[i][3] = w0.w;
            r.w[i][4] = w1.x; r.w[i][5] = w1.y; r.w[i][6] = w1.z; r.w[i][7] = w1.w;
        }
    }
}

#ifndef GHIP_MV_NORM_DPP
#define GHIP_MV_NORM_DPP 1
#endif
// The rms_norm's tree sum and mean (PRO_NORM / PRO_EMBED), kept for finish_activation's check.
struct norm_state {
    double q = 0.0;  // T/n: float(q) is the mean
};

// element values of the activation and the image writer shared by build_ and finish_activation
template <int WT, int PRO, int R, bool NSA, int NTH>
struct act_src {
    const mv_args &a;
    const act_regs<R> &r;
    const float *x;
    int64_t tok = 0;
    int q;
    __device__ act_src(const mv_args &a_, int col, const act_regs<R> &r_) : a(a_), r(r_) {
        x = (const float *)((const uint8_t *)a.x + (int64_t)col * a.x_col_stride);
        if (PRO == PRO_EMBED) tok = ((const int *)a.x)[*a.tok_pos];
        q = threadIdx.x & 3;
    }
    // value of block (tid>>2) + i*nquads: from registers when cached, else loaded now (RELOAD: always
    // loaded, so the registers are dead past the first image)
    template <bool RELOAD = false>
    __device__ __forceinline__ void get(int i, int64_t b, float v[8]) const {
        constexpr bool CACHED = (PRO == PRO_F32 || PRO == PRO_NORM) && !RELOAD;
        if (CACHED && i < R) {
#pragma unroll
            for (int j = 0; j < 8; ++j) v[j] = r.x[i < R ? i : 0][j];
        } else {
            load8<WT, PRO>(a, x, tok, b * 32 + q * 8, v);
        }
    }
    // the image of rms_norm(x)*norm_w (PRO_NORM / PRO_EMBED, scale sc) or of x (PRO_F32)
    template <bool RELOAD = false>
    __device__ void emit(uint8_t *smem, const lds_map &m, float sc) const {
        const int nquads = NTH >> 2;
        int i = 0;
        for (int64_t b = threadIdx.x >> 2; b < a.nb; b += nquads, ++i) {
            float v[8];
            get<RELOAD>(i, b, v);
            if (PRO == PRO_NORM || PRO == PRO_EMBED) {
                float wv[8];
                if (PRO == PRO_NORM && i < R && !RELOAD) {
#pragma unroll
                    for (int j = 0; j < 8; ++j) wv[j] = r.w[i < R ? i : 0][j];
                } else {
                    const float4 w0 = *(const float4 *)(a.norm_w + b * 32 + q * 8);
                    const float4 w1 = *(const float4 *)(a.norm_w + b * 32 + q * 8 + 4);
                    wv[0] = w0.x; wv[1] = w0.y; wv[2] = w0.z; wv[3] = w0.w;
                    wv[4] = w1.x; wv[5] = w1.y; wv[6] = w1.z; wv[7] = w1.w;
                }
#pragma unroll
                for (int j = 0; j < 8; ++j) {
                    const float t = v[j] * sc;  // rms_norm output
                    v[j] = t * wv[j];           // ggml_mul by the norm weight
                }
            }
            put_quad<WT, NSA>(smem, m, b, q, v);
        }
    }
};

template <int WT, int PRO, int R, bool NSA, int NTH>
__device__ norm_state build_activation(const mv_args &a, int col, uint8_t *smem, const lds_map &m, const act_regs<R> &r) {
    constexpr int BT = wfmt<WT>::BT;
    const int tid = threadIdx.x, nth = NTH;
    const int64_t nb = a.nb, nb_pad = a.n_bt * BT;
    const int q = tid & 3;
    const int nquads = nth >> 2;
    norm_state ns;
    // padded tail blocks: zero (d = 0 makes every chain step an exact no-op)
    for (int64_t b = nb + (tid >> 2); b < nb_pad; b += nquads) {
        float z[8] = {0, 0, 0, 0, 0, 0, 0, 0};
        put_quad<WT, NSA>(smem, m, b, q, z);
    }
    if (PRO == PRO_Q8) {
        const block_q8_0 *xb = (const block_q8_0 *)((const uint8_t *)a.x + (int64_t)col * a.x_col_stride);
        for (int64_t b = tid; b < nb; b += nth) put_block_q8<WT, NSA>(smem, m, b, xb + b);
        return ns;
    }
    if (PRO == PRO_IMG) {
        const int64_t n_act = nb * 2, T = n_act + nb / 4;
        auto put = [&](int64_t it, uint4 v) {
            if (it < n_act) {
                ((uint4 *)(smem + m.act))[it] = v;
                if (WT == T_Q4_0 && NSA)  // -8 * sum of the 4 int8 of each dword, exact
                    ((uint4 *)(smem + m.ns))[it] = make_uint4((uint32_t)sdot4(v.x, 0xF8F8F8F8u, 0),
                                                              (uint32_t)sdot4(v.y, 0xF8F8F8F8u, 0),
                                                              (uint32_t)sdot4(v.z, 0xF8F8F8F8u, 0),
                                                              (uint32_t)sdot4(v.w, 0xF8F8F8F8u, 0));
            } else {
                ((uint4 *)(smem + m.da))[it - n_act] = v;
            }
        };
#pragma unroll
        for (int i = 0; i < 2 * R; ++i) {
            const int64_t it = tid + (int64_t)i * nth;
            const float *src = (i & 1) ? &r.w[i >> 1][0] : &r.x[i >> 1][0];
            if (it < T)
                put(it, make_uint4(__builtin_bit_cast(uint32_t, src[0]), __builtin_bit_cast(uint32_t, src[1]),
                                   __builtin_bit_cast(uint32_t, src[2]), __builtin_bit_cast(uint32_t, src[3])));
        }
        for (int64_t it = tid + (int64_t)2 * R * nth; it < T; it += nth) put(it, *img_item(a, it));  // long K
        return ns;
    }
    const act_src<WT, PRO, R, NSA, NTH> src(a, col, r);
    float scale = 1.0f;
    if (PRO == PRO_NORM || PRO == PRO_EMBED) {
        // rms_norm: double sum of fp32 squares in a fixed tree.  Its mean is checked
        // against ggml's sequential sum by finish_activation, which rebuilds the image from the
        // sequential sum in the rare case the check fails
        double part = 0.0;
        int i = 0;
        for (int64_t b = tid >> 2; b < nb; b += nquads, ++i) {
            float v[8];
            src.get(i, b, v);
#pragma unroll
            for (int j = 0; j < 8; ++j) {
                const float sq = v[j] * v[j];
                part += (double)sq;
            }
            if (PRO == PRO_EMBED && a.emb_out && blockIdx.x == 0 && col == 0) {
                *(float4 *)(a.emb_out + b * 32 + q * 8) = make_float4(v[0], v[1], v[2], v[3]);
                *(float4 *)(a.emb_out + b * 32 + q * 8 + 4) = make_float4(v[4], v[5], v[6], v[7]);
            }
        }
        double *red = (double *)(smem + m.red);
#if GHIP_MV_NORM_DPP
        part = wave_sum_f64(part);  // DPP + v_readlane: no ds_bpermute round trips (any order: §3)
#else
#pragma unroll
        for (int off = 32; off >= 1; off >>= 1) part += __shfl_xor(part, off);  // (once per launch)
#endif
        if ((tid & 63) == 0) red[tid >> 6] = part;
        __syncthreads();
        double sum = 0.0;
        for (int w = 0; w < nth / 64; ++w) sum += red[w];
        ns.q = div_by_n(sum, nb * 32);
        scale = 1.0f / sqrtf((float)ns.q + a.eps);
    }
    src.emit(smem, m, scale);
    return ns;
}

// The norm's check (rms_mean_certain: a few integer ops on T/n's bits, after the image is
// built), before the caller issues the rest of its weight ring (the fallback's registers beside a full
// ring cost occupancy and spills).  Workgroup-uniform; in the rare failing case ggml's sequential sum
// (seq_sumsq_wave, every wave) and the image rebuilt.
template <int WT, int PRO, int R, bool NSA, int NTH>
__device__ __forceinline__ void finish_activation(const mv_args &a, int col, uint8_t *smem, const lds_map &m,
                                                  const act_regs<R> &r, const norm_state &ns) {
    if (PRO != PRO_NORM && PRO != PRO_EMBED) return;
#ifdef GHIP_NO_NORM_CHECK  // A/B builds only (scripts/build_variant.sh): the check's cost
    return;
#endif
    const int64_t n = a.nb * 32;
    if (__builtin_expect(rms_mean_certain(ns.q, n), 1)) return;  // the fallback placed out of line
    const act_src<WT, PRO, R, NSA, NTH> src(a, col, r);
    const float mean = (float)(seq_sumsq_wave(n, [&](int64_t i0, float v[8]) { load8<WT, PRO>(a, src.x, src.tok, i0, v); }) /
                               (double)n);
    src.template emit<true>(smem, m, 1.0f / sqrtf(mean + a.eps));  // reloads x and w: the prologue's
}                                                                  // registers are dead here

// ---- one 8-row x BT-block tile for this thread's (row rr, lane l) ----------------------------
// d = f32(dw) * da with the fp16 operand converted inside v_fma_mix_f32 (addend +0: the sign of a
// zero d never reaches the result, since fmaf(+-0, s, acc) == acc for the accumulators here).
__device__ __forceinline__ float mix_lo(uint32_t h2, float y) {
    float d;
    asm("v_fma_mix_f32 %0, %1, %2, 0 op_sel_hi:[1,0,0]" : "=v"(d) : "v"(h2), "v"(y));
    return d;
}
__device__ __forceinline__ float mix_hi(uint32_t h2, float y) {
    float d;
    asm("v_fma_mix_f32 %0, %1, %2, 0 op_sel:[1,0,0] op_sel_hi:[1,0,0]" : "=v"(d) : "v"(h2), "v"(y));
    return d;
}

// One block tile's activation operands (LDS), loaded once and applied to every weight tile of
// that block tile the wave holds (gate and up of EPI_GELU_MUL): each ds_read_b128 moves 1 KiB
// through the LDS pipe even when broadcast, so sharing the operands halves the LDS traffic.
template <int WT> struct act_tile;
template <> struct act_tile<T_Q4_0> { uint32_t av[8], nv[8]; float dav[8]; };
template <> struct act_tile<T_Q8_0> { uint32_t av[4]; float dav[4]; };

template <int WT, bool NSA>
__device__ __forceinline__ act_tile<WT> load_act(const uint8_t *smem, const lds_map &m, int64_t bt, int l) {
    act_tile<WT> t;
    const float *da = (const float *)(smem + m.da);
    const uint4 *act = (const uint4 *)(smem + m.act);
    if constexpr (WT == T_Q4_0) {
        const uint4 A0 = act[(bt * 2) * 8 + l], A1 = act[(bt * 2 + 1) * 8 + l];
        t.av[0] = A0.x; t.av[1] = A0.y; t.av[2] = A0.z; t.av[3] = A0.w;
        t.av[4] = A1.x; t.av[5] = A1.y; t.av[6] = A1.z; t.av[7] = A1.w;
        if (NSA) {
            const uint4 *ns = (const uint4 *)(smem + m.ns);
            const uint4 N0 = ns[(bt * 2) * 8 + l], N1 = ns[(bt * 2 + 1) * 8 + l];
            t.nv[0] = N0.x; t.nv[1] = N0.y; t.nv[2] = N0.z; t.nv[3] = N0.w;
            t.nv[4] = N1.x; t.nv[5] = N1.y; t.nv[6] = N1.z; t.nv[7] = N1.w;
        } else {
#pragma unroll
            for (int j = 0; j < 8; ++j) t.nv[j] = (uint32_t)sdot4(t.av[j], 0xF8F8F8F8u, 0);
        }
        const float4 DA0 = *(const float4 *)(da + bt * 8), DA1 = *(const float4 *)(da + bt * 8 + 4);
        t.dav[0] = DA0.x; t.dav[1] = DA0.y; t.dav[2] = DA0.z; t.dav[3] = DA0.w;
        t.dav[4] = DA1.x; t.dav[5] = DA1.y; t.dav[6] = DA1.z; t.dav[7] = DA1.w;
    } else {
        const uint4 A = act[bt * 8 + l];
        t.av[0] = A.x; t.av[1] = A.y; t.av[2] = A.z; t.av[3] = A.w;
        const float4 DA = *(const float4 *)(da + bt * 4);
        t.dav[0] = DA.x; t.dav[1] = DA.y; t.dav[2] = DA.z; t.dav[3] = DA.w;
    }
    return t;
}

// the same arithmetic as tile_dot<WT, false, NSA>, on preloaded operands
template <int WT>
__device__ __forceinline__ float tile_dot_a(uint4 q, uint4 scv, const act_tile<WT> &t, float acc) {
    const uint32_t qv[4] = {q.x, q.y, q.z, q.w};
    if constexpr (WT == T_Q4_0) {
        const uint32_t sv[4] = {scv.x, scv.y, scv.z, scv.w};
#pragma unroll
        for (int p = 0; p < 4; ++p) {
            const uint32_t lo = qv[p] & 0x0F0F0F0Fu, hi = (qv[p] >> 4) & 0x0F0F0F0Fu;
            const int s0 = sdot4(lo, t.av[2 * p], (int)t.nv[2 * p]);
            const int s1 = sdot4(hi, t.av[2 * p + 1], (int)t.nv[2 * p + 1]);
            const float d0 = mix_lo(sv[p], t.dav[2 * p]);
            const float d1 = mix_hi(sv[p], t.dav[2 * p + 1]);
            acc = __builtin_fmaf(d0, (float)s0, acc);
            acc = __builtin_fmaf(d1, (float)s1, acc);
        }
    } else {
        const uint32_t sv[2] = {scv.x, scv.y};
#pragma unroll
        for (int p = 0; p < 4; ++p) {
            const int s = sdot4(qv[p], t.av[p], 0);
            const float d = (p & 1) ? mix_hi(sv[p >> 1], t.dav[p]) : mix_lo(sv[p >> 1], t.dav[p]);
            acc = __builtin_fmaf(d, (float)s, acc);
        }
    }
    return acc;
}

// STASH: store the exact (d, (float)isum) terms for the carry instead of accumulating
template <int WT, bool STASH, bool NSA>
__device__ __forceinline__ float tile_dot(uint4 q, uint4 scv, const uint8_t *smem, const lds_map &m, int64_t bt, int l,
                                          float acc, void *st_s_, float *st_d, int j0) {
    float *st_s = (float *)st_s_;
    const float *da = (const float *)(smem + m.da);
    const uint4 *act = (const uint4 *)(smem + m.act);
    const uint32_t qv[4] = {q.x, q.y, q.z, q.w};
    if (WT == T_Q4_0) {
        const uint4 A0 = act[(bt * 2) * 8 + l], A1 = act[(bt * 2 + 1) * 8 + l];
        const uint32_t av[8] = {A0.x, A0.y, A0.z, A0.w, A1.x, A1.y, A1.z, A1.w};
        uint32_t nv[8];
        if (NSA) {
            const uint4 *ns = (const uint4 *)(smem + m.ns);
            const uint4 N0 = ns[(bt * 2) * 8 + l], N1 = ns[(bt * 2 + 1) * 8 + l];
            nv[0] = N0.x; nv[1] = N0.y; nv[2] = N0.z; nv[3] = N0.w; nv[4] = N1.x; nv[5] = N1.y; nv[6] = N1.z; nv[7] = N1.w;
        }
        const float4 DA0 = *(const float4 *)(da + bt * 8), DA1 = *(const float4 *)(da + bt * 8 + 4);
        const float dav[8] = {DA0.x, DA0.y, DA0.z, DA0.w, DA1.x, DA1.y, DA1.z, DA1.w};
        const uint32_t sv[4] = {scv.x, scv.y, scv.z, scv.w};
        uint32_t pk[4];
        float dk[8];
#pragma unroll
        for (int p = 0; p < 4; ++p) {
            const uint32_t lo = qv[p] & 0x0F0F0F0Fu, hi = (qv[p] >> 4) & 0x0F0F0F0Fu;
            // sum((nib - 8) * a) = sum(nib * a) - 8 * sum(a), exact in int32
            const int n0 = NSA ? (int)nv[2 * p] : sdot4(av[2 * p], 0xF8F8F8F8u, 0);
            const int n1 = NSA ? (int)nv[2 * p + 1] : sdot4(av[2 * p + 1], 0xF8F8F8F8u, 0);
            const int s0 = sdot4(lo, av[2 * p], n0);
            const int s1 = sdot4(hi, av[2 * p + 1], n1);
            const float d0 = mix_lo(sv[p], dav[2 * p]);
            const float d1 = mix_hi(sv[p], dav[2 * p + 1]);
            if (STASH) {
                pk[p] = ((uint32_t)s0 & 0xFFFFu) | ((uint32_t)s1 << 16);
                dk[2 * p] = d0;
                dk[2 * p + 1] = d1;
            } else {
                acc = __builtin_fmaf(d0, (float)s0, acc);
                acc = __builtin_fmaf(d1, (float)s1, acc);
            }
        }
        if (STASH) {
            *(uint4 *)((int16_t *)st_s_ + j0) = make_uint4(pk[0], pk[1], pk[2], pk[3]);
            if (l == 0) {
                *(float4 *)(st_d + j0) = make_float4(dk[0], dk[1], dk[2], dk[3]);
                *(float4 *)(st_d + j0 + 4) = make_float4(dk[4], dk[5], dk[6], dk[7]);
            }
        }
    } else {
        const uint4 A = act[bt * 8 + l];
        const uint32_t av[4] = {A.x, A.y, A.z, A.w};
        const float4 DA = *(const float4 *)(da + bt * 4);
        const float dav[4] = {DA.x, DA.y, DA.z, DA.w};
        const uint32_t sv[2] = {scv.x, scv.y};
        float dd[4], ss[4];
#pragma unroll
        for (int p = 0; p < 4; ++p) {
            const int s = sdot4(qv[p], av[p], 0);
            const float d = (p & 1) ? mix_hi(sv[p >> 1], dav[p]) : mix_lo(sv[p >> 1], dav[p]);
            dd[p] = d;
            ss[p] = (float)s;
            if (!STASH) acc = __builtin_fmaf(d, (float)s, acc);
        }
        if (STASH) {
            *(float4 *)(st_s + j0) = make_float4(ss[0], ss[1], ss[2], ss[3]);
            if (l == 0) *(float4 *)(st_d + j0) = make_float4(dd[0], dd[1], dd[2], dd[3]);
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

// ordered fold of the 8 lanes (hsum_float_8): xor 4, then 2, then 1
__device__ __forceinline__ float fold8(float v) {
    return fold8_dpp(v);
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
    if (EPI == EPI_GELU_MUL) y[row] = gelu_tab(a, v) * vb;  // gelu(gate) then ggml_mul by up
    if (EPI == EPI_ARGMAX) {
        y[row] = v;
        const unsigned long long k = argmax_key(v, row);
        best = k > best ? k : best;
    }
}

// ---- the tile stream: a wave's sequence of (matrix, row tile, block tile) items ----------------
// item k -> row tile rt0 + (k / per_rt) * rstride; within it matrix (k % per_rt) / nbt and block
// tile bt0 + (k % per_rt) % nbt.  Cursors advance incrementally (no divisions in the loop).
struct cursor {
    int64_t rt;
    int m;
    int bt;
};

// Ordered carry (wave 0): acc continues through the stashed (d, isum) terms of segments 1..KS-1 in
// block order — the exact fmaf chain of the sequential loop.  The run is linear in LDS (stash
// layout above) and read AHEAD chunks of 4 blocks ahead of the FMAs, so the chain runs at FMA
// latency, not LDS latency.  Reads are never inside a branch: past the end the index is clamped.
template <int G, bool EXACT>
__device__ __forceinline__ float carry_run(const float4 *ps, const float4 *pd, int total, float acc) {
    float4 as[G], ad[G], bs[G], bd[G];
    auto load = [&](float4 (&S)[G], float4 (&D)[G], int c0) {
#pragma unroll
        for (int r = 0; r < G; ++r) {
            const int i = EXACT ? c0 + r : (c0 + r < total - 1 ? c0 + r : total - 1);
            S[r] = ps[i];
            D[r] = pd[i];
        }
    };
    auto chain = [&](const float4 (&S)[G], const float4 (&D)[G], int c0) {
#pragma unroll
        for (int r = 0; r < G; ++r) {
            if (EXACT || c0 + r < total) {
                acc = __builtin_fmaf(D[r].x, S[r].x, acc);
                acc = __builtin_fmaf(D[r].y, S[r].y, acc);
                acc = __builtin_fmaf(D[r].z, S[r].z, acc);
                acc = __builtin_fmaf(D[r].w, S[r].w, acc);
            }
        }
    };
    load(as, ad, 0);
    load(bs, bd, G);
    for (int c = 0; c < total; c += 2 * G) {
        // the empty asm statements pin each set's reads one half-step ahead of their FMAs
        asm volatile("" ::: "memory");
        chain(as, ad, c);
        asm volatile("" ::: "memory");
        if (!EXACT || c + 2 * G < total) load(as, ad, c + 2 * G);
        asm volatile("" ::: "memory");
        chain(bs, bd, c + G);
        asm volatile("" ::: "memory");
        if (!EXACT || c + 3 * G < total) load(bs, bd, c + 3 * G);
    }
    return acc;
}

// Q4_0 form: chunks of 8 blocks = one b128 of int16 sums + two b128 of d.  total % (2G) == 0; the
// reloads are unconditional (a set is refilled in place right after its FMAs, so the register
// allocator needs no copies and the waitcnt before a set's FMAs only covers that set).  The final
// reloads run up to 2G chunks past the run: they stay inside the LDS image (the stash pads and the
// regions behind it) and are never used.
template <int G>
__device__ __forceinline__ float carry_run16(const uint4 *ps, const float4 *pd, int total, float acc) {
    uint4 as[G], bs[G];
    float4 ad[G][2], bd[G][2];
    auto load = [&](uint4 (&S)[G], float4 (&D)[G][2], int c0) {
#pragma unroll
        for (int r = 0; r < G; ++r) {
            S[r] = ps[c0 + r];
            D[r][0] = pd[2 * (c0 + r)];
            D[r][1] = pd[2 * (c0 + r) + 1];
        }
    };
    auto chain = [&](const uint4 (&S)[G], const float4 (&D)[G][2]) {
#pragma unroll
        for (int r = 0; r < G; ++r) {
            const uint32_t w[4] = {S[r].x, S[r].y, S[r].z, S[r].w};
            const float d[8] = {D[r][0].x, D[r][0].y, D[r][0].z, D[r][0].w,
                                D[r][1].x, D[r][1].y, D[r][1].z, D[r][1].w};
#pragma unroll
            for (int k = 0; k < 4; ++k) {
                acc = __builtin_fmaf(d[2 * k], (float)(int)(int16_t)(w[k] & 0xFFFFu), acc);
                acc = __builtin_fmaf(d[2 * k + 1], (float)((int)w[k] >> 16), acc);
            }
        }
    };
    load(as, ad, 0);
    load(bs, bd, G);
    for (int c = 0; c < total; c += 2 * G) {
        asm volatile("" ::: "memory");
        chain(as, ad);
        asm volatile("" ::: "memory");
        load(as, ad, c + 2 * G);
        asm volatile("" ::: "memory");
        chain(bs, bd);
        asm volatile("" ::: "memory");
        load(bs, bd, c + 3 * G);
    }
    return acc;
}

// Explicitly pipelined carry: NS = 4 chunk sets in flight.  Each set is refilled in place right
// after its FMAs, and sched_barrier(0) pins every load group and FMA group where it is written, so
// the scheduler can neither sink a refill next to its use nor hoist it above the FMAs that still
// read the set (the compiler's own waitcnt insertion then waits, before a set's FMAs, only for that
// set: LDS ops retire in order).  The ring over-reads up to NS chunks past the run (inside the LDS
// image: stash pads, the d stash, the red area); those values are never used.
template <bool I16>
struct carry_set {
    uint4 s;
    float4 d0, d1;
};
template <bool I16>
__device__ __forceinline__ void carry_load(carry_set<I16> &k, const uint4 *ps, const float4 *pd, int c) {
    k.s = ps[c];
    if (I16) {
        k.d0 = pd[2 * c];
        k.d1 = pd[2 * c + 1];
    } else {
        k.d0 = pd[c];
    }
}
template <bool I16>
__device__ __forceinline__ float carry_fma(const carry_set<I16> &k, float acc) {
    if (I16) {
        const float d[8] = {k.d0.x, k.d0.y, k.d0.z, k.d0.w, k.d1.x, k.d1.y, k.d1.z, k.d1.w};
        const uint32_t w[4] = {k.s.x, k.s.y, k.s.z, k.s.w};
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            acc = __builtin_fmaf(d[2 * j], (float)(int)(int16_t)(w[j] & 0xFFFFu), acc);
            acc = __builtin_fmaf(d[2 * j + 1], (float)((int)w[j] >> 16), acc);
        }
    } else {
        acc = __builtin_fmaf(k.d0.x, __builtin_bit_cast(float, k.s.x), acc);
        acc = __builtin_fmaf(k.d0.y, __builtin_bit_cast(float, k.s.y), acc);
        acc = __builtin_fmaf(k.d0.z, __builtin_bit_cast(float, k.s.z), acc);
        acc = __builtin_fmaf(k.d0.w, __builtin_bit_cast(float, k.s.w), acc);
    }
    return acc;
}

// chunks [0, total) of the run; total % 4 == 0.  I16 (Q4_0): chunk = 8 blocks (s: 8 x int16 in one
// uint4, d: two float4); else (Q8_0): 4 blocks (s: 4 x f32, d: one float4).
template <bool I16>
__device__ __forceinline__ float carry_ring(const uint4 *ps, const float4 *pd, int total, float acc) {
    carry_set<I16> A, B, C, D;
    carry_load<I16>(A, ps, pd, 0);
    carry_load<I16>(B, ps, pd, 1);
    carry_load<I16>(C, ps, pd, 2);
    carry_load<I16>(D, ps, pd, 3);
    for (int c = 0; c < total; c += 4) {
        __builtin_amdgcn_sched_barrier(0);
        acc = carry_fma<I16>(A, acc);
        __builtin_amdgcn_sched_barrier(0);
        carry_load<I16>(A, ps, pd, c + 4);
        __builtin_amdgcn_sched_barrier(0);
        acc = carry_fma<I16>(B, acc);
        __builtin_amdgcn_sched_barrier(0);
        carry_load<I16>(B, ps, pd, c + 5);
        __builtin_amdgcn_sched_barrier(0);
        acc = carry_fma<I16>(C, acc);
        __builtin_amdgcn_sched_barrier(0);
        carry_load<I16>(C, ps, pd, c + 6);
        __builtin_amdgcn_sched_barrier(0);
        acc = carry_fma<I16>(D, acc);
        __builtin_amdgcn_sched_barrier(0);
        carry_load<I16>(D, ps, pd, c + 7);
    }
    __builtin_amdgcn_sched_barrier(0);
    return acc;
}

// gl = row * 8 + lane-of-row in the wave-0 numbering of the stash
template <int WT, int KS>
__device__ __forceinline__ float carry_chain(const void *st_s, const float *st_d, const lds_map &m, int seg_blocks,
                                             int gl, float acc) {
    const float4 *pd = (const float4 *)(st_d + (size_t)(gl >> 3) * m.sbpd);
    if (WT == T_Q4_0) {
        const uint4 *ps = (const uint4 *)((const int16_t *)st_s + (size_t)gl * m.sbp);
        const int total = (KS - 1) * (seg_blocks >> 3);  // chunks of 8 blocks
        if (total % 4 == 0) return carry_ring<true>(ps, pd, total, acc);
        if (total % 4 == 0) return carry_run16<2>(ps, pd, total, acc);
        if (total % 2 == 0) return carry_run16<1>(ps, pd, total, acc);
        // odd: the last chunk alone, after an even run
        acc = total > 1 ? carry_run16<1>(ps, pd, total - 1, acc) : acc;
        const uint4 S = ps[total - 1];
        const float4 D0 = pd[2 * (total - 1)], D1 = pd[2 * (total - 1) + 1];
        const uint32_t w[4] = {S.x, S.y, S.z, S.w};
        const float d[8] = {D0.x, D0.y, D0.z, D0.w, D1.x, D1.y, D1.z, D1.w};
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            acc = __builtin_fmaf(d[2 * k], (float)(int)(int16_t)(w[k] & 0xFFFFu), acc);
            acc = __builtin_fmaf(d[2 * k + 1], (float)((int)w[k] >> 16), acc);
        }
        return acc;
    }
    const float4 *ps = (const float4 *)((const float *)st_s + (size_t)gl * m.sbp);
    const int total = (KS - 1) * (seg_blocks >> 2);  // chunks of 4 blocks
    if (total % 4 == 0) return carry_ring<false>((const uint4 *)ps, pd, total, acc);
    // whole double-steps: no bounds test inside the dependent chain
    if (total % 8 == 0) return carry_run<4, true>(ps, pd, total, acc);
    if (total % 4 == 0) return carry_run<2, true>(ps, pd, total, acc);
    return carry_run<2, false>(ps, pd, total, acc);
}

#ifndef GHIP_NOSCALE
#define GHIP_NOSCALE 0
#endif
#ifndef GHIP_HOSTDIV
#define GHIP_HOSTDIV 1  // 1: the wave's item count from launch_t's precomputed quotient (no 64-bit division)
#endif
#ifndef GHIP_UPRE
#define GHIP_UPRE 4
#endif
#ifndef GHIP_MV_XFIRST
#define GHIP_MV_XFIRST 1  // decode 1,527-1,529 -> 1,529-1,536 tok/s (4 interleaved reps)
#endif
#ifndef GHIP_SCL
#define GHIP_SCL 1  // gate/up scales as one 1 KiB run per row tile and matrix (k_matvec SCL)
#endif
// ONE_SHOT: every wave's items fit the register ring (n_items <= U): no refills in the stream loop
template <int WT, int KS, int PRO, int EPI, int U, int R, bool NSA, bool ONE_SHOT>
__global__ void __launch_bounds__(512) k_matvec(mv_args a) {
    extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
    constexpr int BT = wfmt<WT>::BT, SB = wfmt<WT>::SCALE_BYTES;
    constexpr int NM = EPI == EPI_GELU_MUL ? 2 : 1;  // matrices per row tile (gate, up)
    // readfirstlane: makes the wave index (and every cursor derived from it) provably uniform, so
    // the stream bookkeeping lives in SGPRs and its branches are scalar (cdna_hip_programming T20)
    constexpr int NTH = KS > 1 ? 64 * KS : 256;  // launch_t's block size
    const int tid = threadIdx.x, lane = tid & 63, wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int rr = lane >> 3, l = lane & 7;
    const int col = blockIdx.y;
    if (GHIP_STAMPS && a.dbg_t && tid == 0) a.dbg_t[((int64_t)blockIdx.y * gridDim.x + blockIdx.x) * 16 + 0] = __builtin_amdgcn_s_memrealtime();
    const int64_t seg_tiles = KS > 1 ? a.n_bt / KS : a.n_bt;
    // EPI_GELU_MUL with an image output: row-tile groups (4 consecutive tiles = one Q8_0 block of y)
    // this workgroup produces, buffered in LDS until the end
    const bool yimg = EPI == EPI_GELU_MUL && KS == 1 && a.out_act != nullptr;
    const int64_t ygroups = !yimg ? 0 : GHIP_HOSTDIV ? a.ygroups : ((a.n_rt >> 2) + gridDim.x - 1) / gridDim.x;
    const lds_map m = make_lds_map<WT, NSA>(KS, a.n_bt, seg_tiles, ygroups);
    const int nbt = (int)seg_tiles;
    const int bt0 = KS > 1 ? wave * nbt : 0;
    // this wave's row tiles
    int64_t rt0, rstride;
    if (KS == 1) {
        constexpr int nw = NTH >> 6;
        rt0 = (int64_t)blockIdx.x * nw + wave;
        rstride = (int64_t)gridDim.x * nw;
    } else {
        rt0 = blockIdx.x;
        rstride = gridDim.x;
    }
    const int64_t n_my_rt = GHIP_HOSTDIV ? a.rt_q + (rt0 < a.rt_r ? 1 : 0)
                                         : rt0 < a.n_rt ? (a.n_rt - rt0 + rstride - 1) / rstride : 0;
    const int64_t n_items = n_my_rt * NM * nbt;

    // SCL (gate/up, every wave at most one row tile whose scale planes are 1 KiB each): the wave's
    // gate and up scales come in with ONE 16-B load per lane per matrix (lane L: bytes 16L.. of the
    // row tile's contiguous scale run) and are read per block tile from a per-wave LDS copy,
    // instead of one 16-B load per (item, lane) that 8 lanes of a row issue redundantly
    constexpr bool SCL = KS == 1 && NM == 2 && ONE_SHOT;
    static_assert(!SCL || 8 * SB * (WT == T_Q4_0 ? 8 : 16) == 1024, "SCL: one 1 KiB scale run per row tile");

    // 0) this thread's activation values (older than the weight loads -> waited for by count)
    act_regs<R> ar;
    prefetch_activation<WT, PRO, R, NTH>(a, col, ar);
    uint4 scl_g = make_uint4(0, 0, 0, 0), scl_u = scl_g;
    if constexpr (SCL) {
        const int64_t rts = n_items ? rt0 : 0;
        scl_g = ld_sc16(a.sc + rts * 1024 + lane * 16);
        scl_u = ld_sc16(a.sc2 + rts * 1024 + lane * 16);
    }
    // GHIP_MV_XFIRST: every wave's activation loads go out before any wave's weight ring (one
    // s_barrier, no wait) — the K-quant prologue's measured +0.5-1 % (kquant.hip GHIP_KQ_EARLY 2)
    if (GHIP_MV_XFIRST && (PRO == PRO_NORM || PRO == PRO_EMBED)) __builtin_amdgcn_s_barrier();

    // 1) fill the register ring: the HBM round trip overlaps the prologue below.  Loads are
    //    never inside a runtime branch (hipcc would wait vmcnt(0) around them): past the last item
    //    the cursor stays put and the same tile is re-read (L2 hit, at most U-1 per wave).  The
    //    tile base is uniform (SGPR pair) and the lane offset 32-bit: global_load v, v_off, s[base].
    uint4 qb[U], sb[U];
    cursor ic{n_items ? rt0 : 0, 0, 0};
    int64_t issued = 0;
    const uint32_t q_off = (uint32_t)lane * 16u, s_off = (uint32_t)rr * SB;
    auto issue = [&](uint4 &qd, uint4 &sd) {
        const bool second = NM == 2 && ic.m;
        const int64_t tile = ic.rt * a.n_bt + bt0 + ic.bt;
        const uint8_t *qt = (second ? a.qs2 : a.qs) + tile * 1024;
        const uint8_t *st = (second ? a.sc2 : a.sc) + tile * 8 * SB;
        // weights are read once per token by one CU: non-temporal loads (MI355X_MICROARCH nt-weights:
        // issued -> landed -18 %, decode layer -5..10 %)
        qd = ld_nt16(qt + q_off);
        if constexpr (SCL) {
            (void)st; (void)sd;
        } else {
#if GHIP_NOSCALE  // timing only: no scale loads (wrong results)
        sd = make_uint4(0x3c003c00u, 0x3c003c00u, 0x3c003c00u, 0x3c003c00u);
        (void)st;
#else
        if (WT == T_Q4_0) {
            sd = ld_sc16(st + s_off);
        } else {
            const uint2 v = ld_sc8(st + s_off);
            sd = make_uint4(v.x, v.y, 0, 0);
        }
#endif
        }
        ++issued;
        if (issued < n_items) {
            if (NM == 2) {  // gate and up of one block tile back to back (shared act operands)
                if (++ic.m == 2) {
                    ic.m = 0;
                    if (++ic.bt == nbt) {
                        ic.bt = 0;
                        ic.rt += rstride;
                    }
                }
            } else if (++ic.bt == nbt) {
                ic.bt = 0;
                if (++ic.m == NM) {
                    ic.m = 0;
                    ic.rt += rstride;
                }
            }
        }
    };
    // UPRE ring slots go out before the prologue, the rest after it: a full ring from every wave at
    // once oversubscribes the CU's load queue and would hold the prologue behind the issue
    constexpr int UP = GHIP_UPRE < U ? GHIP_UPRE : U;
#pragma unroll
    for (int u = 0; u < UP; ++u) issue(qb[u], sb[u]);
    if (GHIP_STAMPS && a.dbg_t && tid == 0) a.dbg_t[((int64_t)blockIdx.y * gridDim.x + blockIdx.x) * 16 + 1] = __builtin_amdgcn_s_memrealtime();

    // 2) activation image in LDS
    norm_state ns;
    if (!(a.ablate & 1)) {  // timing ablations only
        ns = build_activation<WT, PRO, R, NSA, NTH>(a, col, smem, m, ar);
        // the norm's check before the rest of the ring: the fallback's registers would otherwise sit
        // beside the whole ring's (measured: VGPRs 44 -> 74 on the rr kernel, spills on long K)
        finish_activation<WT, PRO, R, NSA, NTH>(a, col, smem, m, ar, ns);
    }
#pragma unroll
    for (int u = UP; u < U; ++u) issue(qb[u], sb[u]);
    if (GHIP_STAMPS && a.dbg_t && tid == 0) a.dbg_t[((int64_t)blockIdx.y * gridDim.x + blockIdx.x) * 16 + 2] = __builtin_amdgcn_s_memrealtime();
    uint8_t *scl_w = smem + m.total + (size_t)wave * 2048;  // SCL: this wave's [gate | up] scale runs
    if constexpr (SCL) {
        *(uint4 *)(scl_w + lane * 16) = scl_g;
        *(uint4 *)(scl_w + 1024 + lane * 16) = scl_u;
    }
    __syncthreads();
    if (GHIP_STAMPS && a.dbg_t && tid == 0) a.dbg_t[((int64_t)blockIdx.y * gridDim.x + blockIdx.x) * 16 + 3] = __builtin_amdgcn_s_memrealtime();

    // 3) stream
    const int seg_blocks = nbt * BT;
    constexpr int SW = WT == T_Q4_0 ? 2 : 4;
    uint8_t *st_s = smem + m.stash_s;
    float *st_d = (float *)(smem + m.stash_d);
    void *my_s = st_s + ((size_t)lane * m.sbp + (size_t)(wave > 0 ? wave - 1 : 0) * nbt * BT) * SW;
    float *my_d = st_d + (size_t)rr * m.sbpd + (size_t)(wave > 0 ? wave - 1 : 0) * nbt * BT;
    unsigned long long best = 0;
    int y_it = 0;  // row tiles this wave has finished (EPI_GELU_MUL image buffer slot)
    cursor cc{rt0, 0, 0};
    float acc = 0.0f, va = 0.0f;
    const int64_t n_pad = ONE_SHOT && !SCL ? U : (n_items + U - 1) / U * U;
    if constexpr (NM == 2) {
        // (gate, up) item pairs of the same block tile; two ordered chains (acc: gate, acc2: up)
        static_assert(KS == 1 && U % 2 == 0, "gate/up pairing");
        float acc2 = 0.0f;
        for (int64_t k = 0; k < n_pad; k += U) {
#pragma unroll
            for (int u = 0; u < U; u += 2) {
                const uint4 q0 = qb[u], q1 = qb[u + 1];
                uint4 s0 = sb[u], s1 = sb[u + 1];
                if constexpr (SCL) {  // block tile cc.bt, row rr: bytes (bt*8 + rr)*SB of each run
                    const uint8_t *sp = scl_w + (cc.bt * 8 + rr) * SB;
                    if constexpr (WT == T_Q4_0) {
                        s0 = *(const uint4 *)sp;
                        s1 = *(const uint4 *)(sp + 1024);
                    } else {
                        const uint2 g2 = *(const uint2 *)sp, u2 = *(const uint2 *)(sp + 1024);
                        s0 = make_uint4(g2.x, g2.y, 0, 0);
                        s1 = make_uint4(u2.x, u2.y, 0, 0);
                    }
                }
                issue(qb[u], sb[u]);
                issue(qb[u + 1], sb[u + 1]);
                if (k + u < n_items) {
                    if (a.ablate & 8) {  // timing only: the loads without the dot products
                        acc += __builtin_bit_cast(float, q0.x ^ s0.x ^ q1.y ^ s1.y);
                    } else {
                        const act_tile<WT> at = load_act<WT, NSA>(smem, m, cc.bt, l);
                        acc = tile_dot_a<WT>(q0, s0, at, acc);
                        acc2 = tile_dot_a<WT>(q1, s1, at, acc2);
                    }
                    if (cc.bt + 1 == nbt) {
                        const float vg = fold8(acc), vu = fold8(acc2);
                        acc = 0.0f;
                        acc2 = 0.0f;
                        if ((lane & 7) == 0) {
                            epilogue<EPI>(a, col, cc.rt * 8 + rr, vg, vu, best);
                            if (yimg) ((float *)(smem + m.ybuf))[y_it * 32 + wave * 8 + rr] = gelu_tab(a, vg) * vu;
                        }
                        ++y_it;
                        cc.bt = 0;
                        cc.rt += rstride;
                    } else {
                        ++cc.bt;
                    }
                }
            }
        }
    } else
    for (int64_t k = 0; k < n_pad; k += U) {
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const uint4 qc = qb[u], scc = sb[u];
            if (!ONE_SHOT) issue(qb[u], sb[u]);
            if (k + u < n_items) {
                const int64_t bt = bt0 + cc.bt;
                if (KS == 1 || wave == 0)
                    acc = tile_dot<WT, false, NSA>(qc, scc, smem, m, bt, l, acc, nullptr, nullptr, 0);
                else
                    tile_dot<WT, true, NSA>(qc, scc, smem, m, bt, l, 0.0f, my_s, my_d, cc.bt * BT);
                if (cc.bt + 1 == nbt) {
                    // end of this wave's part of a (matrix, row tile)
                    if (KS == 1) {
                        const float v = fold8(acc);
                        acc = 0.0f;
                        if (NM == 2 && cc.m == 0) {
                            va = v;
                        } else {
                            if ((lane & 7) == 0) {
                                epilogue<EPI>(a, col, cc.rt * 8 + rr, NM == 2 ? va : v, v, best);
                                if (EPI == EPI_GELU_MUL && yimg)
                                    ((float *)(smem + m.ybuf))[y_it * 32 + wave * 8 + rr] = gelu_tab(a, va) * v;
                            }
                            ++y_it;
                        }
                    } else {
                        // ordered carry: wave 0 hands its accumulators over through LDS, then after ONE
                        // barrier the carrier waves continue the chains of their rows through the
                        // stashed terms of segments 1..KS-1, in block order.  The chain is bound by
                        // the carrier's LDS read issue (2 x b128 per 4 steps), not by the FMA latency
                        // (7.5 clk/step): tests/micro/carry_bench*.hip.
                        float *hand = (float *)(smem + m.red);
                        if (wave == 0) hand[lane] = acc;
                        if (GHIP_STAMPS && a.dbg_t && tid == 0) a.dbg_t[((int64_t)blockIdx.y * gridDim.x + blockIdx.x) * 16 + 6] = __builtin_amdgcn_s_memrealtime();
                        __syncthreads();
                        if (GHIP_STAMPS && a.dbg_t && tid == 0) a.dbg_t[((int64_t)blockIdx.y * gridDim.x + blockIdx.x) * 16 + 7] = __builtin_amdgcn_s_memrealtime();
                        {
                            // one carrier wave: a wave pays ~16-21 clk per ds_read_b128 whatever its
                            // active lanes, so more carriers only add LDS-array contention
                            constexpr int NCAR = 1, RPW = 8 / NCAR;
                            const int gl = wave * RPW * 8 + lane;
                            if (wave < NCAR && lane < RPW * 8) {
                                float c = hand[gl];
                                if (!(a.ablate & 4)) c = carry_chain<WT, KS>(st_s, st_d, m, seg_blocks, gl, c);
                                if (GHIP_STAMPS && a.dbg_t && tid == 0) a.dbg_t[((int64_t)blockIdx.y * gridDim.x + blockIdx.x) * 16 + 8] = __builtin_amdgcn_s_memrealtime();
                                const float v = fold8(c);
                                if ((lane & 7) == 0) epilogue<EPI>(a, col, cc.rt * 8 + (gl >> 3), v, 0.0f, best);
                                if (GHIP_STAMPS && a.dbg_t && tid == 0) a.dbg_t[((int64_t)blockIdx.y * gridDim.x + blockIdx.x) * 16 + 9] = __builtin_amdgcn_s_memrealtime();
                            }
                        }
                        acc = 0.0f;
                        __syncthreads();
                        if (GHIP_STAMPS && a.dbg_t && tid == 0) a.dbg_t[((int64_t)blockIdx.y * gridDim.x + blockIdx.x) * 16 + 10] = __builtin_amdgcn_s_memrealtime();
                    }
                }
                if (++cc.bt == nbt) {
                    cc.bt = 0;
                    if (++cc.m == NM) {
                        cc.m = 0;
                        cc.rt += rstride;
                    }
                }
            }
        }
    }
    if (GHIP_STAMPS && a.dbg_t && tid == 0) a.dbg_t[((int64_t)blockIdx.y * gridDim.x + blockIdx.x) * 16 + 4] = __builtin_amdgcn_s_memrealtime();
    if (EPI == EPI_GELU_MUL && yimg) {
        // y's Q8_0 image: group g = blockIdx.x + k*gridDim.x of 4 row tiles is block g of y
        __syncthreads();
        const int64_t n_groups = a.n_rt >> 2;
        const int64_t mine = blockIdx.x < n_groups ? (n_groups - blockIdx.x + gridDim.x - 1) / gridDim.x : 0;
        for (int64_t t = tid; t < mine * 4; t += NTH) {
            const int64_t k = t >> 2;
            const float *yv = (const float *)(smem + m.ybuf) + k * 32 + (t & 3) * 8;
            float v[8];
#pragma unroll
            for (int j = 0; j < 8; ++j) v[j] = yv[j];
            image_put_quad(a.out_act, nullptr, a.out_da, blockIdx.x + k * gridDim.x, (int)(t & 3), v);
        }
    }
    if (EPI == EPI_ARGMAX) {
#pragma unroll
        for (int off = 32; off >= 1; off >>= 1) {
            const unsigned long long o = __shfl_xor(best, off);
            best = o > best ? o : best;
        }
        // one plain store per workgroup into its own slot (a single-word atomic from every wave
        // serialises at the memory side: MI355X_MICROARCH fan-in row); k_advance reduces the slots
        unsigned long long *red = (unsigned long long *)(smem + m.red);
        __syncthreads();
        if (lane == 0) red[wave] = best;
        __syncthreads();
        if (tid == 0) {
            for (int w = 1; w < NTH / 64; ++w) best = red[w] > best ? red[w] : best;
            a.argmax_key[(int64_t)blockIdx.y * gridDim.x + blockIdx.x] = best;
        }
    }
    if (GHIP_STAMPS && a.dbg_t && tid == 0) a.dbg_t[((int64_t)blockIdx.y * gridDim.x + blockIdx.x) * 16 + 5] = __builtin_amdgcn_s_memrealtime();
}

// gate/up with the two matrices on separate waves (launch_matvec ks = 2, EPI_GELU_MUL): wave w of a
// 512-thread workgroup streams matrix w & 1 (gate, up) of row tile 4*blockIdx.x + (w >> 1)
// (+ k * 4*gridDim.x), each in its own ordered chain exactly as the paired form computes it.  Twice
// the waves with half the items each: at Gemma-2B shapes the register ring holds a wave's whole row
// tile (one-shot), so all of the launch's weight loads are in flight after the prologue.  The two
// chains meet in LDS for gelu(gate)*up and the optional Q8_0 image of y.
template <int WT, int U, bool ONE_SHOT>
__global__ void __launch_bounds__(512) k_matvec_gu2(mv_args a) {
    extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
    constexpr int NTH = 512, SB = wfmt<WT>::SCALE_BYTES;
    constexpr bool NSA = true;
    const int tid = threadIdx.x, lane = tid & 63, wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int rr = lane >> 3, l = lane & 7, mat = wave & 1, pair = wave >> 1;
    const lds_map m = make_lds_map<WT, NSA>(1, a.n_bt, a.n_bt, 0);
    float *vbuf = (float *)(smem + m.ybuf);  // [round][gate | up][32 rows of the 4 row tiles]
    const int nbt = (int)a.n_bt;
    const int64_t rt0 = (int64_t)blockIdx.x * 4 + pair, rstride = (int64_t)gridDim.x * 4;
    const int64_t n_my_rt = a.rt_q + (rt0 < a.rt_r ? 1 : 0);
    const int64_t n_items = n_my_rt * nbt;
    act_regs<1> ar;
    prefetch_activation<WT, PRO_NORM, 1, NTH>(a, 0, ar);
    const uint8_t *qsm = mat ? a.qs2 : a.qs, *scm = mat ? a.sc2 : a.sc;
    uint4 qb[U], sb[U];
    int64_t rt_i = n_items ? rt0 : 0, issued = 0;
    int bt_i = 0;
    const uint32_t q_off = (uint32_t)lane * 16u, s_off = (uint32_t)rr * SB;
    auto issue = [&](uint4 &qd, uint4 &sd) {  // past the last item the cursor stays (L2 re-read)
        const int64_t tile = rt_i * a.n_bt + bt_i;
        qd = ld_nt16(qsm + tile * 1024 + q_off);
        if (WT == T_Q4_0) {
            sd = ld_sc16(scm + tile * 8 * SB + s_off);
        } else {
            const uint2 v = ld_sc8(scm + tile * 8 * SB + s_off);
            sd = make_uint4(v.x, v.y, 0, 0);
        }
        ++issued;
        if (issued < n_items && ++bt_i == nbt) {
            bt_i = 0;
            rt_i += rstride;
        }
    };
    constexpr int UP = GHIP_UPRE < U ? GHIP_UPRE : U;
#pragma unroll
    for (int u = 0; u < UP; ++u) issue(qb[u], sb[u]);
    const norm_state ns = build_activation<WT, PRO_NORM, 1, NSA, NTH>(a, 0, smem, m, ar);
    finish_activation<WT, PRO_NORM, 1, NSA, NTH>(a, 0, smem, m, ar, ns);
#pragma unroll
    for (int u = UP; u < U; ++u) issue(qb[u], sb[u]);
    __syncthreads();
    float acc = 0.0f;
    int bt_c = 0, y_it = 0;
    const int64_t n_pad = ONE_SHOT ? U : (n_items + U - 1) / U * U;
    for (int64_t k = 0; k < n_pad; k += U) {
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const uint4 q = qb[u], sc = sb[u];
            if (!ONE_SHOT) issue(qb[u], sb[u]);
            if (k + u < n_items) {
                const act_tile<WT> at = load_act<WT, NSA>(smem, m, bt_c, l);
                acc = tile_dot_a<WT>(q, sc, at, acc);
                if (++bt_c == nbt) {
                    const float v = fold8(acc);
                    acc = 0.0f;
                    bt_c = 0;
                    if (l == 0) vbuf[(y_it * 2 + mat) * 32 + pair * 8 + rr] = v;
                    ++y_it;
                }
            }
        }
    }
    __syncthreads();
    // y = gelu(gate) * up for this workgroup's rows (round k: row tiles 4*blockIdx.x + k*rstride + 0..3)
    const bool yimg = a.out_act != nullptr;
    for (int64_t t = tid; (int64_t)blockIdx.x * 4 + (t >> 5) * rstride < a.n_rt; t += NTH) {
        const int64_t k = t >> 5;
        const int j = (int)(t & 31);
        const int64_t rt = (int64_t)blockIdx.x * 4 + k * rstride + (j >> 3);
        if (rt >= a.n_rt) continue;
        const float yv = gelu_tab(a, vbuf[(k * 2) * 32 + j]) * vbuf[(k * 2 + 1) * 32 + j];
        const int64_t row = rt * 8 + (j & 7);
        if (row < a.rows) a.y[row] = yv;
        if (yimg) vbuf[(k * 2) * 32 + j] = yv;  // the image reads y from the gate slot
    }
    if (yimg) {
        __syncthreads();
        // group g = blockIdx.x + k*gridDim.x of 4 row tiles is Q8_0 block g of y (n_rt % 4 == 0)
        for (int64_t t = tid; (int64_t)blockIdx.x * 4 + (t >> 2) * rstride < a.n_rt; t += NTH) {
            const int64_t k = t >> 2;
            const float *yv = vbuf + (k * 2) * 32 + (t & 3) * 8;
            float v[8];
#pragma unroll
            for (int j = 0; j < 8; ++j) v[j] = yv[j];
            image_put_quad(a.out_act, nullptr, a.out_da, blockIdx.x + k * gridDim.x, (int)(t & 3), v);
        }
    }
}

template <int WT>
int launch_gu2(const mv_args &a, int grid_x, hipStream_t s) {
    constexpr int U = 8;
    const bool yimg = a.out_act != nullptr;
    if (a.ncols != 1) {
        set_error("matvec: the split gate/up form is single-column");
        return -1;
    }
    if (yimg && (a.n_rt % 4 || a.rows % 32)) {
        set_error("matvec: the gelu image output needs whole 32-row blocks");
        return -1;
    }
    mv_args la = a;
    const int64_t rstride = (int64_t)grid_x * 4;
    la.rt_q = a.n_rt / rstride;
    la.rt_r = a.n_rt % rstride;
    const int64_t rounds = la.rt_q + (la.rt_r ? 1 : 0);
    const lds_map m = make_lds_map<WT, true>(1, a.n_bt, a.n_bt, 0);
    const size_t lds = m.total + (size_t)rounds * 2 * 32 * 4;
    if (lds > 160 * 1024) {
        set_error("matvec: LDS image too large");
        return -1;
    }
    const bool one_shot = rounds <= 1 && a.n_bt <= U;
    const void *fn = one_shot ? (const void *)k_matvec_gu2<WT, U, true> : (const void *)k_matvec_gu2<WT, U, false>;
    if (lds > 64 * 1024) GHIP_CHECK(hipFuncSetAttribute(fn, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
    if (one_shot) hipLaunchKernelGGL((k_matvec_gu2<WT, U, true>), dim3(grid_x), dim3(512), lds, s, la);
    else hipLaunchKernelGGL((k_matvec_gu2<WT, U, false>), dim3(grid_x), dim3(512), lds, s, la);
    GHIP_CHECK(hipGetLastError());
    return 0;
}

template <int WT, int KS, int PRO, int EPI>
int launch_t(const mv_args &a, int grid_x, hipStream_t s) {
    constexpr bool NSA = KS != 8;  // 8-way split: recompute -8*sum(a) to leave LDS for the stash
    const int64_t seg = KS > 1 ? a.n_bt / KS : a.n_bt;
    const bool yimg = EPI == EPI_GELU_MUL && KS == 1 && a.out_act != nullptr;
    if (yimg && (a.n_rt % 4 || a.rows % 32)) {
        set_error("matvec: the gelu image output needs whole 32-row blocks");
        return -1;
    }
    if (PRO == PRO_IMG && a.nb % 4) {
        set_error("matvec: PRO_IMG needs K % 128 == 0");
        return -1;
    }
    const int64_t ygroups = yimg ? ((a.n_rt >> 2) + grid_x - 1) / grid_x : 0;
    const lds_map m = make_lds_map<WT, NSA>(KS, a.n_bt, seg, ygroups);
    const int threads = KS > 1 ? 64 * KS : 256;  // = k_matvec's NTH
    if (KS > 1 && a.n_bt % KS != 0) {
        set_error("matvec: n_bt not divisible by KS");
        return -1;
    }
    if (m.total > 160 * 1024) {
        set_error("matvec: LDS image too large");
        return -1;
    }
    // register ring depth (16 for gate/up measured slower: issue stalls at 32 loads per wave)
    constexpr int U = 8;
    constexpr int R = KS == 8 ? 4 : 1;  // activation blocks per quad held in registers
    // one-shot when every wave owns at most one row tile of at most U items
    const int64_t waves_x = (int64_t)grid_x * (KS > 1 ? 1 : threads / 64);
    const bool one_shot = KS > 1 && seg <= U && waves_x >= a.n_rt;
    mv_args la = a;  // + the launch geometry (see mv_args::rt_q)
    const int64_t rstride = KS > 1 ? grid_x : (int64_t)grid_x * (threads / 64);
    la.rt_q = a.n_rt / rstride;
    la.rt_r = a.n_rt % rstride;
    la.ygroups = ygroups;
    // gate/up (KS 1): ONE_SHOT selects the SCL scale-run form (k_matvec) when every wave has at most
    // one row tile and a row tile's scales are one 1 KiB run per matrix; + 2 KiB of LDS per wave
    const bool scl = KS == 1 && EPI == EPI_GELU_MUL && GHIP_SCL && a.n_bt * 8 * wfmt<WT>::SCALE_BYTES == 1024 &&
                     waves_x >= a.n_rt;
    const bool os = one_shot || scl;
    const size_t lds = m.total + (scl ? (size_t)(threads / 64) * 2048 : 0);
    if (lds > 160 * 1024) {
        set_error("matvec: LDS image too large");
        return -1;
    }
    const void *fn = os ? (const void *)k_matvec<WT, KS, PRO, EPI, U, R, NSA, KS != 1 || EPI == EPI_GELU_MUL>
                        : (const void *)k_matvec<WT, KS, PRO, EPI, U, R, NSA, false>;
    if (lds > 64 * 1024) GHIP_CHECK(hipFuncSetAttribute(fn, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
    if (os)
        hipLaunchKernelGGL((k_matvec<WT, KS, PRO, EPI, U, R, NSA, KS != 1 || EPI == EPI_GELU_MUL>), dim3(grid_x, a.ncols),
                           dim3(threads), lds, s, la);
    else
        hipLaunchKernelGGL((k_matvec<WT, KS, PRO, EPI, U, R, NSA, false>), dim3(grid_x, a.ncols), dim3(threads), lds, s, la);
    GHIP_CHECK(hipGetLastError());
    return 0;
}

// only the (prologue, epilogue) pairs the engine and the C-ABI use are instantiated
template <int WT, int KS>
int dispatch_pro(int pro, int epi, const mv_args &a, int g, hipStream_t s) {
    if (pro == PRO_Q8 && epi == EPI_STORE) return launch_t<WT, KS, PRO_Q8, EPI_STORE>(a, g, s);       // C-ABI
    if (pro == PRO_NORM && epi == EPI_STORE) return launch_t<WT, KS, PRO_NORM, EPI_STORE>(a, g, s);   // qkv
    if (pro == PRO_EMBED && epi == EPI_STORE) return launch_t<WT, KS, PRO_EMBED, EPI_STORE>(a, g, s); // qkv, layer 0
    if (pro == PRO_F32 && epi == EPI_ADD) return launch_t<WT, KS, PRO_F32, EPI_ADD>(a, g, s);         // wo, wdown
    if (pro == PRO_IMG && epi == EPI_ADD) return launch_t<WT, KS, PRO_IMG, EPI_ADD>(a, g, s);         // wo, wdown (image)
    if (KS == 1 && pro == PRO_NORM && epi == EPI_GELU_MUL)
        return launch_t<WT, 1, PRO_NORM, EPI_GELU_MUL>(a, g, s);                                      // gate/up
    if (KS == 2 && pro == PRO_NORM && epi == EPI_GELU_MUL) return launch_gu2<WT>(a, g, s);            // gate/up, split
    if (KS == 1 && pro == PRO_NORM && epi == EPI_ARGMAX)
        return launch_t<WT, 1, PRO_NORM, EPI_ARGMAX>(a, g, s);                                        // logits
    if (pro == PRO_F32 && epi == EPI_STORE) return launch_t<WT, KS, PRO_F32, EPI_STORE>(a, g, s);
    set_error("matvec: (prologue, epilogue) combination not instantiated");
    return -1;
}

}  // namespace
}  // namespace ghip
