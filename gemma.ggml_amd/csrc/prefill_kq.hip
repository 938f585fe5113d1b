// prefill_kq.hip — the exact K-quant prefill GEMM on the matrix cores (SURVEY §8(a) a6 with T
// columns, §8(f) rank 1): y[t][r] = vec_dot_{q4_K,q6_K}_q8_K(weight row r, Q8_K column t) for every
// prompt position t, bit-identical to ggml's AVX2 lane order (oracle/kquants_cpu.cpp) and to the
// decode matvec of kquant.hip.
//
// Why the matrix cores can do it exactly.  Per super-block (256 values) ggml forms, for each of the
// 8 AVX2 lanes l, an exact int32 sum over the lane's 32 values (bytes 4l..4l+3 of every 32-value
// chunk c, times the chunk's integer scale), converts it to fp32 and chains
// acc_l = fmaf(y.d*f16(x.d), (float)isum_l, acc_l) over super-blocks; Q4_K adds the mins lanes
// accm_k = fmaf(-y.d*f16(x.dmin), (float)(mn·S)_k, accm_k).  isum_l is an integer dot product of
// length 32 whose terms are exact in f16 (Q4_K: nibble*scale <= 945, whose integer bits are the f16
// denormal (nibble*scale) * 2^-24, the 2^24 folded into the row's d; Q6_K: (q6-32)*scale split into
// an even part |.| <= 4096 and its low bit), and every partial sum stays below 2^24 — so an f16
// MFMA with fp32 accumulation returns isum_l EXACTLY, as the float ggml converts it to.  Ordering K
// lane-major (the 32 values of lane l are K = 0..31) makes that a DENSE GEMM per lane: for each
// super-block and lane, two chained v_mfma_f32_32x32x16_f16 give isum_l for a 32-row x 32-token tile
// (Q6_K: four, even part and low bit), then one fmaf per (row, token, lane) — ggml's chain, in the
// same order.  No product is masked out (the Q4_0 path of prefill.hip masks 3/4 of its MFMA rows,
// because its fp32 chain runs per 32-value block).  The Q4_K mins term is one more small exact
// GEMM per super-block: M = (row, k) rows of [mn_2k, mn_2k+1, 64 mn_2k, 64 mn_2k+1], K = the token's
// pair sums split S = 64*Sh + Sl (both exact in f16), fed to the same lane-resident fmaf chain.
//
// Layout: a workgroup is 64 weight rows x 64 tokens, 4 waves of 32 x 32; K is staged one
// super-block at a time (weights converted to f16 A fragments in LDS, activations copied from the
// lane-major f16 image k_q8k_expand writes once per Q8_K INIT), the next super-block's global loads
// in flight during the current one's MFMAs.  blockIdx.x walks tokens, so the token tiles of one
// weight tile run together and the weight tile leaves HBM about once per XCD.
#include <type_traits>
#include <atomic>
#include <climits>
#include <cstdlib>

#include "device_util.h"
#include "kernels.h"

namespace ghip {
namespace {

typedef _Float16 gh8 __attribute__((ext_vector_type(8)));
typedef _Float16 gh4 __attribute__((ext_vector_type(4)));
typedef _Float16 gh2 __attribute__((ext_vector_type(2)));
typedef short gs2 __attribute__((ext_vector_type(2)));
typedef float gf4 __attribute__((ext_vector_type(4)));
typedef uint32_t gu4 __attribute__((ext_vector_type(4)));

// two u16 fields v (each < 1024) -> f16 pair of (v - bias): f16(1024 + v) has bits 0x6400 | v, and
// the f16 subtraction of the bias pair is exact
__device__ __forceinline__ uint32_t pair_f16(uint32_t v, uint32_t bias_pair) {
    typedef _Float16 h2 __attribute__((ext_vector_type(2)));
    const h2 r = __builtin_bit_cast(h2, v | 0x64006400u) - __builtin_bit_cast(h2, bias_pair);
    return __builtin_bit_cast(uint32_t, r);
}
__device__ __forceinline__ uint32_t i2h(int v) { return (uint32_t)__builtin_bit_cast(uint16_t, (_Float16)(float)v); }

// ---- Q8_K columns -> lane-major f16 image, d, mins operand (one wave per (token, super-block)) ----
__global__ void __launch_bounds__(256) k_q8k_expand(q8kx_args a) {
    const int tid = threadIdx.x, e4 = tid & 63;
    const int64_t idx = (int64_t)blockIdx.x * 4 + (tid >> 6);
    if (idx >= (int64_t)a.T * a.nsb) return;
    const int64_t t = idx / a.nsb;
    const int sb = (int)(idx - t * a.nsb);
    const uint8_t *blk = a.x + t * a.x_col_stride + (int64_t)sb * 292;
    const uint32_t q = *(const uint32_t *)(blk + 4 + 4 * e4) ^ 0x80808080u;  // int8 + 128
    const int c = e4 >> 3, l = e4 & 7;  // values 32c + 4l .. +3 -> positions 32l + 4c .. +3
    const uint32_t lo = pair_f16(__builtin_amdgcn_perm(0u, q, 0x0c010c00u), 0x64806480u);
    const uint32_t hi = pair_f16(__builtin_amdgcn_perm(0u, q, 0x0c030c02u), 0x64806480u);
    *(uint2 *)(a.xh + t * a.ldh + (int64_t)sb * 256 + 32 * l + 4 * c) = make_uint2(lo, hi);
    if (e4 == 0) a.xd[t * a.ldd + sb] = *(const float *)blk;
    if (a.xm && e4 >= 4 && e4 < 8) {
        const int k = e4 - 4;
        const int16_t *bs = (const int16_t *)(blk + 260);
        const int S0 = (int)bs[4 * k] + (int)bs[4 * k + 1], S1 = (int)bs[4 * k + 2] + (int)bs[4 * k + 3];
        const uint32_t w0 = i2h(S0 & 63) | (i2h(S1 & 63) << 16);
        const uint32_t w1 = i2h(S0 >> 6) | (i2h(S1 >> 6) << 16);
        *(uint2 *)(a.xm + (t * a.ldm + sb) * 16 + 4 * k) = make_uint2(w0, w1);
    }
}

#ifndef GHIP_GQ_ABL
#define GHIP_GQ_ABL 0  // timing ablations (wrong results): 1 no weight conversion, 2 no compute, 4 no
#endif                 // global loads after the first super-block, 8 no mins GEMM
constexpr int GQ_ABL = GHIP_GQ_ABL;
constexpr int GQ_NT = 256;         // 4 waves, each 16 rows x 32 tokens
// LDS images of one super-block: 16-B fragments (row or token, lane l, K group j = 0..3), stored
// fragment-major — slot (4l + j) * rows + (row ^ swizzle) — so the 16 rows a ds_read_b128 lane
// group reads are 16 consecutive slots (conflict-free for the b128 lane groups {0-3,12-15,20-27} ...),
// and the swizzle (A: l, B: (4l + j) & 7) spreads each write group's 8 lanes over the banks
constexpr int GQ_MBS = 48;         // bytes per staged token of the mins operand
// workgroup tile: Q4_K 64 rows x 32 tokens (fewer bytes staged per output than 32 x 64); Q6_K
// 32 rows x 64 tokens (its two A planes): ~55 / ~68 KB of LDS, two workgroups per CU
template <int WT> struct gq_tile { static constexpr int M = WT == T_Q4_K ? 64 : 32, N = WT == T_Q4_K ? 32 : 64; };

template <int WT> struct gq_raw;
template <> struct gq_raw<T_Q4_K> { gu4 h, q; };
template <> struct gq_raw<T_Q6_K> { gu4 ql, sc; uint2 qh; uint32_t d; };

enum { GQ_STORE = 0, GQ_ADD = 1, GQ_GATE = 2 };

// a 2-byte aligned dword (raw Q6_K super-blocks are 210 B)
__device__ __forceinline__ uint32_t gq_u32_a2(const uint8_t *p) {
    const uint16_t *h = (const uint16_t *)p;
    return (uint32_t)h[0] | ((uint32_t)h[1] << 16);
}

// TL: the engine's lane-contiguous layout (launch_kq_retile); otherwise ggml's row-major blocks
#ifndef GHIP_GQ_DEN
#define GHIP_GQ_DEN 1  // Q4_K A operand as f16 denormals (T = 2048 Q4_K_M prefill 57.25 -> 55.8 ms; 0: biased normals)
#endif
#ifndef GHIP_GQ_WPE
#define GHIP_GQ_WPE 0  // > 0: amdgpu_waves_per_eu (VGPR cap) for the GEMM
#endif
template <int WT, int EPI, bool TL>
__global__ void __launch_bounds__(GQ_NT)
#if GHIP_GQ_WPE
__attribute__((amdgpu_waves_per_eu(GHIP_GQ_WPE, GHIP_GQ_WPE)))
#endif
k_gemm_kq(kqg_args a) {
    constexpr bool Q4 = WT == T_Q4_K;
    constexpr int M = gq_tile<WT>::M, N = gq_tile<WT>::N, NT = GQ_NT, WR = M / 16;
    constexpr int WREC = M * 8 / NT;         // (row, lane) weight records per thread
    constexpr int XREC = N * 512 / 16 / NT;  // 16-B activation records per thread
    static_assert(WREC * NT == M * 8 && XREC * NT * 16 == N * 512 && WR * (N / 32) * 64 == NT, "tile split");
    constexpr int NA = Q4 ? 1 : 2;  // A planes: Q4_K nibble*scale; Q6_K even part and low bit
    // A fragment (row, lane l, j): the 8 K values 8j .. 8j+7 of lane l (chunks 2j and 2j + 1, 4
    // values each) at slot (4l + j) * M + (row ^ l); B fragment (token, l, j) at (4l + j) * N +
    // (token ^ ((4l + j) & 7))
    __shared__ __attribute__((aligned(16))) uint8_t WA[NA * M * 512];
    __shared__ __attribute__((aligned(16))) uint8_t XB[N * 512];
    __shared__ __attribute__((aligned(16))) uint2 MA[Q4 ? M * 4 + 1 : 1];  // mins A (row, k) + a zero slot
    __shared__ __attribute__((aligned(16))) uint8_t MB[Q4 ? N * GQ_MBS : 16];
    __shared__ __attribute__((aligned(16))) float DW[M], DM[M], DX[N];
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int l16 = lane & 15, kg = lane >> 4;
    const int wr = (wave % WR) * 16, wt = (wave / WR) * 32;  // wave tile: rows wr.. (16), tokens wt.. (2 x 16)
    const int64_t t0 = (int64_t)blockIdx.x * N, r0 = (int64_t)blockIdx.y * M;
    if (Q4 && tid == 0) MA[M * 4] = make_uint2(0u, 0u);

    // D register i of column tile ct: row wr + 4kg + i, token wt + 16ct + l16
    float acc[8][2][4], accm[2][4][4];  // accm[ct][i][mins lane k]
#pragma unroll
    for (int ct = 0; ct < 2; ++ct)
#pragma unroll
        for (int i = 0; i < 4; ++i) {
#pragma unroll
            for (int l = 0; l < 8; ++l) acc[l][ct][i] = 0.0f;
#pragma unroll
            for (int k = 0; k < 4; ++k) accm[ct][i][k] = 0.0f;
        }

    gq_raw<WT> wraw[WREC];
    gu4 xr[XREC];
    gu4 mr = {0u, 0u, 0u, 0u};
    float xdv = 0.0f;
    auto gload = [&](int sb) {
#pragma unroll
        for (int k = 0; k < WREC; ++k) {
            const int rec = tid + NT * k, row = rec >> 3, l = rec & 7;
            int64_t r = r0 + row;
            r = r < a.rows ? r : a.rows - 1;
            const uint8_t *wrow = a.w + r * a.row_bytes;
            if constexpr (Q4 && TL) {
                const uint8_t *blk = wrow + (int64_t)sb * 144;
                wraw[k].h = *(const gu4 *)blk;
                wraw[k].q = *(const gu4 *)(blk + 16 + 16 * l);
            } else if constexpr (Q4) {
                const uint8_t *blk = wrow + (int64_t)sb * 144;
                wraw[k].h = *(const gu4 *)blk;
#pragma unroll
                for (int j = 0; j < 4; ++j) wraw[k].q[j] = *(const uint32_t *)(blk + 16 + 32 * j + 4 * l);
            } else if constexpr (!TL) {
                const uint8_t *blk = wrow + (int64_t)sb * 210;
                wraw[k].ql = gu4{gq_u32_a2(blk + 4 * l), gq_u32_a2(blk + 32 + 4 * l), gq_u32_a2(blk + 64 + 4 * l),
                                 gq_u32_a2(blk + 96 + 4 * l)};
                wraw[k].qh = make_uint2(gq_u32_a2(blk + 128 + 4 * l), gq_u32_a2(blk + 160 + 4 * l));
                wraw[k].sc = gu4{gq_u32_a2(blk + 192), gq_u32_a2(blk + 196), gq_u32_a2(blk + 200), gq_u32_a2(blk + 204)};
                wraw[k].d = *(const uint16_t *)(blk + 208);
            } else {
                const uint8_t *grp = wrow + (int64_t)(sb >> 3) * 1680;
                const int i = sb & 7;
                wraw[k].ql = *(const gu4 *)(grp + 128 * i + 16 * l);
                wraw[k].qh = *(const uint2 *)(grp + 1024 + 64 * i + 8 * l);
                wraw[k].sc = *(const gu4 *)(grp + 1536 + 16 * i);
                wraw[k].d = *(const uint16_t *)(grp + 1664 + 2 * i);
            }
        }
#pragma unroll
        for (int k = 0; k < XREC; ++k) {
            const int rec = tid + NT * k, tok = rec >> 5, seg = rec & 31;
            int64_t t = t0 + tok;
            t = t < a.T ? t : a.T - 1;
            xr[k] = *(const gu4 *)(a.xh + t * a.ldh + (int64_t)sb * 256 + seg * 8);
        }
        if (tid < N) {
            int64_t t = t0 + tid;
            t = t < a.T ? t : a.T - 1;
            xdv = a.xd[t * a.ldd + sb];
        } else if (Q4 && tid < 3 * N) {
            const int j = tid - N, tok = j >> 1, h = j & 1;
            int64_t t = t0 + tok;
            t = t < a.T ? t : a.T - 1;
            mr = *(const gu4 *)(a.xm + (t * a.ldm + sb) * 16 + 8 * h);
        }
    };
    auto lstore = [&]() {
#pragma unroll
        for (int k = 0; k < WREC; ++k) {
            const int rec = tid + NT * k, row = rec >> 3, l = rec & 7;
            if (GQ_ABL & 1) break;
            if constexpr (Q4) {
                // six-bit scales and mins (src/kernals.cl:79-84)
                const uint32_t u0 = wraw[k].h.y, u1 = wraw[k].h.z, u2 = wraw[k].h.w;
                const uint32_t s03 = u0 & 0x3f3f3f3fu, s47 = (u2 & 0x0f0f0f0fu) | (((u0 >> 6) & 0x03030303u) << 4);
                const uint32_t m03 = u1 & 0x3f3f3f3fu, m47 = ((u2 >> 4) & 0x0f0f0f0fu) | (((u1 >> 6) & 0x03030303u) << 4);
#pragma unroll
                for (int j = 0; j < 4; ++j) {  // quant dword j: chunk 2j (low nibbles), 2j + 1 (high)
                    const uint32_t scw = j < 2 ? s03 : s47;
                    const uint32_t sl = (scw >> (16 * (j & 1))) & 0xFFu, sh = (scw >> (16 * (j & 1) + 8)) & 0xFFu;
                    const uint32_t qd = wraw[k].q[j];
                    const uint32_t lo = qd & 0x0F0F0F0Fu, hi = (qd >> 4) & 0x0F0F0F0Fu;
#if GHIP_GQ_DEN
                    // the products' integer bits ARE f16 denormals v * 2^-24 (v < 1024): no conversion;
                    // the 2^24 goes into the row's d (exact power-of-two scaling)
                    const uint4 f = make_uint4(__umul24(__builtin_amdgcn_perm(0u, lo, 0x0c010c00u), sl),
                                               __umul24(__builtin_amdgcn_perm(0u, lo, 0x0c030c02u), sl),
                                               __umul24(__builtin_amdgcn_perm(0u, hi, 0x0c010c00u), sh),
                                               __umul24(__builtin_amdgcn_perm(0u, hi, 0x0c030c02u), sh));
#else
                    const uint4 f = make_uint4(pair_f16(__umul24(__builtin_amdgcn_perm(0u, lo, 0x0c010c00u), sl), 0x64006400u),
                                               pair_f16(__umul24(__builtin_amdgcn_perm(0u, lo, 0x0c030c02u), sl), 0x64006400u),
                                               pair_f16(__umul24(__builtin_amdgcn_perm(0u, hi, 0x0c010c00u), sh), 0x64006400u),
                                               pair_f16(__umul24(__builtin_amdgcn_perm(0u, hi, 0x0c030c02u), sh), 0x64006400u));
#endif
                    *(uint4 *)(WA + ((4 * l + j) * M + (row ^ l)) * 16) = f;
                }
                if (l < 4) {  // mins A fragment (row, k = l): [mn_2k, mn_2k+1, 64 mn_2k, 64 mn_2k+1] at K 4k..
                    const uint32_t mw = l < 2 ? m03 : m47;
                    const uint32_t mn0 = (mw >> (16 * (l & 1))) & 0xFFu, mn1 = (mw >> (16 * (l & 1) + 8)) & 0xFFu;
                    const uint32_t v0 = pair_f16(mn0 | (mn1 << 16), 0x64006400u);
                    const uint32_t v1 = i2h(64 * (int)mn0) | (i2h(64 * (int)mn1) << 16);
                    MA[row * 4 + l] = make_uint2(v0, v1);
                } else if (l == 4) {
                    DW[row] = GHIP_GQ_DEN ? h2f(wraw[k].h.x) * 16777216.0f : h2f(wraw[k].h.x);
                    DM[row] = h2f(wraw[k].h.x >> 16);
                }
            } else {
                // Q6_K lane l (vec_dot_q6_K_q8_K AVX2): half u, chunk i' of 4: value q6 - 32, scale
                // byte 8u + 2i' + (l >> 2); A = (q6 - 32) * scale = (A & ~1) + (A & 1)
                const uint32_t qla[2] = {wraw[k].ql.x, wraw[k].ql.z}, qlb[2] = {wraw[k].ql.y, wraw[k].ql.w};
                const uint32_t qhw[2] = {wraw[k].qh.x, wraw[k].qh.y};
                const uint32_t scd[4] = {wraw[k].sc.x, wraw[k].sc.y, wraw[k].sc.z, wraw[k].sc.w};
#pragma unroll
                for (int u = 0; u < 2; ++u) {
                    const uint32_t qa = qla[u], qb = qlb[u], qh = qhw[u];
                    const uint32_t q6[4] = {(qa & 0x0F0F0F0Fu) | ((qh & 0x03030303u) << 4),
                                            (qb & 0x0F0F0F0Fu) | (((qh >> 2) & 0x03030303u) << 4),
                                            ((qa >> 4) & 0x0F0F0F0Fu) | (((qh >> 4) & 0x03030303u) << 4),
                                            ((qb >> 4) & 0x0F0F0F0Fu) | (((qh >> 6) & 0x03030303u) << 4)};
#pragma unroll
                    for (int gg = 0; gg < 2; ++gg) {
                        uint32_t fe[4], fo[4];
#pragma unroll
                        for (int cc = 0; cc < 2; ++cc) {
                            const int ip = 2 * gg + cc, bi = 8 * u + 2 * ip + (l >> 2);
                            const short sc = (short)(int8_t)(uint8_t)(scd[bi >> 2] >> (8 * (bi & 3)));
#pragma unroll
                            for (int p = 0; p < 2; ++p) {  // values 2p, 2p+1 as an int16 pair: (q6 - 32) * scale
                                const gs2 q = __builtin_bit_cast(gs2, __builtin_amdgcn_perm(0u, q6[ip], p ? 0x0c030c02u : 0x0c010c00u));
                                const gs2 A = (q - (gs2){32, 32}) * (gs2){sc, sc};  // |A| <= 4096: exact in int16
                                const gs2 ev = A & (gs2){(short)0xFFFE, (short)0xFFFE};
                                fe[2 * cc + p] = __builtin_bit_cast(uint32_t, __builtin_convertvector(ev, gh2));
                                fo[2 * cc + p] = __umul24(__builtin_bit_cast(uint32_t, A) & 0x00010001u, 0x3C00u);
                            }
                        }
                        const int off = ((4 * l + 2 * u + gg) * M + (row ^ l)) * 16;
                        *(uint4 *)(WA + off) = make_uint4(fe[0], fe[1], fe[2], fe[3]);
                        *(uint4 *)(WA + M * 512 + off) = make_uint4(fo[0], fo[1], fo[2], fo[3]);
                    }
                }
                if (l == 0) DW[row] = h2f(wraw[k].d);
            }
        }
#pragma unroll
        for (int k = 0; k < XREC; ++k) {
            const int rec = tid + NT * k, tok = rec >> 5, seg = rec & 31;
            *(gu4 *)(XB + (seg * N + (tok ^ (seg & 7))) * 16) = xr[k];
        }
        if (tid < N) {
            DX[tid] = xdv;
        } else if (Q4 && tid < 3 * N) {
            const int j = tid - N;
            *(gu4 *)(MB + (j >> 1) * GQ_MBS + 16 * (j & 1)) = mr;
        }
    };

    // this lane's mins A fragment (v_mfma_f32_16x16x16_f16, MFMA i): row l16 = 4 rho + k stands for
    // weight row wr + 4 rho + i, so D register k of lane (kg, l16) is mins lane k of row wr + 4kg + i —
    // the row of the main tile's register i; K 4k..4k+3 live in lane group kg == k, the others read zeros
    const int rho = l16 >> 2, mk = l16 & 3;
    const bool m_act = mk == kg;
    const uint2 *ma_ptr = m_act ? &MA[(wr + 4 * rho) * 4 + mk] : &MA[Q4 ? M * 4 : 0];
    const int ma_stride = m_act ? 4 : 0;
    // this lane's fragment slots: A (l, kg) at (4l + kg) * M + wr + (l16 ^ l); B (l, kg, ct) at
    // (4l + kg) * N + wt + 16ct + (l16 ^ ((4l + kg) & 7)), the swizzle depending on l's parity only
    const uint8_t *ab = WA + (kg * M + wr) * 16;
    const uint8_t *bb0 = XB + (kg * N + wt + (l16 ^ kg)) * 16, *bb1 = XB + (kg * N + wt + (l16 ^ (kg + 4))) * 16;

    // Q4_K with GHIP_GQ_DEN: DW = x.d * 2^24 and the MFMA returns isum * 2^-24, so ggml's
    // fmaf(d, isum, acc) with d = y.d * x.d is fmaf(d * 2^24, isum * 2^-24, acc) exactly — provided
    // d * 2^24 is d scaled, not a fresh rounding.  d is therefore rounded as ggml rounds it (unscaled,
    // a subnormal when |y.d * x.d| < 2^-126) and then scaled by 2^24 (exact): (y.d * (DW * 2^-24)) *
    // 2^24.  Assumption kept: |y.d * x.d| < 2^104, i.e. activations below ~3e26 for any
    // f16 x.d (beyond, d * 2^24 overflows; ggml's d would not)
    auto compute = [&]() {
        float dd[2][4], dm[2][4];
        float4 w4 = *(const float4 *)&DW[wr + 4 * kg];
        if constexpr (Q4 && GHIP_GQ_DEN) {
            constexpr float inv = 1.0f / 16777216.0f;  // exact: DW = x.d * 2^24
            w4.x *= inv; w4.y *= inv; w4.z *= inv; w4.w *= inv;
        }
        float4 m4;
        if constexpr (Q4) m4 = *(const float4 *)&DM[wr + 4 * kg];
#pragma unroll
        for (int ct = 0; ct < 2; ++ct) {
            const float yd = DX[wt + 16 * ct + l16];
            dd[ct][0] = yd * w4.x; dd[ct][1] = yd * w4.y; dd[ct][2] = yd * w4.z; dd[ct][3] = yd * w4.w;
            if constexpr (Q4 && GHIP_GQ_DEN) {
#pragma unroll
                for (int i = 0; i < 4; ++i) dd[ct][i] = pin(dd[ct][i]) * 16777216.0f;
            }
            if constexpr (Q4) {
                const float ny = -yd;
                dm[ct][0] = ny * m4.x; dm[ct][1] = ny * m4.y; dm[ct][2] = ny * m4.z; dm[ct][3] = ny * m4.w;
            }
        }
        const gf4 z = {0.0f, 0.0f, 0.0f, 0.0f};
#pragma unroll
        for (int l = 0; l < 8; ++l) {  // lane l's 32 values of the super-block = K of one MFMA
            gh8 a0, a1;
            if (GQ_ABL & 16) {
                a0 = (gh8){(_Float16)(float)l, 1, 2, 3, 4, 5, 6, (_Float16)(float)lane};
                a1 = a0;
            } else {
                a0 = *(const gh8 *)(ab + (4 * l * M + (l16 ^ l)) * 16);
                if constexpr (!Q4) a1 = *(const gh8 *)(ab + M * 512 + (4 * l * M + (l16 ^ l)) * 16);
            }
#pragma unroll
            for (int ct = 0; ct < 2; ++ct) {
                gh8 b;
                if (GQ_ABL & 16) b = a0 + (_Float16)(float)ct;
                else b = *(const gh8 *)((l & 1 ? bb1 : bb0) + (4 * l * N + 16 * ct) * 16);
                gf4 D;
                if (GQ_ABL & 32) {
                    D = (gf4){(float)a0[0], (float)b[1], (float)a0[2], (float)b[3]};
                } else {
                    D = __builtin_amdgcn_mfma_f32_16x16x32_f16(a0, b, z, 0, 0, 0);
                    if constexpr (!Q4) D = __builtin_amdgcn_mfma_f32_16x16x32_f16(a1, b, D, 0, 0, 0);
                }
#pragma unroll
                for (int i = 0; i < 4; ++i) acc[l][ct][i] = __builtin_fmaf(dd[ct][i], D[i], acc[l][ct][i]);
            }
        }
        if constexpr (Q4 && !(GQ_ABL & 8)) {
#pragma unroll
            for (int ct = 0; ct < 2; ++ct) {
                const gh4 mb = *(const gh4 *)(MB + (wt + 16 * ct + l16) * GQ_MBS + 8 * kg);
#pragma unroll
                for (int i = 0; i < 4; ++i) {
                    const gh4 ma = *(const gh4 *)(ma_ptr + i * ma_stride);
                    const gf4 Dm = __builtin_amdgcn_mfma_f32_16x16x16f16(ma, mb, z, 0, 0, 0);
#pragma unroll
                    for (int k = 0; k < 4; ++k) accm[ct][i][k] = __builtin_fmaf(dm[ct][i], Dm[k], accm[ct][i][k]);
                }
            }
        }
    };

    gload(0);
    for (int sb = 0; sb < a.nsb; ++sb) {
        lstore();
        __syncthreads();
        if (sb + 1 < a.nsb && !(GQ_ABL & 4)) gload(sb + 1);
        if (!(GQ_ABL & 2)) compute();
        __syncthreads();
    }

    // hsum_float_8 of the lanes, + (m0+m2)+(m1+m3) for Q4_K, then the epilogue: 4 consecutive rows
    // of one token per lane and column tile
    const int64_t rb = r0 + wr + 4 * kg;
    const bool vec = rb + 3 < a.rows && (a.ldy & 3) == 0 && (((uintptr_t)a.y | (uintptr_t)a.resid | (uintptr_t)a.gate_in) & 15) == 0;
#pragma unroll
    for (int ct = 0; ct < 2; ++ct) {
        const int64_t t = t0 + wt + 16 * ct + l16;
        float v[4];
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            float (&q)[8][2][4] = acc;
            v[i] = ((q[0][ct][i] + q[4][ct][i]) + (q[2][ct][i] + q[6][ct][i])) +
                   ((q[1][ct][i] + q[5][ct][i]) + (q[3][ct][i] + q[7][ct][i]));
            if (Q4) v[i] = v[i] + ((accm[ct][i][0] + accm[ct][i][2]) + (accm[ct][i][1] + accm[ct][i][3]));
        }
        if (t >= a.T) continue;
        const int64_t o = t * a.ldy + rb;
        float e[4] = {0.0f, 0.0f, 0.0f, 0.0f};
        if (EPI != GQ_STORE) {
            const float *src = EPI == GQ_GATE ? a.gate_in : a.resid;
            if (vec) {
                const float4 f = *(const float4 *)(src + o);
                e[0] = f.x; e[1] = f.y; e[2] = f.z; e[3] = f.w;
            } else {
#pragma unroll
                for (int i = 0; i < 4; ++i)
                    if (rb + i < a.rows) e[i] = src[o + i];
            }
        }
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            if (EPI == GQ_GATE) {  // gelu(gate) then ggml_mul by up (src/gemma_model.cpp:444-452)
                const float gv = e[i];
                const float gl = (a.gelu_clamp && gv <= -10.0f) ? 0.0f : (a.gelu_clamp && gv >= 10.0f) ? gv : h2f(a.gelu_tab[f2h(gv)]);
                v[i] = gl * v[i];
            } else if (EPI == GQ_ADD) {
                v[i] = v[i] + e[i];
            }
        }
        if (vec) {
            *(float4 *)(a.y + o) = make_float4(v[0], v[1], v[2], v[3]);
        } else {
#pragma unroll
            for (int i = 0; i < 4; ++i)
                if (rb + i < a.rows) a.y[o + i] = v[i];
        }
    }
}

}  // namespace

static std::atomic<int> g_kq_gemm_min{-1};
int kq_gemm_min() {
    const int v = g_kq_gemm_min.load();
    if (v >= 0) return v;
    return 8;  // default: the MFMA GEMM from 8 columns (hpc_set_kq_gemm_min moves it)
}
void set_kq_gemm_min(int v) { g_kq_gemm_min.store(v); }

int launch_q8k_expand(const q8kx_args &a, hipStream_t s) {
    if (a.T <= 0 || a.nsb <= 0 || !a.x || !a.xh || !a.xd || a.x_col_stride % 4 || a.x_col_stride < (int64_t)a.nsb * 292 ||
        a.ldh < (int64_t)a.nsb * 256 || a.ldh % 8 || a.ldd < a.nsb || (a.xm && a.ldm < a.nsb) || ((uintptr_t)a.x & 3) ||
        ((uintptr_t)a.xh & 15) || ((uintptr_t)a.xm & 15)) {
        set_error("q8k_expand: bad shape or alignment");
        return -1;
    }
    const int64_t n = ((int64_t)a.T * a.nsb + 3) / 4;
    if (n > 0x7fffffff) {
        set_error("q8k_expand: too many super-blocks");
        return -1;
    }
    hipLaunchKernelGGL(k_q8k_expand, dim3((unsigned)n), dim3(256), 0, s, a);
    GHIP_CHECK(hipGetLastError());
    return 0;
}

int launch_gemm_kq(int wtype, const kqg_args &a, hipStream_t s) {
    const bool q4 = wtype == T_Q4_K;
    if ((wtype != T_Q4_K && wtype != T_Q6_K) || a.nsb <= 0 || a.T <= 0 || a.rows <= 0 || !a.w || !a.xh || !a.xd || !a.y ||
        a.ldh % 8 || a.ldh < (int64_t)a.nsb * 256 || a.ldd < a.nsb || a.ldy < a.rows || ((uintptr_t)a.xh & 15) ||
        ((uintptr_t)a.w & (q4 ? 15 : 3)) || (q4 && (!a.xm || a.ldm < a.nsb || ((uintptr_t)a.xm & 15) || a.row_bytes != (int64_t)a.nsb * 144)) ||
        (!q4 && ((a.tiled && a.nsb % 8) || a.row_bytes != (int64_t)a.nsb * 210)) || (a.gate_in && !a.gelu_tab)) {
        set_error("gemm_kq: unsupported type, shape or alignment (lane-tiled Q4_K, or Q6_K with K % 2048 == 0)");
        return -1;
    }
    const int M = q4 ? gq_tile<T_Q4_K>::M : gq_tile<T_Q6_K>::M, N = q4 ? gq_tile<T_Q4_K>::N : gq_tile<T_Q6_K>::N;
    const int64_t gy = (a.rows + M - 1) / M, gx = (a.T + N - 1) / N;
    if (gy > 65535 || gx > 0x7fffffff) {
        set_error("gemm_kq: too many rows");
        return -1;
    }
    const dim3 grid((unsigned)gx, (unsigned)gy);
    const int epi = a.gate_in ? GQ_GATE : a.resid ? GQ_ADD : GQ_STORE;
#define GQ_GO(WT, E)                                                                        \
    do {                                                                                    \
        if (a.tiled) hipLaunchKernelGGL((k_gemm_kq<WT, E, true>), grid, dim3(GQ_NT), 0, s, a);  \
        else hipLaunchKernelGGL((k_gemm_kq<WT, E, false>), grid, dim3(GQ_NT), 0, s, a);         \
    } while (0)
    if (q4) {
        if (epi == GQ_GATE) GQ_GO(T_Q4_K, GQ_GATE);
        else if (epi == GQ_ADD) GQ_GO(T_Q4_K, GQ_ADD);
        else GQ_GO(T_Q4_K, GQ_STORE);
    } else {
        if (epi == GQ_GATE) GQ_GO(T_Q6_K, GQ_GATE);
        else if (epi == GQ_ADD) GQ_GO(T_Q6_K, GQ_ADD);
        else GQ_GO(T_Q6_K, GQ_STORE);
    }
#undef GQ_GO
    GHIP_CHECK(hipGetLastError());
    return 0;
}

}  // namespace ghip
