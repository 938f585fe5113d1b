// token.hip — a decode token's transformer layers as ONE persistent launch.
//
// Replaces the 5 dependent launches per layer of the per-token graph (src/gemma_model.cpp:231-286
// running build_compute_graph :665-747): rms_norm*w -> Wq|Wk|Wv -> rope/KQ/softmax/KQV -> Wo (+x) ->
// rms_norm*w -> Wgate, Wup -> gelu*mul -> Wdown (+sa), for all layers, with the same arithmetic and
// bits as the separate kernels (ggml's AVX2 lane order, matvec_impl.h / matvec_rr.hip / attn_impl.h).
//
// Why one launch pays here when the fused layer front (layer_front.hip) did not: every CU reads
// ITS share of every weight matrix once per token, and those bytes do not depend on the
// activations.  So each CU streams its weights ahead of the dependency edges into an LDS ring
// (LDS-DMA, `global_load_lds_dwordx4 ... nt`: MI355X_MICROARCH nt-weights / prefetch-credit): while
// the chip waits for a hand-off (attention, an all-gather of x), the next matrices are already
// landing, and the matvec after the edge runs from LDS instead of paying a launch ramp to its
// first weight byte (~2.8 us per launch).
//
// Workgroups: grid = E/8 (one 8-row tile of Wo / Wdown per workgroup; one workgroup per CU, all
// resident), 576 threads = 8 TERM waves + 1 CARRIER wave (the round-pipelined matvec's roles,
// matvec_rr.hip).  Work of workgroup c per layer:
//   qkv   row tile c (and c + grid when qkv has more tiles): rr rounds, rows -> granules
//   attn  (c % 8 == 0, c/8 < H*S) head (c/8)/S, KQV dims slice (c/8)%S — attn_head_dev
//   o     row tile c: rr rounds, sa = o + x, rows -> granules
//   ffn   gate/up row tile 8c + w on term wave w (two ordered chains per wave, shared operands),
//         gelu(gate)*up -> the two Q8_0 blocks of h this workgroup owns -> granules
//   down  row tile c: rr rounds, x' = down + sa -> granules (the next layer's input)
// Term wave w owns a private ring of NR weight-tile slots (1 KiB quants + the tile's scales) and
// consumes tiles in a fixed order (its share of qkv, o, gate/up, down, then the next layer...); each
// consumed slot is refilled at once with the tile NR ahead in that order (past the end: a harmless
// re-read), so exactly NR tiles are in flight and `s_waitcnt vmcnt(2*(NR-1))` retires the oldest.
// The DMA is inline asm (hipcc's own waits never drain it; its counted waits only over-wait).
//
// Hand-offs: 8-byte {payload, tag} granules stored by one agent-scope relaxed atomic store each
// (write-through, `sc1`) and polled by every consuming workgroup with agent-scope loads until the
// tags match (cdna_hip_programming Guideline 16 R2; MI355X_MICROARCH handoff-1to1 / allgather):
// the data is the flag, no fences, no counters.  tag = epoch*256 + layer*8 + edge + 1 with epoch
// a device counter k_advance / k_set_position bump once per token, so stale granules of an earlier
// token never match.  A buffer is rewritten only after a later all-to-all edge, i.e. after every
// consumer has read it.  Every poll is bounded in time: on a timeout the workgroup sets the sticky
// error word and stops waiting for the rest of the launch (wrong numbers, never a hung GPU).
#include "attn_impl.h"
#include "matvec_rr.h"

#include <type_traits>

namespace ghip {
namespace {

constexpr int TK_TW = 8;                     // term waves (each with its weight ring)
constexpr int TK_AUX = 4;                    // aux waves: wave 8 = the carrier; all 4 gather and norm
constexpr int TK_NTH = 64 * (TK_TW + TK_AUX);
constexpr int TK_ATH = 64 * TK_AUX;          // aux threads
constexpr int TK_SLOT = 1152;                // ring slot: 1 KiB quants + up to 128 B scales
constexpr int TK_MAXL = 32;                  // layers the LDS pointer table holds
constexpr int TK_TABB = (int)sizeof(tok_layer);  // bytes per layer in that table (14 pointers)
// the launch's arguments live in device memory and are read through the constant address space:
// scalar loads (lgkmcnt), never a vector load that a term wave's counted wait would also drain
typedef const __attribute__((address_space(4))) tok_args ctok;
constexpr int TK_MAXCTX = 1024;              // the attention scratch overlays the down image
#ifndef TK_DEFER
#define TK_DEFER 0
#endif

enum { EDGE_X = 0, EDGE_QKV = 1, EDGE_ATT = 2, EDGE_SA = 3, EDGE_H = 4 };

__device__ __forceinline__ uint32_t lds_u32(const void *p) { return (uint32_t)(uintptr_t)p; }

// one wave instruction: 16 B per active lane from `g` into LDS at m0 + 16*lane (nt: read once)
__device__ __forceinline__ void dma16(const void *g, uint32_t lds_addr) {
    const uint32_t lds = __builtin_amdgcn_readfirstlane(lds_addr);  // wave-uniform by construction
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
}

// the carrier's exact-term stash, one slot per rr round (ping-pong).  Q4_0: s as int16 (|sum of 4
// (nib-8)*a| <= 4064), the carry_ring<true> chunk layout (8 blocks = one uint4 of s + two float4 of
// d); Q8_0: f32 s (17 bits), rr_geom's layout.  Slots end with slack for the carry ring's over-reads.
template <int WT>
struct tk_stash;
template <>
struct tk_stash<T_Q4_0> {
    static constexpr bool I16 = true;
    static constexpr int RUN = 64, SBP = RUN + 8 /* int16: 144 B lane stride */, SBPD = RUN + 4;
    static constexpr uint32_t S_BYTES = 64 * SBP * 2 + 256, D_BYTES = 8 * SBPD * 4 + 512, SLOT = S_BYTES + D_BYTES;
};
template <>
struct tk_stash<T_Q8_0> {
    static constexpr bool I16 = false;
    static constexpr int RUN = rr_geom<T_Q8_0>::RUN, SBP = rr_geom<T_Q8_0>::SBP, SBPD = rr_geom<T_Q8_0>::SBPD;
    static constexpr uint32_t S_BYTES = rr_geom<T_Q8_0>::S_BYTES, D_BYTES = rr_geom<T_Q8_0>::D_BYTES + 256,
                              SLOT = S_BYTES + D_BYTES;
};

// LDS byte layout of the launch, compile-time for the shapes (E, F) the kernel is built for.  IMG
// holds the activation image of the current matvec (K = E: act, ns (Q4_0), da; K = F: act, da —
// the down matvec recomputes ns); the attention phase's scratch (q16/k16, scores, P16, then the
// gathered q|k|v) overlays it between the q|k|v matvec and the attention-output gather.
template <int WT, int NR, int E, int F>
struct tok_layout {
    static constexpr int BT = wfmt<WT>::BT;
    static constexpr int NBE = E / 32 / BT, NBF = F / 32 / BT;  // block tiles per row at K = E / K = F
    static constexpr uint32_t IMG_F = (uint32_t)F + (uint32_t)(F / 32) * 4;
    static constexpr uint32_t RING = 0;
    static constexpr uint32_t IMG = (uint32_t)TK_TW * NR * TK_SLOT;
    static constexpr uint32_t XF = IMG + ((IMG_F + 15) & ~15u);
    static constexpr uint32_t STASH = XF + (uint32_t)E * 4;
    static constexpr uint32_t SMALL = STASH + 2 * tk_stash<WT>::SLOT;
    static constexpr uint32_t TOTAL = SMALL + 1024 + TK_MAXL * TK_TABB;
    // image maps (offsets inside IMG): K = E (with ns) and K = F (no ns plane)
    static constexpr uint32_t E_ACT = 0, E_NS = E, E_DA = WT == T_Q4_0 ? 2 * E : E;
    static constexpr uint32_t F_ACT = 0, F_NS = 0, F_DA = F;
    static constexpr uint32_t ATT_QKV(int ctx) { return ((uint32_t)(1024 + 6 * ctx + 16) + 15) & ~15u; }
    static constexpr bool att_fits(int ctx, int qkv_rows) {
        return ATT_QKV(ctx) + (uint32_t)qkv_rows * 4 <= IMG_F && E_DA + E / 8 <= IMG_F;
    }
};
__host__ __device__ constexpr lds_map tok_map(uint32_t act, uint32_t ns, uint32_t da) {
    lds_map m{};
    m.act = act; m.ns = ns; m.da = da;
    return m;
}
// SMALL: [0, 512) gate and up values of this workgroup's 64 ffn rows (f32), [512, 544) sa rows
// (8 f32), [576, 704) 16 doubles of the norm reduction, [768] the workgroup's failed flag, [784] a
// sink word;
// [1024, 1024 + 112 * n_layer) the layers' tok_layer pointer records (the ring's address table and
// the norms / caches: an LDS read instead of two dependent loads, ~1.4 us when they miss)
constexpr int SM_H = 0, SM_SA = 512, SM_RED = 576, SM_FAIL = 768, SM_SINK = 784, SM_TAB = 1024;

__device__ __forceinline__ uint32_t tag_of(uint32_t ep, int layer, int edge) {
    return ep * 256u + (uint32_t)layer * 8u + (uint32_t)edge + 1u;
}

__device__ void note_timeout(ctok &a, int site, int layer) {
    typedef __attribute__((address_space(1))) int gi_t;
    __hip_atomic_store((gi_t *)a.err + 1, site, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    __hip_atomic_store((gi_t *)a.err + 2, layer, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    __hip_atomic_store((gi_t *)a.err, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// All-gather of n granules (n even) into LDS by the aux threads (atid 0..TK_ATH-1; they have no
// weight DMAs in flight, so a wait for a granule never waits for the ring): every thread polls its
// granule pairs (16-B sc1 loads, both halves untorn) until both tags match, all its pairs re-read
// together per pass.  dst[i] = payload of granule i; ns (optional) = -8 * sum of the payload's 4
// int8 (the Q4_0 image's ns plane).  The caller joins a barrier before reading dst.
template <int MAXP>
__device__ void gather(int atid, bool *fail, ctok &a, const unsigned long long *g, int n, uint32_t tag,
                       uint32_t *dst, uint32_t *ns, int site, int layer) {
    const int np = n >> 1;
    if ((atid & ~63) >= np) return;  // wave-uniform: nothing for this wave (short vectors)
    const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc((void *)g, 0, n * 8, 0x00020000);
    uint32_t v[MAXP][4];
    bool ok = false;
    const bool failed = *fail;  // written before the last barrier (LDS)
    const unsigned t0 = (unsigned)__builtin_amdgcn_s_memrealtime();
    for (;;) {
#pragma unroll
        for (int k = 0; k < MAXP; ++k) {
            int p = atid + k * TK_ATH;
            p = p < np ? p : np - 1;  // clamp: no branch around the load
            const auto r = __builtin_amdgcn_raw_buffer_load_b128(rs, p * 16, 0, 16 /* sc1 */);
            v[k][0] = r[0]; v[k][1] = r[1]; v[k][2] = r[2]; v[k][3] = r[3];
        }
        ok = true;
#pragma unroll
        for (int k = 0; k < MAXP; ++k) ok &= (v[k][1] == tag) & (v[k][3] == tag);
        if (ok || failed) break;
        if ((unsigned)__builtin_amdgcn_s_memrealtime() - t0 > a.timeout) {
            *fail = true;
            note_timeout(a, site, layer);
            break;
        }
        __builtin_amdgcn_s_sleep(4);
    }
#pragma unroll
    for (int k = 0; k < MAXP; ++k) {
        const int p = atid + k * TK_ATH;
        if (p < np) {
            dst[2 * p] = v[k][0];
            dst[2 * p + 1] = v[k][2];
            if (ns) {
                ns[2 * p] = (uint32_t)sdot4(v[k][0], 0xF8F8F8F8u, 0);
                ns[2 * p + 1] = (uint32_t)sdot4(v[k][2], 0xF8F8F8F8u, 0);
            }
        }
    }
}

// Wait until one granule pair per producer is tagged (pairs first + k*stride, k < count <= TK_ATH;
// one pair per aux thread): a cheap probe (a few KB per pass, backed-off polls) before the full
// gather reads every granule once.  Polling the whole vector instead kept ~36 KB per CU per pass
// in flight chip-wide and slowed the weight stream of the workgroups still computing.
__device__ void probe(int atid, bool *fail, ctok &a, const unsigned long long *g, int n, int first, int stride, int count,
                      uint32_t tag, int site, int layer) {
    if ((atid & ~63) >= count) return;  // wave-uniform
    const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc((void *)g, 0, n * 8, 0x00020000);
    const int k = atid < count ? atid : count - 1;
    const int p = first + k * stride;
    if (*fail) return;
    const unsigned t0 = (unsigned)__builtin_amdgcn_s_memrealtime();
    for (;;) {
        const auto r = __builtin_amdgcn_raw_buffer_load_b128(rs, p * 16, 0, 16 /* sc1 */);
        if (r[1] == tag && r[3] == tag) break;
        if ((unsigned)__builtin_amdgcn_s_memrealtime() - t0 > a.timeout) {
            *fail = true;
            note_timeout(a, site, layer);
            break;
        }
        __builtin_amdgcn_s_sleep(4);
    }
}

// rms_norm(xf) * w, then quantize_row_q8_0 into the image (build_activation's arithmetic on an LDS
// source: double sum of the fp32 squares, exact), by the aux threads; every wave
// of the workgroup calls it (one barrier inside)
template <int E>
struct norm_w {  // an aux thread's norm weights, loaded ahead of the gather the norm waits for
    static constexpr int NQ = TK_ATH / 4, NB = E / 32, NI = (NB + NQ - 1) / NQ;
    float v[NI][8];
    __device__ __forceinline__ void load(int atid, const float *w) {
        const int q = atid & 3;
#pragma unroll
        for (int i = 0; i < NI; ++i) {
            const int b = (atid >> 2) + i * NQ, bb = b < NB ? b : 0;
            const float4 w0 = *(const float4 *)(w + bb * 32 + q * 8), w1 = *(const float4 *)(w + bb * 32 + q * 8 + 4);
            v[i][0] = w0.x; v[i][1] = w0.y; v[i][2] = w0.z; v[i][3] = w0.w;
            v[i][4] = w1.x; v[i][5] = w1.y; v[i][6] = w1.z; v[i][7] = w1.w;
        }
    }
};
template <int WT, int E>
__device__ void norm_quant(bool aux, int atid, const float *xf, const norm_w<E> &wv, float eps, uint8_t *img, const lds_map &m,
                           double *red) {
    constexpr int NQ = norm_w<E>::NQ, NB = norm_w<E>::NB, NI = norm_w<E>::NI;
    const int q = atid & 3;
    double part = 0.0;
    if (aux) {
#pragma unroll
        for (int i = 0; i < NI; ++i) {
            const int b = (atid >> 2) + i * NQ;
            if (b >= NB) break;
            const float4 u = *(const float4 *)(xf + b * 32 + q * 8), v4 = *(const float4 *)(xf + b * 32 + q * 8 + 4);
            const float v[8] = {u.x, u.y, u.z, u.w, v4.x, v4.y, v4.z, v4.w};
#pragma unroll
            for (int j = 0; j < 8; ++j) {
                const float sq = v[j] * v[j];
                part += (double)sq;
            }
        }
#pragma unroll
        for (int off = 32; off >= 1; off >>= 1) part += __shfl_xor(part, off);
        if ((atid & 63) == 0) red[atid >> 6] = part;
    }
    lds_barrier();
    if (aux) {
        double sum = 0.0;
        for (int k = 0; k < TK_AUX; ++k) sum += red[k];
        const double qm = div_by_n(sum, E);
        float mean = (float)qm;
        if (__builtin_expect(!rms_mean_certain(qm, E), 0))  // uniform over the aux waves; rare: ggml's own order
            mean = (float)(seq_sumsq_wave(E, [&](int64_t i0, float v[8]) {
                               const float4 u = *(const float4 *)(xf + i0), u4 = *(const float4 *)(xf + i0 + 4);
                               v[0] = u.x; v[1] = u.y; v[2] = u.z; v[3] = u.w; v[4] = u4.x; v[5] = u4.y; v[6] = u4.z; v[7] = u4.w;
                           }) / (double)E);
        const float scale = 1.0f / sqrtf(mean + eps);
#pragma unroll
        for (int i = 0; i < NI; ++i) {
            const int b = (atid >> 2) + i * NQ;
            if (b >= NB) break;
            const float4 u = *(const float4 *)(xf + b * 32 + q * 8), v4 = *(const float4 *)(xf + b * 32 + q * 8 + 4);
            float v[8] = {u.x, u.y, u.z, u.w, v4.x, v4.y, v4.z, v4.w};
#pragma unroll
            for (int j = 0; j < 8; ++j) {
                const float s = v[j] * scale;  // rms_norm output
                v[j] = s * wv.v[i][j];         // ggml_mul by the norm weight
            }
            put_quad<WT, true>(img, m, b, q, v);
        }
    }
}

// Q4_0 exact terms of one tile into the int16 stash (tile_dot<T_Q4_0, STASH>'s packing, on the
// operands of load_act): s of blocks (2p, 2p+1) in dword p, d as 8 floats (lane 0 of the row)
template <bool NSA>
__device__ __forceinline__ void terms16(uint4 q, uint4 scv, const uint8_t *img, const lds_map &m, int bt, int l,
                                        int16_t *st_s, float *st_d) {
    const act_tile<T_Q4_0> t = load_act<T_Q4_0, NSA>(img, m, bt, l);
    const uint32_t qv[4] = {q.x, q.y, q.z, q.w}, sv[4] = {scv.x, scv.y, scv.z, scv.w};
    uint32_t pk[4];
    float dk[8];
#pragma unroll
    for (int p = 0; p < 4; ++p) {
        const uint32_t lo = qv[p] & 0x0F0F0F0Fu, hi = (qv[p] >> 4) & 0x0F0F0F0Fu;
        const int s0 = sdot4(lo, t.av[2 * p], (int)t.nv[2 * p]);
        const int s1 = sdot4(hi, t.av[2 * p + 1], (int)t.nv[2 * p + 1]);
        pk[p] = ((uint32_t)s0 & 0xFFFFu) | ((uint32_t)s1 << 16);
        dk[2 * p] = mix_lo(sv[p], t.dav[2 * p]);
        dk[2 * p + 1] = mix_hi(sv[p], t.dav[2 * p + 1]);
    }
    *(uint4 *)st_s = make_uint4(pk[0], pk[1], pk[2], pk[3]);
    if (l == 0) {
        *(float4 *)st_d = make_float4(dk[0], dk[1], dk[2], dk[3]);
        *(float4 *)(st_d + 4) = make_float4(dk[4], dk[5], dk[6], dk[7]);
    }
}

// the carrier wave pulls a norm weight vector (E floats) into its XCD's L2 ahead of the norm that
// reads it (the ring's nt weight stream leaves it cold otherwise); the loads are consumed by a
// test that never holds
__device__ __forceinline__ void touch_l2(const float *p, int n, int lane, float *sink) {
    float acc = 0.0f;
    for (int i = lane * 4; i < n; i += 256) acc += *(const float *)(p + i);
    if (acc == 1.0e-30f) *sink = acc;
}

__device__ __forceinline__ float gelu_of(ctok &a, float x) {
    if (a.gelu_clamp && x <= -10.0f) return 0.0f;
    if (a.gelu_clamp && x >= 10.0f) return x;
    return h2f(a.gelu_tab[f2h(x)]);
}

// the args live in device memory and are re-read (scalar cache) where used: an opaque copy of the
// pointer per use stops the compiler from hoisting ~30 pointers into registers for the whole launch
__device__ __forceinline__ ctok *fresh(const tok_args *p) {
    asm volatile("" : "+s"(p));
    return (ctok *)p;
}

template <int WT, int NR, int NRQ, int E, int F>
__global__ void __launch_bounds__(TK_NTH) k_token(const tok_args *ap) {
    extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
    using ST = tk_stash<WT>;
    using LY = tok_layout<WT, NR, E, F>;
    constexpr int BT = wfmt<WT>::BT, SB = wfmt<WT>::SCALE_BYTES;
    constexpr int NBE = LY::NBE, NBF = LY::NBF, NRD = NBF / TK_TW;
    constexpr lds_map m_e = tok_map(LY::E_ACT, LY::E_NS, LY::E_DA);
    constexpr lds_map m_f = tok_map(LY::F_ACT, LY::F_NS, LY::F_DA);
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    // per-lane values are re-derived from an opaque copy of the thread index at every phase: the
    // compiler would otherwise hoist every phase's per-lane LDS addresses out of the layer loop and
    // keep them all live (spills at the 168-VGPR budget of a 12-wave workgroup)
    int tid = threadIdx.x, lane = tid & 63, rr = lane >> 3, l = lane & 7, atid = tid - TK_TW * 64;
    const int c = blockIdx.x, G = gridDim.x;
    const bool term = wave < TK_TW, carrier = wave == TK_TW, aux = !term;
    uint8_t *img = smem + LY::IMG;
    float *xf = (float *)(smem + LY::XF);
    uint8_t *small = smem + LY::SMALL;
    float *hbuf = (float *)(small + SM_H), *sa8 = (float *)(small + SM_SA);
    double *red = (double *)(small + SM_RED);
    bool *fail = (bool *)(small + SM_FAIL);
    float *sink = (float *)(small + SM_SINK);
    if (tid == 0) *fail = false;
    const uint32_t ep = *fresh(ap)->epoch;
    const int n_layer = fresh(ap)->n_layer;
    auto LT = [&](int layer) -> const tok_layer & { return *((const tok_layer *)(small + SM_TAB) + layer); };
    auto fresh_lane = [&]() {
        asm volatile("" : "+v"(tid));
        lane = tid & 63;
        rr = lane >> 3;
        l = lane & 7;
        atid = tid - TK_TW * 64;
    };

    const int nq = c + G < fresh(ap)->qkv_rows / 8 ? 2 : 1;  // qkv row tiles of this workgroup
    const int per_layer = nq * NRQ + NRQ + 2 * NBE + NRD;      // ring tiles per term wave per layer
    unsigned long long *const dbg = GHIP_STAMPS ? fresh(ap)->dbg_t : nullptr;  // stamps build only
#define TK_STAMP(L, i) \
    if (GHIP_STAMPS && tid == 0 && dbg) dbg[((int64_t)c * n_layer + (L)) * 16 + (i)] = __builtin_amdgcn_s_memrealtime()

    // ---- the term wave's weight ring ------------------------------------------------------------
    const uint32_t ring0 = lds_u32(smem + LY::RING) + (uint32_t)(term ? wave : 0) * NR * TK_SLOT;
    int i_layer = 0, i_k = 0;  // issue cursor (wave-uniform)
    // the next tile's source addresses, prepared one refill ahead: the pointer-table read and the
    // address arithmetic overlap the tile compute instead of stalling the refill (~0.25 us each)
    const uint8_t *nx_q = nullptr, *nx_s = nullptr;
    auto prep = [&]() {
        const bool past = i_layer >= n_layer;
        const int layer = past ? n_layer - 1 : i_layer;
        int k = past ? per_layer - 1 : i_k;  // past the end: re-read the last tile
        int tile, mat;  // mat: 0 qkv, 1 o, 2 gate, 3 up, 4 down (tok_layer's pointer pairs)
        if (k < nq * NRQ) {
            const int j = NRQ == 1 ? k : k / NRQ, r = NRQ == 1 ? 0 : k % NRQ;
            tile = (j == 0 ? c : c + G) * NBE + wave + TK_TW * r;
            mat = 0;
        } else if ((k -= nq * NRQ) < NRQ) {
            tile = c * NBE + wave + TK_TW * k;
            mat = 1;
        } else if ((k -= NRQ) < 2 * NBE) {
            tile = (8 * c + wave) * NBE + (k >> 1);
            mat = 2 + (k & 1);
        } else {
            k -= 2 * NBE;
            tile = c * NBF + wave + TK_TW * k;
            mat = 4;
        }
        const uint64_t *tp = (const uint64_t *)(small + SM_TAB + layer * TK_TABB) + 2 * mat;
        nx_q = (const uint8_t *)tp[0] + (size_t)tile * 1024 + lane * 16;
        nx_s = (const uint8_t *)tp[1] + (size_t)tile * 8 * SB + lane * 16;
        if (++i_k == per_layer) {
            i_k = 0;
            ++i_layer;
        }
    };
    // ring state (wave-uniform): tiles issued / popped so far; tile t lives in slot t % NR.  A slot
    // is refilled (tile t + NR) only after tile t was popped.  Refills of tiles the current phase
    // still needs go out at once; the others wait for the phase's end (flush), where the term wave
    // idles at an edge anyway: a DMA issue costs a computing wave ~0.2 us.
    int issued = 0, popped = 0, islot = 0, slot = 0, phase_end = 1 << 30;
    auto issue_next = [&]() {  // the prepared tile into its slot, then prepare the next
        const uint32_t dst = ring0 + (uint32_t)islot * TK_SLOT;
        dma16(nx_q, dst);
        if (lane < SB / 2) dma16(nx_s, dst + 1024);  // 8 rows x SB bytes
        prep();
        ++issued;
        islot = islot + 1 == NR ? 0 : islot + 1;
    };
    auto flush = [&]() {  // every free slot refilled (after the reads of the popped tiles)
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        while (issued < popped + NR) issue_next();
    };
    // TK_DEFER 0: every pop refills at once (measured faster: the flushes at the edges slowed the
    // gathers that share the CU's memory pipe)
    auto begin_phase = [&](int pops) { phase_end = TK_DEFER ? popped + pops : 1 << 30; };
    int stamp_layer = 0;
    int pop_i = 0;  // stamps build: per-pop timing of workgroup 0's wave 0 (layer 1)
    auto pstamp = [&](int k) {
        if (GHIP_STAMPS && c == 0 && wave == 0 && lane == 0 && stamp_layer == 1 && pop_i < 64 && dbg)
            dbg[(int64_t)G * n_layer * 16 + pop_i * 4 + k] = __builtin_amdgcn_s_memrealtime();
    };
    // pop the next tile: its 16 B of quants and its row's scales for this lane
    auto pop = [&](uint4 &q, uint4 &s) {
        pstamp(0);
        if (issued < phase_end && issued < popped + NR) {
            asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // the previous pop's reads done
            do issue_next();
            while (issued < phase_end && issued < popped + NR);
        }
        pstamp(1);
        // tiles popped+1 .. issued-1 may stay in flight: 2 DMA instructions each
        switch (issued - popped - 1) {
#define TK_VM(n) case n: asm volatile("s_waitcnt vmcnt(%0)" ::"n"(2 * n) : "memory"); break;
            TK_VM(0) TK_VM(1) TK_VM(2) TK_VM(3) TK_VM(4) TK_VM(5) TK_VM(6) TK_VM(7) TK_VM(8) TK_VM(9) TK_VM(10)
            TK_VM(11) TK_VM(12) TK_VM(13) TK_VM(14) TK_VM(15)
#undef TK_VM
            default: asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        }
        pstamp(2);
        const uint8_t *p = smem + LY::RING + (wave * NR + slot) * TK_SLOT;
        q = *(const uint4 *)(p + lane * 16);
        if (WT == T_Q4_0) {
            s = *(const uint4 *)(p + 1024 + rr * 16);
        } else {
            const uint2 v = *(const uint2 *)(p + 1024 + rr * 8);
            s = make_uint4(v.x, v.y, 0, 0);
        }
        ++pop_i;
        ++popped;
        slot = slot + 1 == NR ? 0 : slot + 1;
    };
    // the ring's address table into LDS, and layer 0's x = the embedding row (every workgroup: the
    // norm needs all of it), both read before the ring's first DMAs so that no wait for these loads
    // also waits for the ring
    {
        const uint64_t *src = (const uint64_t *)fresh(ap)->layers;
        uint64_t *tab = (uint64_t *)(small + SM_TAB);
        for (int i = tid; i < n_layer * (TK_TABB / 8); i += TK_NTH) tab[i] = src[i];
    }
    {
        ctok &a = *fresh(ap);
        const int tok = a.hist[*a.pos];
        for (int i = tid; i < E; i += TK_NTH)
            xf[i] = emb_value<WT>(a.emb_qs, a.emb_sc, a.emb_n_bt, tok, i >> 5, i & 31) * a.emb_scale;
    }
    lds_barrier();
    if (term) {
        prep();
        for (int k = 0; k < NR; ++k) issue_next();
    }

    // ---- round-pipelined matvec phase (k_matvec_rr's arithmetic): nround rounds of 8 tiles, a row
    // tile every per_rt rounds; the carrier chains round r-1 while the term waves stash round r
    auto slot_base = [&](int r) { return smem + LY::STASH + (r & 1) * ST::SLOT; };
    auto rr_phase = [&](int nround, int per_rt, const lds_map &m, auto nsa, auto epi) {
        constexpr bool NSA = decltype(nsa)::value;
        if (term) {
            begin_phase(nround);
            for (int r = 0; r < nround; ++r) {
                uint4 q, s;
                pop(q, s);
                const int bt = wave + TK_TW * (r % per_rt);
                uint8_t *sb = slot_base(r);
                if constexpr (ST::I16)
                    terms16<NSA>(q, s, img, m, bt, l, (int16_t *)sb + lane * ST::SBP + wave * BT,
                                 (float *)(sb + ST::S_BYTES) + rr * ST::SBPD + wave * BT);
                else
                    tile_terms<WT>(q, s, img, m, bt, l, (float *)sb + lane * ST::SBP, (float *)(sb + ST::S_BYTES) + rr * ST::SBPD,
                                   wave * BT);
                if (nround > 4 && r == 0) TK_STAMP(stamp_layer, 14);
                if (nround > 4 && r == nround - 1) TK_STAMP(stamp_layer, 15);
                lds_barrier();
            }
            flush();  // the phase's deferred refills: the term waves idle at the next edge
        } else {
            if (carrier) __builtin_amdgcn_s_setprio(3);
            float acc = 0.0f;
            for (int r = 0; r <= nround; ++r) {
                if (r > 0 && carrier) {
                    const int rc = r - 1;
                    const uint8_t *sb = slot_base(rc);
                    const float4 *pd = (const float4 *)((const float *)(sb + ST::S_BYTES) + rr * ST::SBPD);
                    if constexpr (ST::I16) {
                        const uint4 *ps = (const uint4 *)((const int16_t *)sb + lane * ST::SBP);
                        acc = carry_ring<true>(ps, pd, ST::RUN / 8, acc);
                    } else {
                        const uint4 *ps = (const uint4 *)((const float *)sb + lane * ST::SBP);
                        acc = carry_ring<false>(ps, pd, ST::RUN / 4, acc);
                    }
                    if ((rc + 1) % per_rt == 0) {
                        const float v = fold8(acc);
                        acc = 0.0f;
                        if (l == 0) epi(rc / per_rt, v);
                    }
                }
                if (r < nround) lds_barrier();
            }
            if (carrier) __builtin_amdgcn_s_setprio(0);
        }
    };

    for (int il = 0; il < n_layer; ++il) {
        fresh_lane();
        stamp_layer = il;
        TK_STAMP(il, 0);
        // ---- x: layer 0's embedding (above) or the previous layer's down outputs
        norm_w<E> nw;
        if (aux) {
            nw.load(atid, LT(il).attn_norm);
            if (il > 0) {  // probe: the pair holding each producer's last row (8c+6, 8c+7)
                probe(atid, fail, *fresh(ap), fresh(ap)->gx, E, 3, 4, E / 8, tag_of(ep, il, EDGE_X), 1, il);
                gather<4>(atid, fail, *fresh(ap), fresh(ap)->gx, E, tag_of(ep, il, EDGE_X), (uint32_t *)xf, nullptr, 1, il);
            }
        }
        lds_barrier();
        TK_STAMP(il, 1);
        fresh_lane();
        norm_quant<WT, E>(aux, atid, xf, nw, fresh(ap)->eps, img, m_e, red);
        lds_barrier();
        TK_STAMP(il, 2);
        fresh_lane();
        // ---- q|k|v rows -> granules
        {
            const uint32_t tg = tag_of(ep, il, EDGE_QKV);
            rr_phase(nq * NRQ, NRQ, m_e, std::true_type{}, [&](int j, float v) {
                const int row = (j == 0 ? c : c + G) * 8 + rr;
                put_granule(fresh(ap)->gqkv + row, tg, __builtin_bit_cast(uint32_t, v));
            });
        }
        if (carrier) {
            touch_l2(LT(il).ffn_norm, E, lane, sink);
            // this workgroup's 1/32 of the gelu table (workgroups c, c+8, ... share an XCD's L2)
            touch_l2((const float *)fresh(ap)->gelu_tab + (c >> 3) * 1024, 1024, lane, sink);
        }
        TK_STAMP(il, 3);
        fresh_lane();
        // ---- attention (the first H*S workgroups of XCD-class 0: the K/V rows of a kv head are
        // read through one L2)
        {
            ctok &a = *fresh(ap);
            const int S = a.att_split, slotc = c >> 3;
            if ((c & 7) == 0 && slotc < a.H * S) {
                const int h = slotc / S, sp = slotc % S, Gq = a.H / a.Hkv, kvh = h / Gq;
                float *qkvl = (float *)(img + LY::ATT_QKV(a.ctx));
                const uint32_t tg = tag_of(ep, il, EDGE_QKV);
                const int qo = h * a.hd, ko = a.H * a.hd + kvh * a.hd, vo = a.H * a.hd + a.Hkv * a.hd + kvh * a.hd;
                if (aux) {
                    gather<1>(atid, fail, a, a.gqkv + qo, a.hd, tg, (uint32_t *)qkvl + qo, nullptr, 2, il);
                    gather<1>(atid, fail, a, a.gqkv + ko, a.hd, tg, (uint32_t *)qkvl + ko, nullptr, 2, il);
                    gather<1>(atid, fail, a, a.gqkv + vo, a.hd, tg, (uint32_t *)qkvl + vo, nullptr, 2, il);
                }
                lds_barrier();
                TK_STAMP(il, 4);
                attn_args at{};
                at.qkv = qkvl;
                at.kc = LT(il).kc;
                at.vc = LT(il).vc;
                at.rope_cur = a.rope_cur;
                at.exp_tab = a.exp_tab;
                at.pos = a.pos;
                at.out = a.att_out;
                at.out_gran = a.gatt;
                at.out_gran_da = a.gatt_da;
                at.gran_tag = tag_of(ep, il, EDGE_ATT);
                at.dsplit = S;
                at.H = a.H; at.Hkv = a.Hkv; at.hd = a.hd; at.ctx = a.ctx;
                at.q_scale = a.q_scale;
                at.mode = ATTN_PER_HEAD;
                attn_head_dev<TK_NTH, false, AH_KPF, AH_VPF, false>(at, h, img, nullptr, sp, tid);
                lds_barrier();
                TK_STAMP(il, 5);
            }
        }
        fresh_lane();
        // ---- attention output image -> LDS; o rows, sa = o + x -> granules
        if (aux) {
            ctok &a = *fresh(ap);
            const uint32_t tg = tag_of(ep, il, EDGE_ATT);
            // the block scales first (two per attention workgroup: the probe), then the image
            gather<1>(atid, fail, a, a.gatt_da, E / 32, tg, (uint32_t *)(img + m_e.da), nullptr, 3, il);
            gather<1>(atid, fail, a, a.gatt, E / 4, tg, (uint32_t *)(img + m_e.act), WT == T_Q4_0 ? (uint32_t *)(img + m_e.ns) : nullptr,
                      3, il);
        }
        lds_barrier();
        TK_STAMP(il, 6);
        fresh_lane();
        {
            const uint32_t tg = tag_of(ep, il, EDGE_SA);
            rr_phase(NRQ, NRQ, m_e, std::true_type{}, [&](int, float v) {
                const int row = c * 8 + rr;
                const float s = v + xf[row];  // ggml_add(attn-out, inpL)
                sa8[rr] = s;
                put_granule(fresh(ap)->gsa + row, tg, __builtin_bit_cast(uint32_t, s));
            });
        }
        TK_STAMP(il, 7);
        fresh_lane();
        // ---- sa -> ffn norm -> gate/up
        norm_w<E> fw;
        if (aux) {
            fw.load(atid, LT(il).ffn_norm);
            probe(atid, fail, *fresh(ap), fresh(ap)->gsa, E, 3, 4, E / 8, tag_of(ep, il, EDGE_SA), 4, il);
            gather<4>(atid, fail, *fresh(ap), fresh(ap)->gsa, E, tag_of(ep, il, EDGE_SA), (uint32_t *)xf, nullptr, 4, il);
        }
        lds_barrier();
        TK_STAMP(il, 8);
        fresh_lane();
        norm_quant<WT, E>(aux, atid, xf, fw, fresh(ap)->eps, img, m_e, red);
        lds_barrier();
        TK_STAMP(il, 9);
        fresh_lane();
        if (term) {
            float accg = 0.0f, accu = 0.0f;
            begin_phase(2 * NBE);
            for (int bt = 0; bt < NBE; ++bt) {
                uint4 qg, sg, qu, su;
                if (bt == NBE - 3) TK_STAMP(il, 13);
                pop(qg, sg);
                pop(qu, su);
                const act_tile<WT> at = load_act<WT, true>(img, m_e, bt, l);
                accg = tile_dot_a<WT>(qg, sg, at, accg);
                accu = tile_dot_a<WT>(qu, su, at, accu);
            }
            const float vg = fold8(accg), vu = fold8(accu);
            if (l == 0) {  // gelu on the aux side: the table lookup is a load the ring would hold up
                hbuf[wave * 8 + rr] = vg;
                hbuf[64 + wave * 8 + rr] = vu;
            }
        } else if (carrier && il + 1 < n_layer) {
            touch_l2(LT(il + 1).attn_norm, E, lane, sink);
        }
        lds_barrier();
        TK_STAMP(il, 10);
        fresh_lane();
        if (term) flush();  // gate/up's deferred refills (down tiles first) while the aux waves hand h on
        // this workgroup's 64 rows of h = Q8_0 blocks 2c, 2c+1 -> granules; the h image -> LDS
        if (aux) {
            ctok &a = *fresh(ap);
            const uint32_t tg = tag_of(ep, il, EDGE_H);
            if (atid < 8) {
                const int bl = atid >> 2, q = atid & 3;
                float v[8];
#pragma unroll
                for (int j = 0; j < 8; ++j) {
                    const int row = bl * 32 + q * 8 + j;
                    v[j] = gelu_of(a, hbuf[row]) * hbuf[64 + row];  // gelu(gate) then ggml_mul by up
                }
                image_put_quad_gran(a.gh, a.gh_da, tg, (int64_t)2 * c + bl, q, v);
            }
            // the block scales first (one pair per producer: the probe), then the image
            gather<1>(atid, fail, a, a.gh_da, F / 32, tg, (uint32_t *)(img + m_f.da), nullptr, 5, il);
            gather<8>(atid, fail, a, a.gh, F / 4, tg, (uint32_t *)(img + m_f.act), nullptr, 5, il);
        }
        lds_barrier();
        TK_STAMP(il, 11);
        fresh_lane();
        // ---- down rows, x' = down + sa -> granules (the next layer's x)
        {
            const bool last = il + 1 == n_layer;
            const uint32_t tg = tag_of(ep, il + 1, EDGE_X);
            rr_phase(NRD, NRD, m_f, std::false_type{}, [&](int, float v) {
                const int row = c * 8 + rr;
                const float xv = v + sa8[rr];  // ggml_add(ffn_out, sa)
                if (last) fresh(ap)->x_out[row] = xv;
                else put_granule(fresh(ap)->gx + row, tg, __builtin_bit_cast(uint32_t, xv));
            });
        }
        TK_STAMP(il, 12);
    }
#undef TK_STAMP
    // the ring's trailing re-reads must land before the workgroup's LDS is released
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
}

template <int WT>
struct tok_cfg;
template <>
struct tok_cfg<T_Q4_0> {
    static constexpr int NR = 11, NRQ = 1;
};
template <>
struct tok_cfg<T_Q8_0> {
    static constexpr int NR = 11, NRQ = 2;
};
constexpr int TK_E = 2048, TK_F = 16384;  // the shapes the launch is built for (Gemma-2B)

int cu_count_tok() {
    static int n = -1;
    if (n < 0) {
        int dev = 0;
        hipDeviceProp_t p;
        n = (hipGetDevice(&dev) == hipSuccess && hipGetDeviceProperties(&p, dev) == hipSuccess) ? p.multiProcessorCount : 0;
    }
    return n;
}

template <int WT>
using tok_ly = tok_layout<WT, tok_cfg<WT>::NR, TK_E, TK_F>;

}  // namespace

tok_gran_sizes token_gran_sizes(int E, int F, int qkv_rows) {
    tok_gran_sizes s;
    s.gx = (size_t)E;
    s.gqkv = (size_t)qkv_rows;
    s.gatt = (size_t)E / 4;  // image dwords
    s.gatt_da = (size_t)E / 32;
    s.gsa = (size_t)E;
    s.gh = (size_t)F / 4;
    s.gh_da = (size_t)F / 32;
    return s;
}

std::string token_unsupported(int wtype, const tok_args &a) {
    if (wtype != T_Q4_0 && wtype != T_Q8_0) return "layer type not Q4_0 / Q8_0";
    if (a.E != TK_E || a.F != TK_F) return "built for E = 2048, F = 16384 (Gemma-2B)";
    const int G = a.E / 8;
    if (a.qkv_rows % 8 || a.qkv_rows / 8 > 2 * G || a.qkv_rows / 8 < G) return "qkv rows not within 1..2 row tiles per workgroup";
    if (a.hd % 32 || a.hd > 256 || a.H % a.Hkv || a.H * a.hd != a.E) return "head shape (H * hd must be E)";
    if (a.att_split < 1 || a.H * a.att_split > G / 8 || (a.hd / a.att_split) % 32) return "attention split";
    if (a.ctx % 32 || a.ctx > TK_MAXCTX) return "context > 1024";
    const bool fits = wtype == T_Q4_0 ? tok_ly<T_Q4_0>::att_fits(a.ctx, a.qkv_rows) : tok_ly<T_Q8_0>::att_fits(a.ctx, a.qkv_rows);
    if (!fits) return "attention scratch for this context does not fit the image region";
    if (a.qkv_rows % 2 || a.hd % 2) return "granule counts must be even";
    if (cu_count_tok() < G) return "fewer CUs than workgroups (all must be resident)";
    if (a.n_layer > TK_MAXL) return "more layers than the LDS address table holds";
    if (!a.layers || !a.epoch || !a.err || !a.x_out || !a.att_out || !a.gx || !a.gqkv || !a.gatt || !a.gatt_da || !a.gsa ||
        !a.gh || !a.gh_da || !a.hist || !a.pos || !a.rope_cur || !a.exp_tab || !a.gelu_tab || !a.emb_qs)
        return "buffers";
    return "";
}

// ap: the args in device memory (written by the engine at graph build, immutable afterwards)
int launch_token(int wtype, const tok_args &a, const tok_args *ap, hipStream_t s) {
    const std::string why = token_unsupported(wtype, a);
    if (!why.empty()) {
        set_error("token launch: " + why);
        return -1;
    }
    const void *fn;
    size_t lds;
    if (wtype == T_Q4_0) {
        fn = (const void *)k_token<T_Q4_0, tok_cfg<T_Q4_0>::NR, tok_cfg<T_Q4_0>::NRQ, TK_E, TK_F>;
        lds = tok_ly<T_Q4_0>::TOTAL;
    } else {
        fn = (const void *)k_token<T_Q8_0, tok_cfg<T_Q8_0>::NR, tok_cfg<T_Q8_0>::NRQ, TK_E, TK_F>;
        lds = tok_ly<T_Q8_0>::TOTAL;
    }
    if (lds > 160 * 1024) {
        set_error("token launch: LDS layout too large");
        return -1;
    }
    GHIP_CHECK(hipFuncSetAttribute(fn, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
    int nb = 0;  // one workgroup per CU must be admitted (the hand-offs need all of them resident)
    GHIP_CHECK(hipOccupancyMaxActiveBlocksPerMultiprocessor(&nb, fn, TK_NTH, lds));
    if (nb < 1) {
        set_error("token launch: the workgroup does not fit a CU");
        return -1;
    }
    const tok_args *arg = ap;
    void *args[] = {(void *)&arg};
    GHIP_CHECK(hipLaunchKernel(fn, dim3(a.E / 8), dim3(TK_NTH), args, lds, s));
    GHIP_CHECK(hipGetLastError());
    return 0;
}

}  // namespace ghip
