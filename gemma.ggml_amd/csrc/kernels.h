// kernels.h — launch wrappers for the gfx950 kernels (host-callable, no torch types).
#pragma once

#include <vector>

#include "common.h"

namespace ghip {

// ---- decode matvec (matvec.hip) ----------------------------------------------------------------
// Prologue: how the activation column is turned into the LDS Q8_0 image.
enum mv_pro : int {
    PRO_F32 = 0,    // x: f32[K] -> quantize_row_q8_0 (AVX2 semantics)
    PRO_NORM = 1,   // x: f32[K] -> rms_norm(x)*norm_w (A.5) -> quantize
    PRO_Q8 = 2,     // x: ggml block_q8_0[K/32] (the C-ABI `wdata`, already converted by ggml INIT)
    PRO_EMBED = 3,  // x: int32 sequence, token = x[*tok_pos]; embedding row (tiled) * emb_scale -> norm
    PRO_IMG = 4,    // x: the Q8_0 activation image its producer already wrote (act u32 [nb/4][8][4]
                    //    + x_da f32 [nb]; DESIGN.md §Activation image): a copy into LDS
};
enum mv_epi : int {
    EPI_STORE = 0,     // y[r] = dot
    EPI_ADD = 1,       // y[r] = dot + resid[r]          (ggml_add, src/gemma_model.cpp:723,731)
    EPI_GELU_MUL = 2,  // y[r] = gelu(dotA) * dotB       (src/gemma_model.cpp:446-449)
    EPI_ARGMAX = 3,    // y[r] = dot and argmax key      (greedy_sample, :532-546)
};

struct mv_args {
    const uint8_t *qs = nullptr, *sc = nullptr;    // weights (tiled)
    const uint8_t *qs2 = nullptr, *sc2 = nullptr;  // second matrix for EPI_GELU_MUL (ffn_up)
    int64_t rows = 0, n_rt = 0, n_bt = 0, nb = 0;  // nb = K/32
    const void *x = nullptr;                       // activation (see mv_pro)
    const float *x_da = nullptr;                   // PRO_IMG: the image's block scales
    int64_t x_col_stride = 0;                      // bytes between columns (multi-column launch)
    const float *norm_w = nullptr;
    float eps = 0.f;
    // PRO_EMBED: embedding source
    const int *tok_pos = nullptr;
    const uint8_t *emb_qs = nullptr, *emb_sc = nullptr;
    int64_t emb_n_bt = 0;
    float emb_scale = 1.f;
    float *emb_out = nullptr;                      // if set, block 0 writes the scaled embedding row
    // epilogue
    float *y = nullptr;
    int64_t y_col_stride = 0;                      // floats between columns
    const float *resid = nullptr;
    const uint16_t *gelu_tab = nullptr;
    int gelu_clamp = 0;
    unsigned long long *argmax_key = nullptr;      // EPI_ARGMAX: one partial key per workgroup [grid]
    uint32_t *out_act = nullptr;                   // EPI_GELU_MUL: also write y's Q8_0 image (the
    float *out_da = nullptr;                       //   next matvec's PRO_IMG input), blocks of y
    int ncols = 1;
    int ablate = 0;  // timing-only ablations (bench): 1 = no prologue, 4 = no carry, 8 = no gate/up dots
    unsigned long long *dbg_t = nullptr;  // diagnostics: 8 s_memrealtime stamps per workgroup
    // launch geometry precomputed by launch_t (no 64-bit divisions in the kernel prologue):
    // a wave's row-tile count is rt_q + (rt0 < rt_r); ygroups = EPI_GELU_MUL image groups per WG
    int64_t rt_q = 0, rt_r = 0, ygroups = 0;
};

// ks: waves that split one row tile's K range (ordered carry hand-off); 1 = one wave per tile.
// ks = KS_RR: the round-pipelined form (matvec_rr.hip): 8 loader waves interleaved over K + a carrier
// wave that runs the chains one round behind the loads; one workgroup per row tile (grid_x ignored).
constexpr int KS_RR = 9;
int launch_matvec(int wtype, int ks, int pro, int epi, const mv_args &a, int grid_x, hipStream_t s);
bool matvec_rr_supported(int wtype, int64_t n_bt);
size_t matvec_lds_bytes(int wtype, int ks, int64_t n_bt, int64_t segment_tiles);

// ---- ggml graph executor kernels (ggml_ops.hip) ----------------------------------------------------
struct gt_desc {  // a device view of a ggml tensor: data, ne, nb (bytes), type
    char *data = nullptr;
    int64_t ne[4] = {1, 1, 1, 1};
    int64_t nb[4] = {0, 0, 0, 0};
    int type = T_F32;
};
int launch_g_get_rows(const gt_desc &src, const gt_desc &idx, const gt_desc &dst, hipStream_t s);
int launch_g_elementwise(int op, const gt_desc &a, const gt_desc &b, const gt_desc &dst, float scale,
                         const uint16_t *gelu_tab, int gelu_clamp, hipStream_t s);
int launch_g_rms_norm(const gt_desc &a, const gt_desc &dst, float eps, hipStream_t s);
int launch_g_rope_neox(const gt_desc &a, const gt_desc &pos, const gt_desc &dst, int n_dims, const float *cs,
                       const float *sn, hipStream_t s);
int launch_g_soft_max(const gt_desc &a, const gt_desc &mask, int has_mask, const gt_desc &dst, float scale, hipStream_t s);
int launch_g_copy(const gt_desc &src, const gt_desc &dst, hipStream_t s);
int launch_g_mul_mat_f16(const gt_desc &a, const uint16_t *b16, int64_t ne10, const gt_desc &dst, int64_t ne11,
                         int64_t ne12, int64_t ne13, hipStream_t s);
// host tables and tiled weights shared with the engine (engine.cpp)
void build_f16_tables(std::vector<uint16_t> &exp_t, std::vector<uint16_t> &gelu_t);
void build_rope(int ctx, int hd, float base, std::vector<float> &c, std::vector<float> &s);
tiled_mat alloc_tiled(int type, int64_t rows, int64_t K, hipStream_t s);
// capi.cpp: the C-ABI weight cache's tiled copy of a host weight (hpc_register_weight / mul_mat)
bool registered_tiled(const void *host, int type, int64_t K, tiled_mat *out);
void free_tiled(tiled_mat &m);

// ---- K-quant matvec (kquant.hip) -----------------------------------------------------------------
struct kq_args {  // y[c][r] = vec_dot_{q4_K,q6_K}_q8_K(row r of w, column c of x), ggml AVX2 lane order
    const uint8_t *w = nullptr;   // ggml row-major super-blocks, row_bytes per row
    int64_t row_bytes = 0, rows = 0;
    int nsb = 0;                  // super-blocks per row (K / 256)
    const uint8_t *x = nullptr;   // Q8_K columns (292 B per super-block), x_col_stride bytes apart
    int64_t x_col_stride = 0;
    float *y = nullptr;
    int64_t y_col_stride = 0;     // floats between output columns
    int ncols = 1;
    // epilogue (engine K-quant layers): y = v + resid (ggml_add), or y = gelu(gate_in) * v (ffn_up)
    const float *resid = nullptr, *gate_in = nullptr;
    const uint16_t *gelu_tab = nullptr;
    int gelu_clamp = 0;
    // fused INIT (no separate Q8_K launch): pro = KQP_F32 quantizes f32 columns xf, KQP_NORM
    // quantizes rms_norm(xf)*norm_w (k_norm_q8K's bytes); KQP_COPY reads the Q8_K columns x
    int pro = 0;
    const float *xf = nullptr;
    int64_t xf_col_stride = 0;    // floats
    const float *norm_w = nullptr;
    float eps = 0.f;
    // fused ffn gate/up: w = gate, w2 = up (same type and shape), y = gelu(gate) * up
    const uint8_t *w2 = nullptr;
    // producer-side INIT of the NEXT matvec (y stored write-through, then a per-wave count):
    // q8_mode = KQO_QUANT: each 256-row super-block of y quantized to Q8_K by the wave completing it;
    // KQO_NORM: rms_norm(y)*q8_norm (eps) quantized by the wave completing the whole column.
    // q8_out: Q8_K columns ((rows/256)*292 B apart); q8_cnt: zero-initialised counters, 32 u32 apart,
    // q8_cnt_cap of them per launch (left zero)
    int q8_mode = 0;
    uint8_t *q8_out = nullptr;
    unsigned *q8_cnt = nullptr;
    int q8_cnt_cap = 0;
    const float *q8_norm = nullptr;
    int q8_abl = 0;  // timing ablation only (wrong bytes): 1 no tail work, 2 no counting, 4 plain stores
    int tiled = 0;   // w (and w2) in the lane-contiguous layout of launch_kq_retile
    unsigned long long *dbg_t = nullptr;  // stamps build: 16 s_memrealtime per workgroup (k_matvec_kq)
};
// ggml K-quant rows <-> the lane-contiguous device layout the matvec reads with one vector load per
// lane (Q4_K any K % 256 == 0, Q6_K K % 2048 == 0); src != dst
int launch_kq_retile(int wtype, const uint8_t *src, uint8_t *dst, int64_t rows, int64_t K, bool to_tiled, hipStream_t s);
enum kq_prologue_mode { KQP_COPY = 0, KQP_F32 = 1, KQP_NORM = 2 };
enum kq_handoff_mode { KQO_NONE = 0, KQO_QUANT = 1, KQO_NORM = 2 };
int launch_matvec_kq(int wtype, const kq_args &a, hipStream_t s);
// two K-split matvecs over one input column in one launch (e.g. q|k and v; types may differ)
int launch_matvec_kq2(int t1, const kq_args &a, int t2, const kq_args &b, hipStream_t s);
// ggml quantize_row_q8_K of ncols rows of K floats (row stride ldx floats) -> Q8_K rows ld_out bytes apart
int launch_quant_q8_K(const float *x, int64_t ldx, int64_t K, int ncols, uint8_t *out, int64_t ld_out,
                      hipStream_t s);
// rows of rms_norm(x)*w quantized to Q8_K (the tied output's INIT when token_embd is Q6_K)
int launch_norm_q8K(const float *x, int64_t ldx, const float *w, int E, float eps, int rows, uint8_t *out,
                    int64_t ld_out, hipStream_t s);
// T rows of get_rows(Q6_K token_embd, tokens)*scale; token of row t: tokens[*pos] if pos else tokens[t]
int launch_embed_q6K(const uint8_t *embd, int64_t row_bytes, const int *tokens, const int *pos, int T, int E,
                     float scale, float *out, hipStream_t s, bool tiled = false);
// synthetic Q4_K / Q6_K rows: oracle orc_synth_kquant(seed) with d (and dmin) rescaled by f
int launch_synth_kquant(int wtype, uint8_t *out, int64_t rows, int64_t K, uint64_t seed, float f, hipStream_t s);

// ---- K-quant prefill GEMM (prefill_kq.hip) -------------------------------------------------------
// T Q8_K columns -> the operand image of k_gemm_kq: xh f16 [T][ldh] with each super-block's 256
// values in AVX2-lane-major order (position 32l + 4c + k holds value 32c + 4l + k), xd f32 [T][ldd]
// (the super-block's d), xm [T][ldm][16] f16 (Q4_K mins operand: per k = 0..3 the pair sums
// S0 = bs[4k]+bs[4k+1], S1 = bs[4k+2]+bs[4k+3] as S & 63, S1 & 63, S0 >> 6, S1 >> 6)
struct q8kx_args {
    const uint8_t *x = nullptr;
    int64_t x_col_stride = 0;
    int nsb = 0, T = 0;
    uint16_t *xh = nullptr;
    int64_t ldh = 0;
    float *xd = nullptr;
    int64_t ldd = 0;
    uint16_t *xm = nullptr;
    int64_t ldm = 0;
};
int launch_q8k_expand(const q8kx_args &a, hipStream_t s);
// y[t][r] = vec_dot_{q4_K,q6_K}_q8_K(row r, column t) for all T columns, ggml AVX2 lane order, on
// v_mfma_f32_32x32x16_f16
struct kqg_args {
    const uint8_t *w = nullptr;
    int64_t row_bytes = 0, rows = 0;
    int nsb = 0, T = 0;
    int tiled = 1;  // w in launch_kq_retile's layout (Q6_K: K % 2048 == 0), else ggml's row-major blocks
    const uint16_t *xh = nullptr;
    int64_t ldh = 0;
    const float *xd = nullptr;
    int64_t ldd = 0;
    const uint16_t *xm = nullptr;
    int64_t ldm = 0;
    float *y = nullptr;
    int64_t ldy = 0;
    // epilogue as kq_args: y = v + resid, or y = gelu(gate_in) * v
    const float *resid = nullptr, *gate_in = nullptr;
    const uint16_t *gelu_tab = nullptr;
    int gelu_clamp = 0;
};
int launch_gemm_kq(int wtype, const kqg_args &a, hipStream_t s);
// the column count from which K-quant mul_mats (C-ABI, graph executor, engine prefill) take
// launch_gemm_kq: GHIP_KQ_MFMA_MIN (default 8; GHIP_KQ_MFMA=0 disables), or hpc_set_kq_gemm_min
int kq_gemm_min();
void set_kq_gemm_min(int v);

// ---- prefill (prefill.hip) ----------------------------------------------------------------------
enum qrow_mode { QR_F32 = 0, QR_NORM = 1, QR_EMBED_NORM = 2, QR_GELU = 3 };
struct qrow_args {  // T rows of K floats -> Q8_0 image q [T][ldq] int8 + da [T][ldd] (f32 of fp16 d)
    const float *x = nullptr, *x2 = nullptr;  // rows (stride ldx); x2 = `up` for QR_GELU (x = gate)
    int64_t ldx = 0, K = 0;
    const float *norm_w = nullptr;
    float eps = 0.f;
    const int *tokens = nullptr;              // QR_EMBED_NORM: token ids; embedding table (tiled)
    const uint8_t *emb_qs = nullptr, *emb_sc = nullptr;
    int emb_type = 0;
    int64_t emb_n_bt = 0;
    float emb_scale = 1.f;
    float *emb_out = nullptr;                 // scaled embedding rows (the residual stream), stride ldx
    const uint16_t *gelu_tab = nullptr;
    int gelu_clamp = 0;
    int8_t *q = nullptr;                      // int8 image (nullptr: not written)
    uint16_t *qh = nullptr;                   // optional f16 image of the same values (exact GEMM)
    int64_t ldq = 0;                          // multiple of 256 (zero padded)
    float *da = nullptr;
    int64_t ldd = 0;                          // >= ldq / 32
};
int launch_quant_rows(int mode, const qrow_args &a, int T, hipStream_t s);
struct gemm_args {  // Y[t][r] (stride ldy) = W (tiled) x Xq[t] (+ resid), t < T, r < rows
    const uint8_t *qs = nullptr, *sc = nullptr;
    int64_t rows = 0, n_rt = 0, n_bt = 0, nb = 0;
    const int8_t *xq = nullptr;
    const uint16_t *xh = nullptr;  // f16 image of xq (the exact GEMM's MFMA operand), same stride
    int64_t ldq = 0;
    const float *da = nullptr;
    int64_t ldd = 0;
    int64_t T = 0;
    float *y = nullptr;
    const float *resid = nullptr;
    int64_t ldy = 0;
};
int launch_gemm_q(int wtype, int epi, const gemm_args &g, hipStream_t s);
// the same product in ggml's AVX2 lane order (bit-identical to mul_mat)
int launch_gemm_exact(int wtype, int epi, const gemm_args &g, hipStream_t s);
bool gemm_x4_i8();        // mode 3: k_gemm_x4 stages the activation from the int8 image (xq)
bool gemm_x4_on();        // the exact GEMM's form: the K = 4 multi-block MFMA kernel (k_gemm_x4) or W32
void set_gemm_x4(int v);

struct ropekv_args {  // RoPE q (-> f16, x q_scale) and k, store k/v of positions p0.. in the layer caches
    const float *qkv = nullptr;  // [T][ldqkv] = q | k | v
    int64_t ldqkv = 0;
    const float *rope_cos = nullptr, *rope_sin = nullptr;
    uint16_t *q16 = nullptr;     // [T][H][hd]
    uint16_t *kc = nullptr, *vc = nullptr;
    int H = 0, Hkv = 0, hd = 0, ctx = 0, p0 = 0;
    float q_scale = 1.f;
};
int launch_rope_kv_prefill(const ropekv_args &a, int T, hipStream_t s);
struct attnp_args {  // causal attention of T prompt tokens against the layer caches
    const uint16_t *q16 = nullptr;
    const uint16_t *kc = nullptr, *vc = nullptr;
    float *out = nullptr;        // [T][ldo], head h at h*hd
    int64_t ldo = 0;
    int T = 0, H = 0, Hkv = 0, hd = 0, ctx = 0, n_kv = 0;
};
int launch_attn_prefill(const attnp_args &a, hipStream_t s);
// exact rows: each prompt row with the decode attention's arithmetic (ops.hip)
int launch_attn_rows(const attnp_args &a, hipStream_t s);
// the same rows on the f32 matrix cores (attn_mx.hip): v_mfma_f32_16x16x4_f32 is an fmaf chain over K,
// so vec_dot_f16's 32 chains ride K four steps at a time; "" when it runs the shapes
const char *attn_mx_unsupported(const attnp_args &a);  // nullptr: the matrix-core form runs these shapes
int launch_attn_mx(const attnp_args &a, hipStream_t s);
// hipFuncAttributeMaxDynamicSharedMemorySize of a kernel raised to the CU's whole LDS, once per
// (slot, device), thread-safe: slots LDS_SLOT_*
enum { LDS_SLOT_ATTN_MX = 0, LDS_SLOT_GELU_LDS = 1, LDS_SLOTS = 2 };
int allow_full_lds(const void *fn, int slot);
int launch_row_argmax(const float *row, int64_t n, unsigned long long *keys, int parts, hipStream_t s);

// ---- weights (ops.hip) ------------------------------------------------------------------------
// ggml row-major blocks (host layout) already on device -> tiled layout
int launch_repack(const tiled_mat &m, const uint8_t *src_rowmajor, int64_t row_bytes, hipStream_t s);
// synthetic generator: same integer stream + reference quantizer as oracle/gemma_cpu.cpp
int launch_synth_tiled(const tiled_mat &m, uint64_t key, float scale, int64_t row_offset, hipStream_t s);
int launch_synth_norm(float *dst, int64_t n, uint64_t key, float scale, hipStream_t s);
int launch_untile(const tiled_mat &m, uint8_t *dst_rowmajor, hipStream_t s);

// ---- small decode ops (ops.hip) -----------------------------------------------------------------
enum attn_mode { ATTN_PER_HEAD = 0, ATTN_SPLIT = 1 };
struct attn_args {
    const float *qkv;       // [q(H*hd) | k(Hkv*hd) | v(Hkv*hd)] for one token
    uint16_t *kc, *vc;      // layer caches: K [ctx][Hkv*hd], V [Hkv*hd][ctx] (f16 bits)
    const float *rope_cos, *rope_sin;  // [ctx][hd/2]
    const float *rope_cur = nullptr;   // [cos | sin | (int)pos] of *pos (k_advance keeps it current)
    const uint16_t *exp_tab;
    const int *pos;         // device scalar (position of this token)
    float *out;             // [H*hd]
    uint32_t *out_act = nullptr;  // per-head mode: also out's Q8_0 image (attn-out's PRO_IMG input)
    float *out_da = nullptr;
    uint8_t *out_q8k = nullptr;   // per-head mode, hd == 256: out's Q8_K image (one super-block per head)
    int dsplit = 1;               // per-head mode: workgroups per head, each the KQV of hd/dsplit dims
    int H, Hkv, hd, ctx;
    float q_scale;
    float *dbg_w = nullptr;      // optional debug taps: [H][ctx] scores, [H][ctx] fp16 P, [H] inv
    uint16_t *dbg_p = nullptr;
    float *dbg_inv = nullptr;
    unsigned long long *dbg_t = nullptr;  // diagnostic phase stamps (s_memrealtime), [grid][8]
    int mode = 0;  // ATTN_PER_HEAD (one workgroup per head) or ATTN_SPLIT (long contexts)
    // split form: workgroups per kv head, scores scratch [Hkv][ctx][G], hand-off counters [Hkv][2]
    // (zero before the first launch; each launch leaves them zero), sticky error word
    int nwg = 0;
    float *sbuf = nullptr;
    int *sync = nullptr;
    int *err = nullptr;
    // per-head mode inside the persistent token launch: the output's Q8_0 image published as
    // {payload, tag} granules (act dwords in the image's dword order, block scales) instead of stores
    unsigned long long *out_gran = nullptr, *out_gran_da = nullptr;
    uint32_t gran_tag = 0;
};
// the front half of a decode layer in one launch (layer_front.hip): qkv (rr, PRO_NORM, EPI_STORE)
// -> per-head attention -> attn-out (rr, PRO_IMG from the attention's image, EPI_ADD)
struct front_args {
    mv_args q;
    attn_args t;
    mv_args o;
    unsigned *cnt = nullptr;  // this layer's hand-off counters [16], zero before the launch
    int *err = nullptr;       // sticky: a hand-off poll timed out
    unsigned long long *dbg_t = nullptr;  // diagnostics (stamps build): 16 s_memrealtime per workgroup
};
bool layer_front_supported(int wtype, const mv_args &q, const attn_args &t, const mv_args &o);
int launch_layer_front(int wtype, const front_args &f, hipStream_t s);
// the decode attention (per-head form) and attn-out (+ residual) in ONE launch (layer_front.hip
// k_attn_o): the attention launch's idle workgroups run attn-out's row tiles, weights in flight
// before the in-launch hand-off of the attention's Q8_0 image
struct attn_o_args {
    attn_args t;              // per-head attention, out_act / out_da set (the handed-off image)
    mv_args o;                // attn-out: PRO_IMG from t.out_act / t.out_da, EPI_ADD
    unsigned *cnt = nullptr;  // this layer's counters: 8 replicas + the consumers' done count, 128 B apart;
                              // zero before the launch, and the launch leaves them zero
    int *err = nullptr;       // sticky: a hand-off poll timed out (err[0]; err[1..4] diagnostics)
    unsigned long long *dbg_t = nullptr;  // stamps build: 16 s_memrealtime per workgroup
};
bool attn_o_supported(int wtype, const attn_args &t, const mv_args &o);
int launch_attn_o(int wtype, const attn_o_args &f, hipStream_t s);

// peer-to-peer all-gather (p2p.hip, GEMMA_TP_P2P): each rank pushes [rank*shard, +shard) of every
// segment's working vector into every peer's inbox (arena offset `inbox`), flags it, and copies
// the peers' shards out of its own inbox; peer[r] = rank r's arena in this process's address space
constexpr int P2P_MAX_RANKS = 8;
struct p2p_seg {
    uint8_t *work = nullptr;  // the full working vector (this rank's shard written by the producer)
    int64_t inbox = 0;        // its inbox's offset in every rank's arena (16-byte aligned)
    int64_t shard = 0;        // bytes per rank (multiple of 4)
};
struct p2p_args {
    p2p_seg seg[2];
    int nseg = 1;
    int rank = 0, n = 1;
    uint8_t *peer[P2P_MAX_RANKS] = {};
    int64_t flags = 0;        // arena offset of the u32 flag words, one per source rank
    unsigned *seq = nullptr;  // [0] gathers done, [1] workgroups finished in the current one (local)
    unsigned *err = nullptr;  // sticky: a flag wait timed out
};
int launch_p2p_gather(const p2p_args &a, hipStream_t s);

// ---- the whole decode token's layers as ONE persistent launch (token.hip) ----------
// per layer: device pointers of the tiled matrices, norms and KV caches (a table in device memory,
// read through the scalar cache: immutable for the launch)
struct tok_layer {
    const uint8_t *qkv_qs = nullptr, *qkv_sc = nullptr, *o_qs = nullptr, *o_sc = nullptr;
    const uint8_t *g_qs = nullptr, *g_sc = nullptr, *u_qs = nullptr, *u_sc = nullptr, *d_qs = nullptr, *d_sc = nullptr;
    const float *attn_norm = nullptr, *ffn_norm = nullptr;
    uint16_t *kc = nullptr, *vc = nullptr;
};
struct tok_args {
    const tok_layer *layers = nullptr;
    int n_layer = 0;
    int E = 0, F = 0, H = 0, Hkv = 0, hd = 0, ctx = 0, qkv_rows = 0;
    int att_split = 0;  // workgroups per query head (each the KQ / softmax and hd / att_split KQV dims)
    float eps = 0.f, emb_scale = 1.f, q_scale = 1.f;
    const uint8_t *emb_qs = nullptr, *emb_sc = nullptr;  // tied embedding (tiled, layer type)
    int64_t emb_n_bt = 0;
    const int *hist = nullptr, *pos = nullptr;
    const float *rope_cur = nullptr;
    const uint16_t *exp_tab = nullptr, *gelu_tab = nullptr;
    int gelu_clamp = 0;
    // in-launch hand-offs: 8-byte {payload, tag} granules (MI355X_MICROARCH handoff-1to1 / allgather)
    unsigned long long *gx = nullptr, *gqkv = nullptr, *gatt = nullptr, *gatt_da = nullptr, *gsa = nullptr,
                       *gh = nullptr, *gh_da = nullptr;
    const unsigned *epoch = nullptr;  // bumped by k_advance / k_set_position: tags are unique per token
    float *x_out = nullptr;           // the last layer's output x (the logits launch's input)
    float *att_out = nullptr;         // attention output scratch (written, unused)
    int *err = nullptr;               // [0] sticky hand-off timeout, [1] site, [2] layer
    unsigned timeout = 2000000u;      // per-wait bound in s_memrealtime ticks (100 MHz): 20 ms
    unsigned long long *dbg_t = nullptr;  // stamps build: [grid][n_layer][16] s_memrealtime
};
// granules each buffer holds for shapes (E, F, qkv_rows)
struct tok_gran_sizes {
    size_t gx, gqkv, gatt, gatt_da, gsa, gh, gh_da;
};
tok_gran_sizes token_gran_sizes(int E, int F, int qkv_rows);
// "" if the shapes / device allow the persistent token launch, else the reason
std::string token_unsupported(int wtype, const tok_args &a);
// a: the args on the host (checked), ap: the same args in device memory (what the kernel reads)
int launch_token(int wtype, const tok_args &a, const tok_args *ap, hipStream_t s);

struct attn_geom {
    int nwg = 0, grid = 0;
    int img = 0;  // the split form can write the output's Q8_0 image (32-dim KQV slices)
    size_t lds = 0, sbuf_floats = 0, sync_ints = 0;
};
attn_geom attn_geometry(int H, int Hkv, int hd, int ctx);
int launch_attn_decode(const attn_args &a, hipStream_t s);
int launch_embed(const uint8_t *qs, const uint8_t *sc, int wtype, int64_t n_bt, const int *token, float scale,
                 float *out, int64_t E, hipStream_t s);
// reduces the n_parts per-workgroup argmax keys, appends the token, advances the position
int launch_exp_f16_all(uint16_t *out, hipStream_t s);
int launch_stream_read(const void *buf, size_t bytes, unsigned *sink, hipStream_t s, int variant = 0);  // roofline probe  // the softmax's exp for all 65536 f16 codes (tests)
int launch_reduce_keys(const unsigned long long *keys, int n, int64_t row_base, unsigned long long *out, hipStream_t s);
struct rope_row {  // k_advance also publishes the new position's RoPE row: cur = [cos | sin | (int)pos]
    const float *cos = nullptr, *sin = nullptr;
    float *cur = nullptr;
    int half = 0, ctx = 0;
    unsigned *epoch = nullptr;  // if set, incremented (the persistent token launch's granule tags)
};
// read `n` weight regions with allocating loads (MALL warm-up for a later kernel), `grid` workgroups
int launch_advance(const unsigned long long *keys, int n_parts, int *token, int *pos, int *hist, int hist_cap,
                   const int *n_fixed, const rope_row &r, hipStream_t s);
int launch_set_position(int token, int p, int *pos, int *hist, int *n_fixed, int fixed, const rope_row &r, hipStream_t s);

// ---- generic ggml-op kernels used by the C-ABI and the ggml-compatible executor ----------------
int launch_mul_mat_f16(const uint16_t *src0, int64_t nb01_elems, int64_t ne01, const uint16_t *src1,
                       int64_t row_size_elems, int64_t ncols, int64_t K, float *dst, hipStream_t s);

}  // namespace ghip
