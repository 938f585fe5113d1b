/*
 * gemma_hpc.h — the C-ABI drop-in boundary of the MI355X hot path (libgemma_hip.so).
 *
 * Plain C types and pointers only; no torch types.  Every entry point names the reference
 * interface it replaces.  Host side: the reference's forked ggml calls `mul_mat` from
 * ggml_compute_forward_mul_mat's COMPUTE phase; the performance path keeps the
 * whole Gemma token on the device (gemma_engine_*, the `hpc_graph_compute` role of SURVEY §8(b)).
 */
#ifndef GEMMA_HPC_H
#define GEMMA_HPC_H

#include <stddef.h>
#include <stdint.h>

#include "ggml.h"

#ifdef __cplusplus
extern "C" {
#endif

/* ---- narrow drop-in: replaces src/hpc.h:22-32 / src/hpc.cpp:216-390 ------------------------
 * Same signature and argument meaning.  dst[(c % ne1)*nb1 + (c / ne1)*nb2 + r*4] =
 * vec_dot(shared_edge, src0 + r*nb01, wdata + c*row_size) for r < ne01, c < ne11*ne12, with the
 * dot computed on the GPU in ggml's AVX2 lane order (bit-identical to the CPU path).
 * src0_type: GGML_TYPE_Q4_0, GGML_TYPE_Q8_0 (wdata = block_q8_0 rows), GGML_TYPE_Q4_K /
 * GGML_TYPE_Q6_K (wdata = block_q8_K rows; ggml's AVX2 K-quant lane order) or GGML_TYPE_F16
 * (wdata = fp16 rows).  `vec_dot` is accepted for link compatibility and not called.
 * Quantized src0 is uploaded + re-tiled once and cached by (src0->data, shape) — weights are
 * immutable for the program's lifetime (src/gemma_model.cpp:24-27).  CONTRACT: a caller that
 * frees or rewrites a quantized src0 buffer calls hpc_unregister_weight(ptr) (or
 * hpc_flush_weights()) first; otherwise a later buffer at the same address gets the stale copy.
 * F16 src0 (KV-cache views) is uploaded on every call.  Errors: no return value (as the reference); the message is kept
 * for hpc_last_error() and, unless hpc_set_error_mode(0), the process exits(1) like
 * src/hpc.cpp:163-166 / src/opencl.cpp:13-17.                                                   */
void mul_mat(int64_t ne01, int64_t ne11, int64_t ne12, int64_t nb01, int64_t ne1, int64_t nb1, int64_t nb2,
             size_t row_size, int64_t shared_edge, struct ggml_tensor *src0, struct ggml_tensor *src1,
             struct ggml_tensor *dst, ggml_vec_dot_t vec_dot, enum ggml_type src0_type, const char *wdata);

/* ---- device-dispatch lifecycle: replaces src/opencl.h:22-38 (init_opencl, get_kernel,
 * create_buffer, enqueue_kernel, wait_queue_finish, release_buffer_in_set) -------------------- */
int hpc_init(int device);                 /* init_opencl (src/opencl.cpp:350-356); 0 = ok        */
void hpc_shutdown(void);                  /* frees the weight cache and the device scratch        */
int hpc_register_weight(const void *host, int type, int64_t ne00, int64_t ne01, size_t nb01);
int hpc_last_error(char *buf, size_t len);/* length of the last error message (0 = none)          */
void hpc_set_error_mode(int exit_on_error);
int hpc_weight_cache_entries(void);
int hpc_unregister_weight(const void *host); /* drop the cached device copies of `host`; returns the count */
void hpc_flush_weights(void);                /* drop every cached device weight                          */
void hpc_set_matvec_ks(int ks);          /* K-split of the quantized matvec (1/2/4/8; tests) */
/* columns from which K-quant mul_mats (and the K-quant engine prefill) run the MFMA GEMM
 * (prefill_kq.hip) instead of the dot4 kernels; -1 = GHIP_KQ_MFMA_MIN or 8 (tests: same bytes) */
void hpc_set_kq_gemm_min(int min_cols);
/* the exact Q4_0 / Q8_0 prefill GEMM's form: 1 (default) = K = 4 multi-block MFMA (k_gemm_x4, dense
   lane fragments, 32 rows x 64 tokens per workgroup), 2 = the same with 64 x 32, 0 = the lane-masked
   32x32x16 form (k_gemm_x); bit-identical every way */
void hpc_set_gemm_x4(int on);

/* ---- graph executor (SURVEY §8(b) `hpc_graph_compute(ggml_cgraph*)`): runs a graph built with the
 * ggml surface of include/ggml.h on the GPU; 0 = ok, else hpc_last_error() tells */
int hpc_graph_compute(struct ggml_cgraph *graph);

/* ---- device-resident Gemma engine (performance path: the Gemma graph encoded as one hipGraph) ---- */
typedef struct gemma_hip_config {
    int n_layer, n_embd, n_head, n_head_kv, head_dim, n_ff, n_vocab, n_ctx;
    int wtype; /* GGML_TYPE_Q4_0 or GGML_TYPE_Q8_0 (the layer matrices) */
    float eps, rope_base;
    uint64_t seed;
    int gelu_clamp;
    int out_type; /* token_embd / tied output: 0 = wtype, or GGML_TYPE_Q6_K (llama.cpp's Q4_0 / Q8_0 files) */
    float out_gain; /* synthetic weights: token_embd / output std x out_gain (0 = 1; SURVEY §8(d) uses 4 for
                       peaked logits in the Gemma-7B TP leg); ignored for GGUF weights */
} gemma_hip_config;

typedef struct gemma_engine gemma_engine;

gemma_engine *gemma_engine_create(const gemma_hip_config *cfg, int device);
/* real weights from a Gemma GGUF file (src/gemma_model.cpp:19-229 loads the same tensors and keys):
 * layer matrices all Q4_0 or all Q8_0, token_embd that type or Q6_K (llama.cpp's layout); NULL with
 * hpc_last_error on anything else.  gemma_engine_config returns the configuration read. */
gemma_engine *gemma_engine_create_from_gguf(const char *path, int n_ctx, int device);
int gemma_engine_config(const gemma_engine *e, gemma_hip_config *out);
/* row-split tensor parallelism: one process per GPU; rank r holds rows
 * [r*rows/n, (r+1)*rows/n) of every matrix and RCCL all-gathers complete each activation vector
 * (4 per layer + one argmax key per rank), so logits are bit-identical to one GPU.
 * gemma_tp_unique_id fills `out` (>= 128 B) on rank 0; every rank passes a copy to create_tp.
 * nccl_id == NULL: all n_ranks shards in one engine on one GPU ("virtual ranks", same shards and
 * key merge, shards written in place instead of gathered) for single-GPU parity tests. */
int gemma_tp_unique_id(void *out, int cap);
gemma_engine *gemma_engine_create_tp(const gemma_hip_config *cfg, int device, int n_ranks, int rank,
                                     const void *nccl_id);
/* n_ranks == 1 with an id: a 1-rank RCCL communicator; every all-gather and the key gather then run
 * through RCCL (captured in the decode hipGraph) exactly as on N GPUs.  tp_info: [ranks, rank,
 * communicator present, shard slots in this engine] */
int gemma_engine_tp_info(const gemma_engine *e, int *out4);
/* layout flags for create_tp2: GEMMA_TP_REP_ATTN keeps Wq|Wk|Wv and Wo whole on every rank (the
 * attention block replicated, 2 all-gathers per layer instead of 4; the FFN and the output head
 * stay row-split; the same bits either way).  tp_flags returns the engine's flags. */
#define GEMMA_TP_REP_ATTN 1
/* GEMMA_TP_P2P (nccl_id NULL, n_ranks > 1, one process per GPU): the all-gathers by peer-to-peer
 * pushes into each peer's uncached inbox arena (p2p.hip) instead of RCCL.  Each rank publishes its
 * arena with gemma_engine_p2p_handle (an IPC handle, <= 64 B), every rank passes all handles in
 * rank order to gemma_engine_p2p_open, then a host barrier, then steps.  p2p_err: a flag wait timed
 * out (sticky; reset clears). */
#define GEMMA_TP_P2P 2
int gemma_engine_p2p_handle(const gemma_engine *e, void *out, int cap);
int gemma_engine_p2p_open(gemma_engine *e, const void *handles, int n);
int gemma_engine_p2p_err(gemma_engine *e, int reset);
gemma_engine *gemma_engine_create_tp2(const gemma_hip_config *cfg, int device, int n_ranks, int rank,
                                      const void *nccl_id, int flags);
int gemma_engine_tp_flags(const gemma_engine *e);
void gemma_engine_free(gemma_engine *e);
/* start a sequence: KV cache cleared, prompt stored on the device */
int gemma_engine_begin(gemma_engine *e, const int32_t *prompt, int n_prompt);
/* run n steps of the ordered (bit-exact) per-token pass starting at the current position;
 * step i processes sequence[pos] and appends the greedy token once the prompt is consumed.
 * logits (n_vocab floats per step) are copied out when logits != NULL. use_graph: replay a
 * captured hipGraph per step (no host sync between steps when logits == NULL). */
int gemma_engine_step(gemma_engine *e, int n, float *logits, int use_graph);
int gemma_engine_tokens(gemma_engine *e, int32_t *out, int cap); /* sequence so far; returns len */
int gemma_engine_pos(gemma_engine *e);
/* batched prefill (the reference's T-token graph, src/gemma_model.cpp:665-747): processes the
 * whole prompt in one pass, writes the last row's logits (and all rows if logits_all), returns
 * the greedy token.  Bit-identical to the CPU path (ggml lane order). */
int gemma_engine_prefill(gemma_engine *e, float *logits_last, float *logits_all);
/* the same on int8/f16 MFMA: fp32 summation order differs from the CPU path (tolerance path) */
int gemma_engine_prefill_fast(gemma_engine *e, float *logits_last, float *logits_all);
/* weights back in ggml row-major layout (tests); tid as in DESIGN.md §Synthetic weights */
int64_t gemma_engine_tensor(gemma_engine *e, int tid, void *dst, int64_t cap);
/* time `iters` launches of one hot kernel with hipEvents on the engine stream; returns avg µs and
 * the algorithmic bytes (or int-ops) per launch.  which: 0 = ffn gate/up matvec, 1 = ffn down,
 * 2 = qkv, 3 = attn out, 4 = output/logits, 5 = whole decode step (graph) */
double gemma_engine_time(gemma_engine *e, int which, int iters, double *algo_bytes);
int gemma_engine_sync(gemma_engine *e);
/* launch plan per matrix class (0 qkv, 1 attn-out, 2 gate/up, 3 down, 4 logits): K split and
 * row-tile groups per workgroup.  tune: coordinate descent over whole decode steps (hipGraph
 * replays of `iters` tokens per candidate); bit-identical results for every plan; clobbers the
 * decode state (call gemma_engine_begin afterwards).  plan/set_plan: 2 ints per class. */
int gemma_engine_tune(gemma_engine *e, int iters);
int gemma_engine_plan(gemma_engine *e, int *out, int cap);
int gemma_engine_set_plan(gemma_engine *e, const int *in, int n);
int gemma_engine_set_fuse(gemma_engine *e, int fuse_front); /* fused layer front on/off (-1 = keep); returns the hand-off timeout word */
/* the decode attention and attn-out (+ residual) in ONE launch per layer (k_attn_o: the attention
   launch's idle workgroups run attn-out's row tiles after an in-launch hand-off; same bits): on 1 /
   off 0 / keep -1; returns the setting.  A hand-off timeout is reported by gemma_engine_step (-1) and
   turns it off. */
int gemma_engine_set_att_o(gemma_engine *e, int on);
/* The measured variants that stay selectable (tests, A/B), set through the API rather than the
   environment: "kq_fuse" (K-quant Q8_K INIT plan 0..6), "kq_dual" (gate+up one launch), "kq_pair"
   (q|k and v one launch), "kq_abl" (timing ablation, wrong results), "att_mx" (exact prefill attention
   on the f32 matrix cores; 0 = the row form), "att_dsplit" (decode attention workgroups per head:
   1/2/4/8), "ks_small" / "ks_down" (launch-plan K split defaults), "grid_big", and the
   gemma_engine_time diagnostics "time_hot" / "ablate".  Returns 0, -1 (unknown name or bad value). */
int gemma_engine_set_option(gemma_engine *e, const char *name, int value);
int gemma_engine_graph_kernels(gemma_engine *e);            /* kernel launches per decode token (captured graph) */
/* the decode step's layers as ONE persistent launch (opt-in: off by default, GHIP_PERSIST=1 or this
 * call; -1 = keep): returns 1 when it runs this engine's steps, 0 when not (hpc_last_error says why:
 * K-quant layers, row-split TP, shapes).  A hand-off timeout inside the launch (a workgroup not
 * co-resident) is reported: gemma_engine_step returns -1 (restart the sequence), the ggml executor's
 * decode redoes the token on the per-layer launches; either way the engine leaves the launch off. */
int gemma_engine_set_persist(gemma_engine *e, int on);
/* its sticky hand-off timeout words [flag, site, layer]; returns the flag (0 = none); reset clears */
int gemma_engine_persist_err(gemma_engine *e, int *out3, int reset);
/* tests: the launch's per-wait bound in 100 MHz ticks (0 = default 20 ms) */
int gemma_engine_set_persist_timeout(gemma_engine *e, unsigned ticks);
/* debugging: one eager step with per-layer taps [n_layer][qkv | attn_out | layer_out] */
int gemma_engine_debug_step(gemma_engine *e, float *host_taps, float *logits);
/* diagnostics: prefill (exact != 0: the exact path) with the residual stream after each layer
 * -> [n_layer][T][n_embd] */
int gemma_engine_prefill_taps(gemma_engine *e, float *host_taps, int exact);
/* diagnostics: one eager step with s_memrealtime phase stamps (100 MHz) of layer `layer`'s five
 * kernels (regions 0..4: qkv, attention, attn-out, gate/up, down) and the logits kernel (region 5);
 * out = 6 * 4096 * 16 u64, slot [region][workgroup][phase], unused slots 0 */
int gemma_engine_stamp_step(gemma_engine *e, int layer, unsigned long long *out);
/* diagnostics: one eager step through the persistent launch with its phase stamps
 * -> out [n_embd / 8][n_layer][16] u64 + 256 per-pop probes (GHIP_STAMPS build) */
int gemma_engine_token_stamps(gemma_engine *e, unsigned long long *out);
/* per-op test entry: one decode-attention block on host buffers (caches updated in place);
 * mode 0 = one workgroup per head, 1 = position-split form with the in-kernel hand-off */
int gemma_test_attn_decode(const float *qkv, uint16_t *kc, uint16_t *vc, int pos, int H, int Hkv, int hd, int ctx,
                           float rope_base, float *out, float *dbg_w, uint16_t *dbg_p, float *dbg_inv,
                           unsigned long long *dbg_t, int mode);

/* per-op test entry: the prefill path's Q8_0 row quantization + int8 MFMA GEMM on host buffers */
int gemma_test_gemm(int type, int64_t rows, int64_t K, int64_t T, const void *W, const float *X, float *Y,
                    int8_t *xq_out, float *da_out);
/* the same with the exact (ggml AVX2 lane order) GEMM of the exact prefill */
int gemma_test_gemm_exact(int type, int64_t rows, int64_t K, int64_t T, const void *W, const float *X, float *Y,
                          int8_t *xq_out, float *da_out);
/* K-quant matvec (Q4_K / Q6_K x Q8_K) timed alone: avg µs per launch over
 * `iters` launches rotating over cold weight copies; *algo_bytes = weights + Q8_K column + y */
double gemma_kq_time(int type, int64_t rows, int64_t K, int iters, double *algo_bytes);
/* measured HBM read roofline: streaming read of `bytes` on `device`, `iters` passes; GB/s — the
   faster of the two probes below */
double gemma_hbm_read_gbs(int device, size_t bytes, int iters);
/* one probe: variant 0 = 16-B nontemporal loads into registers, 1 = LDS-DMA (global_load_lds nt) */
double gemma_hbm_read_probe(int device, size_t bytes, int iters, int variant);
/* per-op test entry: the softmax's exp(f16) for all 65536 codes (compared with ggml's table) */
int gemma_test_exp_f16(uint16_t *out);
/* per-op test entry: one rms_norm kernel on host rows (ggml rms_norm):
 * kind 0 the ggml executor's RMS_NORM (out f32 rows), kind 1 k_norm_q8K (rms_norm * w, then
 * quantize_row_q8_K; out Q8_K rows) */
int gemma_test_rms_norm(int kind, const float *x, const float *w, int rows, int n, float eps, void *out);

#ifdef __cplusplus
}
#endif
#endif
