// engine_ext.h — internal interface between the device-resident Gemma engine (engine.cpp) and the
// ggml graph executor (ggml_api.cpp): an engine built over the host weights a ggml graph references,
// whose per-layer KV caches are the executor's device mirrors of the graph's cache tensors.
#pragma once

#include <stdint.h>

#include <vector>

#include "../../include/gemma_hpc.h"

namespace ghip {

struct host_weights {
    const void *embd = nullptr;  // token_embd, type cfg.out_type (or wtype)
    const float *out_norm = nullptr;
    struct layer {
        const float *attn_norm = nullptr, *ffn_norm = nullptr;
        const void *q = nullptr, *k = nullptr, *v = nullptr, *o = nullptr, *gate = nullptr, *up = nullptr, *down = nullptr;
        int tq = 0, tk = 0, tv = 0, to = 0, tg = 0, tu = 0, td = 0;  // K-quant layers: each matrix's type
    };
    std::vector<layer> layers;
};

}  // namespace ghip

// engine over host weights `hw` (layout of gemma_engine_create_from_gguf) with external per-layer
// caches: kc[il] [n_ctx][kvw] f16, vc[il] [kvw][n_ctx] f16 (the reference's cache tensors)
gemma_engine *gemma_engine_create_ext(const gemma_hip_config *cfg, int device, const ghip::host_weights &hw,
                                      const std::vector<uint16_t *> &kc, const std::vector<uint16_t *> &vc);
// one decode step for `token` at position `pos` (KV rows < pos already in the caches); the logits
// row to host `logits` (n_vocab floats)
int gemma_engine_ext_decode(gemma_engine *e, int token, int pos, float *logits);
// prompt rows 0..T-1 (caches written from position 0); every row's logits to host `logits_all`
int gemma_engine_ext_prefill(gemma_engine *e, const int32_t *tokens, int T, float *logits_all);
