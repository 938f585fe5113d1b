// gemma_graph_driver.cpp — TEST DRIVER (not product code): the reference's model driver restated
// against the ggml surface libgemma_hip.so exports (include/ggml.h), to show that code written like
// src/gemma_model.cpp builds and runs its graphs on the MI355X executor unchanged.
//
// Restated (clean-room, same API calls in the same order) from the reference:
//   init_input_tensor (src/gemma_model.cpp:341-359), init_kv_cache (:361-401),
//   load_input_tokens_to_tensor (:288-338), update_kv_cache (:428-436), graph_build_norm / ffn /
//   kqv / kv_store / kv (:438-529), greedy_sample (:532-546), reset_compute_context (:650-663),
//   build_compute_graph (:665-747), inference (:231-286); constants of src/macro.h:7-24.
// Differences: the KV width is n_head_kv * head_dim (the reference hard-codes one kv head), the
// context / batch sizes are arguments, a fixed number of decode steps runs (no stop at eos), and the
// output matrix is the tied token embedding (src/gemma_model.cpp:161-163).
//
// Weights come either from a GGUF file, loaded as src/gemma_model.cpp:19-229 / 403-415 / 583-601
// does (gguf_init_from_file into a weight context, kv index, ggml_get_tensor by name, hyper
// parameters and tokenizer tables from the metadata; head_dim = gemma.attention.key_length when
// present, else n_embd / n_head as the reference computes it), or from a file of raw tensors.
//
// usage: gemma_graph_driver <model.gguf> <prompt.bin> <out.bin> ctx n_decode
//        gemma_graph_driver <weights.bin> <prompt.bin> <out.bin> n_layer n_embd n_head n_head_kv
//        head_dim n_ff n_vocab ctx wtype n_decode
// out.bin: (1 + n_decode) rows of n_vocab f32 logits (prefill's last row, then each decode step),
//          followed by the (1 + n_decode) greedy token ids (int32).
#include <math.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <algorithm>
#include <chrono>
#include <map>
#include <string>
#include <vector>

#include "gemma_hpc.h"
#include "ggml.h"

namespace {

struct hparams {
    int n_layer, n_embd, n_head, n_head_kv, head_dim, n_ff, n_vocab, ctx, wtype;
    float eps = 1e-6f;
};
struct layer_w {
    ggml_tensor *attn_norm, *q, *k, *v, *o, *ffn_norm, *gate, *up, *down;
};
struct model {
    hparams hp;
    ggml_context *weight_ctx = nullptr, *input_ctx = nullptr, *kv_ctx = nullptr, *compute_ctx = nullptr;
    ggml_tensor *token_embd = nullptr, *output_norm = nullptr;
    std::vector<layer_w> layers;
    ggml_tensor *inp_tokens = nullptr, *inp_pos = nullptr, *inp_KQ_mask = nullptr;
    ggml_backend_buffer_t input_buf = nullptr, kv_buf = nullptr;
    std::vector<ggml_tensor *> k_layer, v_layer;
    int kv_n = 0, kv_head = 0;
    std::vector<char> compute_mem;
    bool no_alloc = false;  // --graph-listing: node metadata only
    // GGUF-loaded models: kv index, tensors by name, tokenizer tables (src/gemma_model.cpp:200-214)
    std::map<std::string, int> kv_index;
    std::map<std::string, ggml_tensor *> tensors;
    std::vector<std::string> tokens;
    int32_t bos = -1, eos = -1;
};

enum stage { PREFILL, DECODE };

bool read_tensor(FILE *f, ggml_tensor *t) { return fread(t->data, 1, ggml_nbytes(t), f) == ggml_nbytes(t); }

bool load_weights(model &m, const char *path) {
    const hparams &h = m.hp;
    const ggml_type wt = (ggml_type)h.wtype;
    const int64_t qw = (int64_t)h.n_head * h.head_dim, kvw = (int64_t)h.n_head_kv * h.head_dim;
    size_t bytes = ggml_row_size(wt, h.n_embd) * h.n_vocab + 4 * h.n_embd;
    bytes += (size_t)h.n_layer * (8 * h.n_embd + ggml_row_size(wt, h.n_embd) * (qw + 2 * kvw + 2 * h.n_ff) +
                                  ggml_row_size(wt, qw) * h.n_embd + ggml_row_size(wt, h.n_ff) * h.n_embd);
    ggml_init_params p = {bytes + (size_t)(h.n_layer * 9 + 2) * (ggml_tensor_overhead() + 64), nullptr, false};
    m.weight_ctx = ggml_init(p);
    FILE *f = fopen(path, "rb");
    if (!f) return false;
    bool ok = true;
    m.token_embd = ggml_new_tensor_2d(m.weight_ctx, wt, h.n_embd, h.n_vocab);
    m.output_norm = ggml_new_tensor_1d(m.weight_ctx, GGML_TYPE_F32, h.n_embd);
    ok = ok && read_tensor(f, m.token_embd) && read_tensor(f, m.output_norm);
    for (int il = 0; il < h.n_layer && ok; ++il) {
        layer_w L;
        L.attn_norm = ggml_new_tensor_1d(m.weight_ctx, GGML_TYPE_F32, h.n_embd);
        L.q = ggml_new_tensor_2d(m.weight_ctx, wt, h.n_embd, qw);
        L.k = ggml_new_tensor_2d(m.weight_ctx, wt, h.n_embd, kvw);
        L.v = ggml_new_tensor_2d(m.weight_ctx, wt, h.n_embd, kvw);
        L.o = ggml_new_tensor_2d(m.weight_ctx, wt, qw, h.n_embd);
        L.ffn_norm = ggml_new_tensor_1d(m.weight_ctx, GGML_TYPE_F32, h.n_embd);
        L.gate = ggml_new_tensor_2d(m.weight_ctx, wt, h.n_embd, h.n_ff);
        L.up = ggml_new_tensor_2d(m.weight_ctx, wt, h.n_embd, h.n_ff);
        L.down = ggml_new_tensor_2d(m.weight_ctx, wt, h.n_ff, h.n_embd);
        for (ggml_tensor *t : {L.attn_norm, L.q, L.k, L.v, L.o, L.ffn_norm, L.gate, L.up, L.down}) ok = ok && read_tensor(f, t);
        m.layers.push_back(L);
    }
    fclose(f);
    return ok;
}

// ---- GGUF loading (src/gemma_model.cpp:19-50 load_model_from_file and the helpers it calls) ----
uint32_t get_u32(gguf_context *g, model &m, const char *key) { return gguf_get_val_u32(g, m.kv_index.at(key)); }

bool load_model_from_file(model &m, const char *path) {
    gguf_init_params gp = {false, &m.weight_ctx};
    gguf_context *g = gguf_init_from_file(path, gp);
    if (!g) return false;
    for (int i = 0; i < gguf_get_n_kv(g); ++i) m.kv_index[gguf_get_key(g, i)] = i;  // :596-603
    for (int i = 0; i < gguf_get_n_tensors(g); ++i) {                               // :583-593
        const char *name = gguf_get_tensor_name(g, i);
        m.tensors[name] = ggml_get_tensor(m.weight_ctx, name);
    }
    auto get = [&](const std::string &n) -> ggml_tensor * {
        auto it = m.tensors.find(n);
        return it == m.tensors.end() ? nullptr : it->second;
    };
    hparams &h = m.hp;  // init_hyper_param (:403-415)
    h.n_layer = (int)get_u32(g, m, "gemma.block_count");
    h.n_embd = (int)get_u32(g, m, "gemma.embedding_length");
    h.n_head = (int)get_u32(g, m, "gemma.attention.head_count");
    h.n_head_kv = (int)get_u32(g, m, "gemma.attention.head_count_kv");
    h.eps = gguf_get_val_f32(g, m.kv_index.at("gemma.attention.layer_norm_rms_epsilon"));
    h.head_dim = m.kv_index.count("gemma.attention.key_length") ? (int)get_u32(g, m, "gemma.attention.key_length")
                                                                 : h.n_embd / h.n_head;
    // composite_model (:145-182): the tied output is token_embd
    m.token_embd = get("token_embd.weight");
    m.output_norm = get("output_norm.weight");
    if (!m.token_embd || !m.output_norm) return false;
    h.n_vocab = (int)m.token_embd->ne[1];
    h.wtype = (int)m.token_embd->type;
    char name[64];
    for (int il = 0; il < h.n_layer; ++il) {
        layer_w L;
        ggml_tensor **slots[9] = {&L.o, &L.k, &L.v, &L.q, &L.gate, &L.up, &L.down, &L.attn_norm, &L.ffn_norm};
        const char *names[9] = {"attn_output", "attn_k", "attn_v", "attn_q", "ffn_gate", "ffn_up", "ffn_down",
                                "attn_norm", "ffn_norm"};
        for (int k = 0; k < 9; ++k) {
            snprintf(name, sizeof(name), "blk.%d.%s.weight", il, names[k]);
            if (!(*slots[k] = get(name))) {
                fprintf(stderr, "missing tensor %s\n", name);
                return false;
            }
        }
        m.layers.push_back(L);
    }
    h.n_ff = (int)m.layers[0].gate->ne[1];
    // load_tokenizer (:200-214)
    m.bos = (int32_t)get_u32(g, m, "tokenizer.ggml.bos_token_id");
    m.eos = (int32_t)get_u32(g, m, "tokenizer.ggml.eos_token_id");
    const int it = m.kv_index.at("tokenizer.ggml.tokens");
    for (int i = 0; i < gguf_get_arr_n(g, it); ++i) m.tokens.push_back(gguf_get_arr_str(g, it, i));
    gguf_free(g);
    return true;
}

// gemma_tokenizer::print_tokens (:757-767): concatenate, drop "<bos>", U+2581 -> ' '
std::string detokenize(const model &m, const std::vector<int32_t> &ids) {
    std::string s;
    for (int32_t id : ids) s += m.tokens.at(id);
    const size_t b = s.find("<bos>");
    if (b != std::string::npos) s.replace(b, 5, "");
    const std::string u = "\xe2\x96\x81";
    for (size_t p = 0; (p = s.find(u, p)) != std::string::npos;) s.replace(p, u.size(), " ");
    return s;
}

void init_input_tensor(model &m) {  // src/gemma_model.cpp:341-359
    ggml_init_params p = {ggml_tensor_overhead() * 4, nullptr, true};
    m.input_ctx = ggml_init(p);
    m.inp_tokens = ggml_new_tensor_1d(m.input_ctx, GGML_TYPE_I32, m.hp.ctx);
    m.inp_pos = ggml_new_tensor_1d(m.input_ctx, GGML_TYPE_I32, m.hp.ctx);
    m.inp_KQ_mask = ggml_new_tensor_2d(m.input_ctx, GGML_TYPE_F32, m.hp.ctx, m.hp.ctx);
    m.input_buf = ggml_backend_alloc_ctx_tensors_from_buft(m.input_ctx, ggml_backend_cpu_buffer_type());
    ggml_backend_buffer_clear(m.input_buf, 0);
}

void init_kv_cache(model &m) {  // src/gemma_model.cpp:361-401
    const int64_t kvw = (int64_t)m.hp.n_head_kv * m.hp.head_dim;
    ggml_init_params p = {2u * m.hp.n_layer * ggml_tensor_overhead(), nullptr, true};
    m.kv_ctx = ggml_init(p);
    for (int i = 0; i < m.hp.n_layer; ++i) {
        ggml_tensor *k = ggml_new_tensor_1d(m.kv_ctx, GGML_TYPE_F16, kvw * m.hp.ctx);
        ggml_tensor *v = ggml_new_tensor_1d(m.kv_ctx, GGML_TYPE_F16, kvw * m.hp.ctx);
        ggml_format_name(k, "cache_k_l%d", i);
        ggml_format_name(v, "cache_v_l%d", i);
        m.k_layer.push_back(k);
        m.v_layer.push_back(v);
    }
    m.kv_buf = ggml_backend_alloc_ctx_tensors_from_buft(m.kv_ctx, ggml_backend_cpu_buffer_type());
    ggml_backend_buffer_clear(m.kv_buf, 0);
}

void update_kv_cache(model &m, const std::vector<int32_t> &input, stage st) {  // :428-436
    m.kv_n = std::min(m.hp.ctx, ((int)input.size() / 32 + 1) * 32);
    m.kv_head = st == PREFILL ? 0 : (int)input.size() - 1;
}

void load_input_tokens_to_tensor(model &m, const std::vector<int32_t> &input, stage st) {  // :288-338
    const size_t n = st == PREFILL ? input.size() : 1;
    ggml_backend_tensor_set(m.inp_tokens, input.data() + (st == PREFILL ? 0 : input.size() - 1), 0,
                            n * ggml_element_size(m.inp_tokens));
    std::vector<int32_t> pos(n);
    for (size_t i = 0; i < n; ++i) pos[i] = st == PREFILL ? (int32_t)i : (int32_t)input.size() - 1;
    ggml_backend_tensor_set(m.inp_pos, pos.data(), 0, n * ggml_element_size(m.inp_pos));
    float *mask = (float *)m.inp_KQ_mask->data;
    size_t begin = st == PREFILL ? 0 : input.size() - 1;
    for (size_t i = 0; i < n; ++i, ++begin)
        for (int j = 0; j < m.kv_n; ++j) mask[i * m.kv_n + j] = (size_t)j > begin ? -INFINITY : 0.0f;
}

ggml_tensor *build_norm(model &m, ggml_context *ctx, ggml_tensor *x, ggml_tensor *w) {  // :438-442
    x = ggml_rms_norm(ctx, x, m.hp.eps);
    return ggml_mul(ctx, x, w);
}

ggml_tensor *build_ffn(ggml_context *ctx, ggml_tensor *cur, ggml_tensor *up, ggml_tensor *gate, ggml_tensor *down) {
    ggml_tensor *tmp = ggml_mul_mat(ctx, up, cur);  // :444-452
    cur = ggml_mul_mat(ctx, gate, cur);
    cur = ggml_gelu(ctx, cur);
    cur = ggml_mul(ctx, cur, tmp);
    return ggml_mul_mat(ctx, down, cur);
}

ggml_tensor *build_kqv(model &m, ggml_context *ctx, ggml_cgraph *g, ggml_tensor *wo, ggml_tensor *q_cur,
                       ggml_tensor *kq_mask, int n_tokens, float kq_scale, int il) {  // :454-497
    const int64_t hd = m.hp.head_dim, H = m.hp.n_head, Hkv = m.hp.n_head_kv, ctx_n = m.hp.ctx;
    ggml_tensor *q = ggml_permute(ctx, q_cur, 0, 2, 1, 3);
    ggml_tensor *k = ggml_view_3d(ctx, m.k_layer[il], hd, m.kv_n, Hkv, ggml_row_size(m.k_layer[il]->type, hd * Hkv),
                                  ggml_row_size(m.k_layer[il]->type, hd), 0);
    ggml_tensor *kq = ggml_mul_mat(ctx, k, q);
    kq = ggml_soft_max_ext(ctx, kq, kq_mask, nullptr, kq_scale, 0.0f);
    ggml_tensor *v = ggml_view_3d(ctx, m.v_layer[il], m.kv_n, hd, Hkv, ggml_element_size(m.v_layer[il]) * ctx_n,
                                  ggml_element_size(m.v_layer[il]) * ctx_n * hd, 0);
    ggml_tensor *kqv = ggml_mul_mat(ctx, v, kq);
    ggml_tensor *merged = ggml_permute(ctx, kqv, 0, 2, 1, 3);
    ggml_tensor *cur = ggml_cont_2d(ctx, merged, hd * H, n_tokens);
    ggml_build_forward_expand(g, cur);
    return ggml_mul_mat(ctx, wo, cur);
}

void build_kv_store(model &m, ggml_context *ctx, ggml_cgraph *g, ggml_tensor *k_cur, ggml_tensor *v_cur, int n_tokens,
                    int il) {  // :499-518
    const int64_t kvw = (int64_t)m.hp.n_head_kv * m.hp.head_dim, ctx_n = m.hp.ctx;
    ggml_tensor *v_cur_t = ggml_transpose(ctx, ggml_reshape_2d(ctx, v_cur, kvw, n_tokens));
    ggml_tensor *k_view = ggml_view_1d(ctx, m.k_layer[il], n_tokens * kvw, ggml_row_size(m.k_layer[il]->type, kvw) * m.kv_head);
    ggml_tensor *v_view = ggml_view_2d(ctx, m.v_layer[il], n_tokens, kvw, ctx_n * ggml_element_size(m.v_layer[il]),
                                       m.kv_head * ggml_element_size(m.v_layer[il]));
    ggml_build_forward_expand(g, ggml_cpy(ctx, k_cur, k_view));
    ggml_build_forward_expand(g, ggml_cpy(ctx, v_cur_t, v_view));
}

void reset_compute_context(model &m) {  // :650-663
    if (m.compute_ctx) ggml_free(m.compute_ctx);
    ggml_init_params p = {m.compute_mem.size(), m.compute_mem.data(), m.no_alloc};
    m.compute_ctx = ggml_init(p);
}

ggml_cgraph *build_compute_graph(model &m, const std::vector<int32_t> &input, stage st) {  // :665-747
    reset_compute_context(m);
    ggml_context *ctx = m.compute_ctx;
    ggml_cgraph *g = ggml_new_graph(ctx);
    const hparams &h = m.hp;
    const int64_t T = st == PREFILL ? (int64_t)input.size() : 1;
    ggml_tensor *tok = ggml_view_1d(ctx, m.inp_tokens, T, 0);
    ggml_set_name(tok, "inp_tokens (view)");
    ggml_tensor *inpL = ggml_get_rows(ctx, m.token_embd, tok);
    inpL = ggml_scale(ctx, inpL, sqrtf((float)h.n_embd));
    ggml_tensor *pos = ggml_view_1d(ctx, m.inp_pos, T, 0);
    ggml_set_name(pos, "inp_pos (view)");
    ggml_tensor *mask = ggml_view_2d(ctx, m.inp_KQ_mask, m.kv_n, T, m.kv_n * ggml_type_size(m.inp_KQ_mask->type), 0);
    ggml_set_name(mask, "inp_KQ_mask (view)");
    for (int il = 0; il < h.n_layer; ++il) {
        const layer_w &L = m.layers[il];
        ggml_tensor *cur = build_norm(m, ctx, inpL, L.attn_norm);
        ggml_tensor *q = ggml_mul_mat(ctx, L.q, cur);
        ggml_tensor *k = ggml_mul_mat(ctx, L.k, cur);
        ggml_tensor *v = ggml_mul_mat(ctx, L.v, cur);
        q = ggml_rope_custom(ctx, ggml_reshape_3d(ctx, q, h.head_dim, h.n_head, T), pos, h.head_dim, 2, 0, 8192, 10000,
                             1, 0, 1, 32, 1);
        q = ggml_scale(ctx, q, 1.0f / sqrtf((float)h.head_dim));
        k = ggml_rope_custom(ctx, ggml_reshape_3d(ctx, k, h.head_dim, h.n_head_kv, T), pos, h.head_dim, 2, 0, 8192,
                             10000, 1, 0, 1, 32, 1);
        ggml_build_forward_expand(g, q);  // graph_build_kv (:520-529)
        ggml_build_forward_expand(g, k);
        ggml_build_forward_expand(g, v);
        build_kv_store(m, ctx, g, k, v, (int)T, il);
        cur = build_kqv(m, ctx, g, L.o, q, mask, (int)T, 1.0f, il);
        ggml_tensor *sa = ggml_add(ctx, cur, inpL);
        cur = build_norm(m, ctx, sa, L.ffn_norm);
        cur = build_ffn(ctx, cur, L.up, L.gate, L.down);
        inpL = ggml_add(ctx, cur, sa);
    }
    ggml_tensor *cur = build_norm(m, ctx, inpL, m.output_norm);
    cur = ggml_mul_mat(ctx, m.token_embd, cur);  // tied output
    ggml_build_forward_expand(g, cur);
    ggml_set_name(g->nodes[g->n_nodes - 1], "result_output");
    return g;
}

int32_t greedy_sample(const ggml_tensor *out) {  // :532-546
    const float *logits = (const float *)out->data + out->ne[0] * (out->ne[1] - 1);
    float max_val = -INFINITY;
    int max_idx = -1;
    for (int i = 0; i < out->ne[0]; ++i)
        if (logits[i] > max_val) {
            max_val = logits[i];
            max_idx = i;
        }
    return max_idx;
}

}  // namespace

// one model's whole run (load, generate, free every context); wpath / opath stand in for argv[1] /
// argv[3], the other arguments as in main
int run_one(int argc, char **argv, const char *wpath, const char *opath) {
    const size_t alen = strlen(wpath);
    const bool gguf = alen > 5 && strcmp(wpath + alen - 5, ".gguf") == 0;
    model m;
    int n_decode;
    double upload_ms = 0.0;
    if (gguf) {
        if (!load_model_from_file(m, wpath)) {
            fprintf(stderr, "gguf: load failed\n");
            return 1;
        }
        m.hp.ctx = atoi(argv[4]);
        n_decode = atoi(argv[5]);
        // the device init of src/app.cpp:34-35 plus INTEGRATION.md §1's load-time weight upload:
        // every quantized weight goes to the device once, here, not inside the first timed graph
        if (!getenv("DRIVER_NO_REGISTER") || !atoi(getenv("DRIVER_NO_REGISTER"))) {
            const auto u0 = std::chrono::steady_clock::now();
            if (hpc_init(0)) return 1;
            std::vector<ggml_tensor *> ws{m.token_embd};
            for (const layer_w &L : m.layers)
                for (ggml_tensor *t : {L.q, L.k, L.v, L.o, L.gate, L.up, L.down}) ws.push_back(t);
            for (ggml_tensor *t : ws)
                if ((t->type == GGML_TYPE_Q4_0 || t->type == GGML_TYPE_Q8_0 || t->type == GGML_TYPE_Q4_K ||
                     t->type == GGML_TYPE_Q6_K) &&
                    hpc_register_weight(t->data, t->type, t->ne[0], t->ne[1], t->nb[1])) {
                    fprintf(stderr, "hpc_register_weight failed\n");
                    return 1;
                }
            upload_ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - u0).count();
        }
    } else {
        m.hp = {atoi(argv[4]), atoi(argv[5]), atoi(argv[6]), atoi(argv[7]), atoi(argv[8]), atoi(argv[9]), atoi(argv[10]),
                atoi(argv[11]), atoi(argv[12])};
        n_decode = atoi(argv[13]);
        if (!load_weights(m, wpath)) {
            fprintf(stderr, "weights: read failed\n");
            return 1;
        }
    }
    std::vector<int32_t> input;
    {
        FILE *f = fopen(argv[2], "rb");
        int32_t t;
        while (f && fread(&t, 4, 1, f) == 1) input.push_back(t);
        if (f) fclose(f);
    }
    init_input_tensor(m);
    init_kv_cache(m);
    // compute context: node metadata + the host copies of the intermediate data
    const size_t T = input.size(), L = m.hp.n_layer, E = m.hp.n_embd, F = m.hp.n_ff;
    const size_t qw = (size_t)m.hp.n_head * m.hp.head_dim, kvw = (size_t)m.hp.n_head_kv * m.hp.head_dim;
    const size_t per_tok = m.hp.n_vocab + 2 * E + L * (6 * F + 16 * E + 8 * qw + 6 * kvw);
    const size_t mid = (T * per_tok + L * T * (size_t)m.hp.ctx * m.hp.n_head * 4) * 4 + (64u << 20);
    m.compute_mem.resize(ggml_tensor_overhead() * 4096 + ggml_graph_overhead() + mid);
    FILE *out = fopen(opath, "wb");
    std::vector<int32_t> toks;
    // timing as begin_one_round_inference reports it (src/gemma_model.cpp:552-572): prefill, then decode
    auto now = [] { return std::chrono::steady_clock::now(); };
    const bool bench = getenv("DRIVER_BENCH") && atoi(getenv("DRIVER_BENCH"));
    // DRIVER_ROUNDS > 1: begin_one_round_inference again on the same prompt with the loaded model
    // (a new sequence from position 0); the timing line reports the last round, whose prefill is
    // compute only (the first round also pays one-time device setup: first_prefill_ms)
    const int rounds = getenv("DRIVER_ROUNDS") ? std::max(1, atoi(getenv("DRIVER_ROUNDS"))) : 1;
    const std::vector<int32_t> prompt = input;
    double first_pf_ms = 0.0;
    auto t_start = now(), t_prefill = t_start;
    for (int round = 0; round < rounds; ++round) {
    if (round > 0) input = prompt;
    t_start = now();
    t_prefill = t_start;
    for (int step = 0; step <= n_decode; ++step) {  // inference (:231-286)
        if (step == 1) t_prefill = now();
        const stage st = step == 0 ? PREFILL : DECODE;
        const auto p0 = now();
        update_kv_cache(m, input, st);
        load_input_tokens_to_tensor(m, input, st);
        ggml_cgraph *g = build_compute_graph(m, input, st);
        const auto p1 = now();
        // src/gemma_model.cpp:237 calls ggml_graph_compute_with_ctx; hpc_graph_compute is the same executor
        if (ggml_graph_compute_with_ctx(m.compute_ctx, g, 1) != GGML_STATUS_SUCCESS) {
            fprintf(stderr, "graph compute failed\n");
            return 1;
        }
        const auto p2 = now();
        const int32_t t = greedy_sample(g->nodes[g->n_nodes - 1]);
        const auto p3 = now();
        if (getenv("DRIVER_PROF"))
            fprintf(stderr, "step %d: build %.1f us compute %.1f us sample %.1f us\n", step,
                    std::chrono::duration<double, std::micro>(p1 - p0).count(), std::chrono::duration<double, std::micro>(p2 - p1).count(),
                    std::chrono::duration<double, std::micro>(p3 - p2).count());
        if (!bench && round == 0) {  // the last row for the tests (bench mode: the timed loop is the reference's)
            const ggml_tensor *o = g->nodes[g->n_nodes - 1];
            fwrite((const float *)o->data + o->ne[0] * (o->ne[1] - 1), 4, (size_t)o->ne[0], out);
        }
        if (round == 0) toks.push_back(t);
        input.push_back(t);
    }
    if (round == 0) first_pf_ms = std::chrono::duration<double, std::milli>((n_decode > 0 ? t_prefill : now()) - t_start).count();
    }
    const auto t_end = now();
    const double pf_ms = std::chrono::duration<double, std::milli>(t_prefill - t_start).count();
    const double dec_ms = std::chrono::duration<double, std::milli>(t_end - t_prefill).count();
    fprintf(stderr, "timing prefill_ms %.3f prompt %zu decode_ms %.3f steps %d decode_tok_s %.2f upload_ms %.3f "
            "first_prefill_ms %.3f rounds %d\n", pf_ms, T, dec_ms, n_decode, n_decode > 0 ? n_decode / (dec_ms * 1e-3) : 0.0,
            upload_ms, first_pf_ms, rounds);
    fwrite(toks.data(), 4, toks.size(), out);
    fclose(out);
    if (gguf) {  // the sequence as text, through the GGUF tokenizer table
        const std::string txt = detokenize(m, input);
        FILE *tf = fopen((std::string(opath) + ".txt").c_str(), "wb");
        if (tf) {
            fwrite(txt.data(), 1, txt.size(), tf);
            fclose(tf);
        }
    }
    ggml_free(m.compute_ctx);
    ggml_backend_buffer_free(m.input_buf);
    ggml_backend_buffer_free(m.kv_buf);
    ggml_free(m.input_ctx);
    ggml_free(m.kv_ctx);
    // the weight buffers go away: drop their device copies first, or a next
    // model loaded at the same addresses would be served these
    if (m.token_embd) hpc_unregister_weight(m.token_embd->data);
    for (const layer_w &L : m.layers)
        for (ggml_tensor *t : {L.q, L.k, L.v, L.o, L.gate, L.up, L.down}) hpc_unregister_weight(t->data);
    ggml_free(m.weight_ctx);
    return 0;
}

// --graph-listing: build_compute_graph on weight / input / cache tensors without data (no device,
// no weights) and print the graph as src/gemma_model.cpp:240-248 dumps it, "node[i]: name", plus
// each node's op — the form of the reference's tensor_dump/tensor_in_target_cgraph listing
int graph_listing(int argc, char **argv) {
    if (argc < 12) return 2;
    model m;
    m.hp = {atoi(argv[2]), atoi(argv[3]), atoi(argv[4]), atoi(argv[5]), atoi(argv[6]), atoi(argv[7]), atoi(argv[8]),
            atoi(argv[9]), atoi(argv[10])};
    const int T = atoi(argv[11]);
    const stage st = argc > 12 && atoi(argv[12]) ? DECODE : PREFILL;
    const hparams &h = m.hp;
    const ggml_type wt = (ggml_type)h.wtype;
    const int64_t qw = (int64_t)h.n_head * h.head_dim, kvw = (int64_t)h.n_head_kv * h.head_dim;
    ggml_init_params p = {(size_t)(h.n_layer * 9 + 2) * ggml_tensor_overhead(), nullptr, true};
    m.weight_ctx = ggml_init(p);
    m.token_embd = ggml_new_tensor_2d(m.weight_ctx, wt, h.n_embd, h.n_vocab);
    ggml_set_name(m.token_embd, "token_embd.weight");
    m.output_norm = ggml_new_tensor_1d(m.weight_ctx, GGML_TYPE_F32, h.n_embd);
    ggml_set_name(m.output_norm, "output_norm.weight");
    for (int il = 0; il < h.n_layer; ++il) {
        layer_w L;
        L.attn_norm = ggml_new_tensor_1d(m.weight_ctx, GGML_TYPE_F32, h.n_embd);
        L.q = ggml_new_tensor_2d(m.weight_ctx, wt, h.n_embd, qw);
        L.k = ggml_new_tensor_2d(m.weight_ctx, wt, h.n_embd, kvw);
        L.v = ggml_new_tensor_2d(m.weight_ctx, wt, h.n_embd, kvw);
        L.o = ggml_new_tensor_2d(m.weight_ctx, wt, qw, h.n_embd);
        L.ffn_norm = ggml_new_tensor_1d(m.weight_ctx, GGML_TYPE_F32, h.n_embd);
        L.gate = ggml_new_tensor_2d(m.weight_ctx, wt, h.n_embd, h.n_ff);
        L.up = ggml_new_tensor_2d(m.weight_ctx, wt, h.n_embd, h.n_ff);
        L.down = ggml_new_tensor_2d(m.weight_ctx, wt, h.n_ff, h.n_embd);
        const char *names[9] = {"attn_norm", "attn_q", "attn_k", "attn_v", "attn_output", "ffn_norm", "ffn_gate", "ffn_up", "ffn_down"};
        ggml_tensor *ts[9] = {L.attn_norm, L.q, L.k, L.v, L.o, L.ffn_norm, L.gate, L.up, L.down};
        for (int k = 0; k < 9; ++k) ggml_format_name(ts[k], "blk.%d.%s.weight", il, names[k]);
        m.layers.push_back(L);
    }
    init_input_tensor(m);
    init_kv_cache(m);
    std::vector<int32_t> input(T, 2);
    update_kv_cache(m, input, st);
    m.compute_mem.resize(ggml_tensor_overhead() * 4096 + ggml_graph_overhead() + (1u << 20));
    m.no_alloc = true;  // metadata only: the listing needs no node data
    ggml_cgraph *g = build_compute_graph(m, input, st);
    for (int i = 0; i < g->n_nodes; ++i) printf("node[%d]: %s\t%s\n", i, g->nodes[i]->name, ggml_op_name((enum ggml_op)g->nodes[i]->op));
    ggml_free(m.compute_ctx);
    ggml_backend_buffer_free(m.input_buf);
    ggml_backend_buffer_free(m.kv_buf);
    ggml_free(m.input_ctx);
    ggml_free(m.kv_ctx);
    ggml_free(m.weight_ctx);
    return 0;
}

int main(int argc, char **argv) {
    if (argc > 1 && strcmp(argv[1], "--graph-listing") == 0) return graph_listing(argc, argv);
    const size_t alen = argc > 1 ? strlen(argv[1]) : 0;
    const bool gguf = alen > 5 && strcmp(argv[1] + alen - 5, ".gguf") == 0;
    if ((gguf && argc < 6) || (!gguf && argc < 14)) {
        fprintf(stderr, "usage: %s model.gguf prompt out ctx n_decode\n"
                        "       %s weights prompt out n_layer n_embd n_head n_head_kv head_dim n_ff n_vocab ctx wtype n_decode\n"
                        "  DRIVER_SECOND=<weights2>: then a second model of the same shapes in the same process (out.2)\n",
                argv[0], argv[0]);
        return 2;
    }
    int r = run_one(argc, argv, argv[1], argv[3]);
    if (r == 0 && getenv("DRIVER_SECOND")) r = run_one(argc, argv, getenv("DRIVER_SECOND"), (std::string(argv[3]) + ".2").c_str());
    return r;
}
