// gemma_cpu.cpp — ORACLE (test infrastructure only; see oracle.h header).
//
// CPU restatement of the reference's Gemma forward pass as wired by
// src/gemma_model.cpp:665-747 (build_compute_graph) and executed by ggml on one thread with
// MUL_MAT fanned out to the worker pool (src/gemma_model.cpp:237, src/hpc.cpp:216-273).
// Deliberate, documented deviations (all "lifted limits"):
//   * n_ctx is a parameter (reference: 512, src/macro.h:9); no 128 MiB arena cap;
//   * head_dim is a parameter (reference derives n_embd/n_head, src/gemma_model.cpp:409-410);
//   * K/V width = n_head_kv*head_dim with GQA broadcast (reference: MQA only, :362-363).
// For Gemma-2B (n_head_kv = 1, head_dim = 256 = 2048/8) these coincide with the reference.
//
// Also holds the synthetic-weight generator (DESIGN.md §Synthetic weights) used by both the
// oracle and, re-implemented as a HIP kernel, by the product; tests check they agree bitwise.
#include <math.h>
#include <string.h>

#include <algorithm>
#include <chrono>
#include <functional>
#include <thread>
#include <vector>

#include "oracle.h"

namespace {

inline uint64_t splitmix64(uint64_t x) {
    x += 0x9E3779B97F4A7C15ull;
    uint64_t z = x;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}

// Irwin–Hall(4) integer sum, centred: exact integer in [-131070, 131070].
inline int32_t synth_int(uint64_t key, uint64_t idx) {
    const uint64_t h = splitmix64(key + idx);
    return (int32_t)((h & 0xFFFF) + ((h >> 16) & 0xFFFF) + ((h >> 32) & 0xFFFF) + (h >> 48)) - 131070;
}

inline uint64_t tensor_key(uint64_t seed, int tid) { return splitmix64(seed ^ ((uint64_t)tid << 40)); }
inline float synth_scale(double stdv) { return (float)(stdv * 1.7320508075688772 / 65536.0); }

enum { TID_EMBD = 0, TID_OUT_NORM = 1 };
inline int tid_layer(int il, int k) { return 16 + il * 16 + k; }
enum { L_ATTN_NORM = 0, L_Q = 1, L_K = 2, L_V = 3, L_O = 4, L_FFN_NORM = 5, L_GATE = 6, L_UP = 7, L_DOWN = 8 };

struct qmat {
    int type = ORC_Q4_0;
    int64_t rows = 0, cols = 0;
    size_t row_bytes = 0;
    std::vector<uint8_t> data;
};

void parallel_rows(int64_t rows, const std::function<void(int64_t, int64_t)> &fn) {
    int nt = (int)std::max(1u, std::thread::hardware_concurrency());
    nt = (int)std::min<int64_t>(nt, std::max<int64_t>(1, rows / 64));
    std::vector<std::thread> th;
    const int64_t per = (rows + nt - 1) / nt;
    for (int t = 0; t < nt; ++t) {
        const int64_t s = t * per, e = std::min(rows, s + per);
        if (s >= e) break;
        th.emplace_back([=, &fn] { fn(s, e); });
    }
    for (auto &t : th) t.join();
}

qmat make_qmat(uint64_t seed, int tid, int64_t rows, int64_t cols, int wtype, double stdv) {
    qmat m;
    m.type = wtype;
    m.rows = rows;
    m.cols = cols;
    m.row_bytes = orc_row_size(wtype, cols);
    m.data.resize(m.row_bytes * rows);
    const uint64_t key = tensor_key(seed, tid);
    const float sc = synth_scale(stdv);
    parallel_rows(rows, [&](int64_t r0, int64_t r1) {
        std::vector<float> buf(cols);
        for (int64_t r = r0; r < r1; ++r) {
            for (int64_t j = 0; j < cols; ++j) buf[j] = (float)synth_int(key, (uint64_t)(r * cols + j)) * sc;
            if (wtype == ORC_Q4_0) orc_quantize_row_q4_0_ref(buf.data(), m.data.data() + r * m.row_bytes, (int)cols);
            else orc_quantize_row_q8_0_ref(buf.data(), m.data.data() + r * m.row_bytes, (int)cols);
        }
    });
    return m;
}

// K-quant matrix: random valid super-blocks (orc_synth_kquant) with d (and dmin) rescaled so the
// dequantized values have roughly the requested standard deviation (Q4_K values ~0.8 and Q6_K
// ~0.68 rms before rescaling).  Weights are data here: the K-quant quantizer is not on the path.
qmat make_kmat(uint64_t seed, int tid, int64_t rows, int64_t cols, int type, double stdv) {
    qmat m;
    m.type = type;
    m.rows = rows;
    m.cols = cols;
    m.row_bytes = orc_row_size(type, cols);
    m.data.resize(m.row_bytes * rows);
    orc_synth_kquant(type, tensor_key(seed, tid), rows, cols, m.data.data());
    const float f = (float)(stdv / (type == ORC_Q4_K ? 0.8 : 0.68));
    const int64_t nb = rows * (cols / 256);
    for (int64_t b = 0; b < nb; ++b) {
        uint8_t *blk = m.data.data() + b * (type == ORC_Q4_K ? 144 : 210);
        uint16_t *d = (uint16_t *)(blk + (type == ORC_Q4_K ? 0 : 208));
        *d = orc_fp32_to_fp16(orc_fp16_to_fp32(*d) * f);
        if (type == ORC_Q4_K) d[1] = orc_fp32_to_fp16(orc_fp16_to_fp32(d[1]) * f);
    }
    return m;
}

void dequantize_row(int type, const uint8_t *row, float *y, int n) {
    switch (type) {
        case ORC_Q4_0: orc_dequantize_row_q4_0(row, y, n); break;
        case ORC_Q8_0: orc_dequantize_row_q8_0(row, y, n); break;
        case ORC_Q4_K: orc_dequantize_row_q4_K(row, y, n); break;
        case ORC_Q6_K: orc_dequantize_row_q6_K(row, y, n); break;
    }
}

std::vector<float> make_norm(uint64_t seed, int tid, int64_t n) {
    std::vector<float> v(n);
    const uint64_t key = tensor_key(seed, tid);
    const float sc = synth_scale(0.05);
    for (int64_t j = 0; j < n; ++j) v[j] = 1.0f + (float)synth_int(key, (uint64_t)j) * sc;
    return v;
}

struct layer_w {
    std::vector<float> attn_norm, ffn_norm;
    qmat q, k, v, o, gate, up, down;
};

}  // namespace

struct orc_model {
    orc_config cfg;
    qmat embd;  // also the tied output matrix (src/gemma_model.cpp:161-163)
    std::vector<float> out_norm;
    std::vector<layer_w> layers;
    std::vector<std::vector<uint16_t>> kc, vc;  // K: [ctx][kvw]   V: [kvw][ctx]  (f16)
    std::vector<std::vector<float>> hidden;    // debug capture of the last call
    std::vector<std::vector<float>> tap_qkv, tap_attn;  // last row: [q|k|v] pre-rope, merged attn
};

extern "C" orc_model *orc_model_create(const orc_config *cfg) {
    orc_init_tables(cfg->gelu_clamp);
    orc_model *m = new orc_model();
    m->cfg = *cfg;
    const orc_config &c = *cfg;
    const int qw = c.n_head * c.head_dim, kvw = c.n_head_kv * c.head_dim;
    if ((c.kmix == 1 && (c.n_embd % 256 || c.n_ff % 256 || qw % 256)) || (c.kmix == 2 && c.n_embd % 256)) {
        delete m;
        return nullptr;
    }
    const double emb_std = (c.out_gain > 0.0f ? (double)c.out_gain : 1.0) / sqrt((double)c.n_embd);
    m->embd = c.kmix ? make_kmat(c.seed, TID_EMBD, c.n_vocab, c.n_embd, ORC_Q6_K, emb_std)
                     : make_qmat(c.seed, TID_EMBD, c.n_vocab, c.n_embd, c.wtype, emb_std);
    m->out_norm = make_norm(c.seed, TID_OUT_NORM, c.n_embd);
    m->layers.resize(c.n_layer);
    for (int il = 0; il < c.n_layer; ++il) {
        layer_w &L = m->layers[il];
        L.attn_norm = make_norm(c.seed, tid_layer(il, L_ATTN_NORM), c.n_embd);
        L.ffn_norm = make_norm(c.seed, tid_layer(il, L_FFN_NORM), c.n_embd);
        // linear weights ~ N(0, 1/fan_in); residual writers (o, down) x4 gain so the tied output
        // is not dominated by the current token (DESIGN.md §Synthetic weights)
        const double se = 1.0 / sqrt((double)c.n_embd), sq = 1.0 / sqrt((double)qw), sf = 1.0 / sqrt((double)c.n_ff);
        auto mat = [&](int k, int64_t rows, int64_t cols, int ktype, double stdv) {
            return c.kmix == 1 ? make_kmat(c.seed, tid_layer(il, k), rows, cols, ktype, stdv)
                          : make_qmat(c.seed, tid_layer(il, k), rows, cols, c.wtype, stdv);
        };
        L.q = mat(L_Q, qw, c.n_embd, ORC_Q4_K, se);
        L.k = mat(L_K, kvw, c.n_embd, ORC_Q4_K, se);
        L.v = mat(L_V, kvw, c.n_embd, ORC_Q6_K, se);
        L.o = mat(L_O, c.n_embd, qw, ORC_Q4_K, 4.0 * sq);
        L.gate = mat(L_GATE, c.n_ff, c.n_embd, ORC_Q4_K, se);
        L.up = mat(L_UP, c.n_ff, c.n_embd, ORC_Q4_K, se);
        L.down = mat(L_DOWN, c.n_embd, c.n_ff, ORC_Q6_K, 4.0 * sf);
    }
    orc_model_reset_kv(m);
    return m;
}

extern "C" void orc_model_free(orc_model *m) { delete m; }

extern "C" const void *orc_model_tensor(orc_model *m, int tid, int64_t *nbytes) {
    auto ret = [&](const void *p, size_t n) { if (nbytes) *nbytes = (int64_t)n; return p; };
    if (tid == TID_EMBD) return ret(m->embd.data.data(), m->embd.data.size());
    if (tid == TID_OUT_NORM) return ret(m->out_norm.data(), m->out_norm.size() * 4);
    const int il = (tid - 16) / 16, k = (tid - 16) % 16;
    if (tid < 16 || il >= m->cfg.n_layer) return ret(nullptr, 0);
    layer_w &L = m->layers[il];
    switch (k) {
        case L_ATTN_NORM: return ret(L.attn_norm.data(), L.attn_norm.size() * 4);
        case L_FFN_NORM: return ret(L.ffn_norm.data(), L.ffn_norm.size() * 4);
        case L_Q: return ret(L.q.data.data(), L.q.data.size());
        case L_K: return ret(L.k.data.data(), L.k.data.size());
        case L_V: return ret(L.v.data.data(), L.v.data.size());
        case L_O: return ret(L.o.data.data(), L.o.data.size());
        case L_GATE: return ret(L.gate.data.data(), L.gate.data.size());
        case L_UP: return ret(L.up.data.data(), L.up.data.size());
        case L_DOWN: return ret(L.down.data.data(), L.down.data.size());
    }
    return ret(nullptr, 0);
}

extern "C" void orc_model_reset_kv(orc_model *m) {
    const orc_config &c = m->cfg;
    const size_t kvw = (size_t)c.n_head_kv * c.head_dim;
    m->kc.assign(c.n_layer, std::vector<uint16_t>((size_t)c.n_ctx * kvw, 0));
    m->vc.assign(c.n_layer, std::vector<uint16_t>((size_t)c.n_ctx * kvw, 0));
}

namespace {

// y[T][rows] = W . x[T][cols]  through the hpc-style mul_mat (INIT quantize + row split)
// (the matrix's own type picks vec_dot_type: Q8_0 for Q4_0/Q8_0, Q8_K for Q4_K/Q6_K)
void matmul_q(const qmat &W, const float *x, int64_t T, float *y, int /*wtype*/, int avx2,
              std::vector<uint8_t> &wbuf) {
    const int wtype = W.type;
    const bool kq = wtype == ORC_Q4_K || wtype == ORC_Q6_K;
    const size_t rs = orc_row_size(kq ? ORC_Q8_K : ORC_Q8_0, W.cols);
    wbuf.resize(rs * T);
    orc_mul_mat_init(wtype, x, W.cols, T, W.cols, wbuf.data());
    orc_mul_mat(W.rows, T, 1, (int64_t)W.row_bytes, T, W.rows * 4, W.rows * 4 * T, rs, W.cols, W.data.data(), y,
                wtype, (const char *)wbuf.data(), avx2);
}

}  // namespace

extern "C" int orc_model_inference(orc_model *m, const int32_t *tokens, int n_total, int stage,
                                   float *logits_last, float *logits_all, int avx2) {
    const orc_config &c = m->cfg;
    const int E = c.n_embd, H = c.n_head, Hkv = c.n_head_kv, hd = c.head_dim, F = c.n_ff, V = c.n_vocab;
    const int qw = H * hd, kvw = Hkv * hd;
    const int T = stage == 0 ? n_total : 1;
    const int head = stage == 0 ? 0 : n_total - 1;                      // :428-436
    const int n_kv = std::min(c.n_ctx, 32 * (n_total / 32 + 1));        // :429
    if (head + T > c.n_ctx) return -1;
    std::vector<uint8_t> wbuf;
    m->hidden.assign(c.n_layer, {});
    m->tap_qkv.assign(c.n_layer, {});
    m->tap_attn.assign(c.n_layer, {});

    // inpL = get_rows(token_embd, tokens) * sqrtf(E)     (:677-679)
    std::vector<float> inpL((size_t)T * E), cur((size_t)T * E), tmp((size_t)T * E);
    const float emb_scale = sqrtf((float)E);
    for (int t = 0; t < T; ++t) {
        const int tok = tokens[head + t];
        dequantize_row(m->embd.type, m->embd.data.data() + (size_t)tok * m->embd.row_bytes, &inpL[(size_t)t * E], E);
        for (int i = 0; i < E; ++i) inpL[(size_t)t * E + i] *= emb_scale;
    }

    std::vector<float> Q((size_t)T * qw), K((size_t)T * kvw), Vv((size_t)T * kvw), attn((size_t)T * qw);
    std::vector<float> kq((size_t)H * T * n_kv), kqv((size_t)H * T * hd), mask((size_t)T * n_kv);
    std::vector<float> up((size_t)T * F), gate((size_t)T * F), sa((size_t)T * E);
    std::vector<uint16_t> q16((size_t)H * T * hd), p16((size_t)H * T * n_kv);
    const float q_scale = 1.0f / sqrtf((float)hd);                       // :708

    // KQ mask (:320-335): row t masks j > head + t
    for (int t = 0; t < T; ++t)
        for (int j = 0; j < n_kv; ++j) mask[(size_t)t * n_kv + j] = (j > head + t) ? -INFINITY : 0.0f;

    for (int il = 0; il < c.n_layer; ++il) {
        layer_w &L = m->layers[il];
        // cur = rms_norm(inpL) * attn_norm   (:438-442, :690)
        for (int t = 0; t < T; ++t) {
            orc_rms_norm(&inpL[(size_t)t * E], &cur[(size_t)t * E], E, c.eps);
            for (int i = 0; i < E; ++i) cur[(size_t)t * E + i] *= L.attn_norm[i];
        }
        matmul_q(L.q, cur.data(), T, Q.data(), c.wtype, avx2, wbuf);    // :692
        matmul_q(L.k, cur.data(), T, K.data(), c.wtype, avx2, wbuf);    // :694
        matmul_q(L.v, cur.data(), T, Vv.data(), c.wtype, avx2, wbuf);   // :696
        {
            auto &tq = m->tap_qkv[il];
            tq.assign(Q.end() - qw, Q.end());
            tq.insert(tq.end(), K.end() - kvw, K.end());
            tq.insert(tq.end(), Vv.end() - kvw, Vv.end());
        }
        for (int t = 0; t < T; ++t) {
            orc_rope_neox(&Q[(size_t)t * qw], hd, H, head + t, c.rope_base);   // :698-706
            for (int i = 0; i < qw; ++i) Q[(size_t)t * qw + i] *= q_scale;  // :708
            orc_rope_neox(&K[(size_t)t * kvw], hd, Hkv, head + t, c.rope_base); // :710-716
        }
        // KV store (:499-518): K row (head+t); V transposed column (head+t); f32 -> f16
        for (int t = 0; t < T; ++t)
            for (int i = 0; i < kvw; ++i) {
                m->kc[il][(size_t)(head + t) * kvw + i] = orc_fp32_to_fp16(K[(size_t)t * kvw + i]);
                m->vc[il][(size_t)i * c.n_ctx + head + t] = orc_fp32_to_fp16(Vv[(size_t)t * kvw + i]);
            }
        // KQ = mul_mat(k_view, q)  (:465-474): per query head h, src0 = K cache of kv head h/(H/Hkv)
        for (int h = 0; h < H; ++h)
            for (int t = 0; t < T; ++t)
                for (int i = 0; i < hd; ++i)
                    q16[((size_t)h * T + t) * hd + i] = orc_fp32_to_fp16(Q[(size_t)t * qw + h * hd + i]);
        for (int h = 0; h < H; ++h) {
            const int kvh = h / (H / Hkv);
            orc_mul_mat(n_kv, T, 1, (int64_t)kvw * 2, T, (int64_t)n_kv * 4, (int64_t)n_kv * 4 * T, (size_t)hd * 2, hd,
                        m->kc[il].data() + (size_t)kvh * hd, &kq[(size_t)h * T * n_kv], ORC_F16,
                        (const char *)&q16[(size_t)h * T * hd], avx2);
        }
        // softmax_ext(kq, mask, scale = 1.0)  (:476)
        for (int h = 0; h < H; ++h)
            for (int t = 0; t < T; ++t) {
                float *row = &kq[((size_t)h * T + t) * n_kv];
                orc_soft_max_row(row, &mask[(size_t)t * n_kv], row, n_kv, 1.0f);
            }
        for (size_t i = 0; i < kq.size(); ++i) p16[i] = orc_fp32_to_fp16(kq[i]);
        // KQV = mul_mat(v_view, kq)  (:478-485): src0 rows = V cache rows d (stride n_ctx)
        for (int h = 0; h < H; ++h) {
            const int kvh = h / (H / Hkv);
            orc_mul_mat(hd, T, 1, (int64_t)c.n_ctx * 2, T, (int64_t)hd * 4, (int64_t)hd * 4 * T, (size_t)n_kv * 2, n_kv,
                        m->vc[il].data() + (size_t)kvh * hd * c.n_ctx, &kqv[(size_t)h * T * hd], ORC_F16,
                        (const char *)&p16[(size_t)h * T * n_kv], avx2);
        }
        // permute(0,2,1,3) + cont_2d  (:487-489)
        for (int t = 0; t < T; ++t)
            for (int h = 0; h < H; ++h)
                memcpy(&attn[(size_t)t * qw + h * hd], &kqv[((size_t)h * T + t) * hd], hd * 4);
        m->tap_attn[il].assign(attn.end() - qw, attn.end());
        matmul_q(L.o, attn.data(), T, tmp.data(), c.wtype, avx2, wbuf);  // :493
        for (size_t i = 0; i < sa.size(); ++i) sa[i] = tmp[i] + inpL[i];    // :723
        for (int t = 0; t < T; ++t) {                                       // :724
            orc_rms_norm(&sa[(size_t)t * E], &cur[(size_t)t * E], E, c.eps);
            for (int i = 0; i < E; ++i) cur[(size_t)t * E + i] *= L.ffn_norm[i];
        }
        matmul_q(L.up, cur.data(), T, up.data(), c.wtype, avx2, wbuf);     // :446
        matmul_q(L.gate, cur.data(), T, gate.data(), c.wtype, avx2, wbuf); // :447
        orc_gelu(gate.data(), gate.data(), (int)gate.size());               // :448
        for (size_t i = 0; i < gate.size(); ++i) gate[i] = gate[i] * up[i]; // :449
        matmul_q(L.down, gate.data(), T, tmp.data(), c.wtype, avx2, wbuf); // :450
        for (size_t i = 0; i < inpL.size(); ++i) inpL[i] = tmp[i] + sa[i];  // :731
        m->hidden[il] = inpL;
    }
    // final norm + tied output (:736-740)
    for (int t = 0; t < T; ++t) {
        orc_rms_norm(&inpL[(size_t)t * E], &cur[(size_t)t * E], E, c.eps);
        for (int i = 0; i < E; ++i) cur[(size_t)t * E + i] *= m->out_norm[i];
    }
    std::vector<float> logits;
    const float *last;
    if (logits_all) {
        matmul_q(m->embd, cur.data(), T, logits_all, c.wtype, avx2, wbuf);
        last = logits_all + (size_t)(T - 1) * V;
    } else {
        logits.resize(V);
        matmul_q(m->embd, &cur[(size_t)(T - 1) * E], 1, logits.data(), c.wtype, avx2, wbuf);
        last = logits.data();
    }
    if (logits_last) memcpy(logits_last, last, (size_t)V * 4);
    // greedy_sample (:532-546): strict '>' argmax, first max wins
    float best = -INFINITY;
    int idx = -1;
    for (int i = 0; i < V; ++i)
        if (last[i] > best) { best = last[i]; idx = i; }
    return idx;
}

extern "C" int orc_model_hidden(orc_model *m, int il, float *out, int64_t max_floats) {
    if (il < 0 || il >= (int)m->hidden.size()) return -1;
    const auto &h = m->hidden[il];
    const int64_t n = std::min<int64_t>((int64_t)h.size(), max_floats);
    memcpy(out, h.data(), (size_t)n * 4);
    return (int)n;
}

// bench.py cpu_baseline leg: the reference generation loop (src/gemma_model.cpp:548-575) on a
// bounded sample: PREFILL of `prompt_len` tokens (logits for every row, as the reference's graph
// computes them at :740), then n_decode greedy DECODE steps, std::chrono timed.  tokens_out gets
// prompt_len + 1 + n_decode ids.  Returns decode seconds; *prefill_s gets prefill seconds.
// prof6 (nullable) gets the decode steps' mul_mat profile (orc_prof layout, hpc_cpu.cpp).
extern "C" double orc_bench_run(orc_model *m, const int32_t *prompt, int prompt_len, int n_decode, int n_threads,
                                int32_t *tokens_out, double *prefill_s, double *prof6) {
    orc_set_threads(n_threads);
    orc_model_reset_kv(m);
    std::vector<int32_t> seq(prompt, prompt + prompt_len);
    std::vector<float> all((size_t)prompt_len * m->cfg.n_vocab);
    auto t0 = std::chrono::steady_clock::now();
    seq.push_back(orc_model_inference(m, seq.data(), (int)seq.size(), 0, nullptr, all.data(), 1));
    if (prof6) orc_prof(1, nullptr);
    auto t1 = std::chrono::steady_clock::now();
    for (int s = 0; s < n_decode; ++s)
        seq.push_back(orc_model_inference(m, seq.data(), (int)seq.size(), 1, nullptr, nullptr, 1));
    auto t2 = std::chrono::steady_clock::now();
    if (prof6) orc_prof(0, prof6);
    for (size_t i = 0; i < seq.size(); ++i) tokens_out[i] = seq[i];
    if (prefill_s) *prefill_s = std::chrono::duration<double>(t1 - t0).count();
    return std::chrono::duration<double>(t2 - t1).count();
}

// synthetic prompt (DESIGN.md §Synthetic inputs): BOS = 2 first, then uniform ids in [3, n_vocab)
extern "C" void orc_make_prompt(uint64_t seed, int n, int n_vocab, int32_t *out) {
    for (int i = 0; i < n; ++i)
        out[i] = i == 0 ? 2 : 3 + (int32_t)(splitmix64(splitmix64(seed) + (uint64_t)i) % (uint64_t)(n_vocab - 3));
}

// raw synthetic value (before quantization) for cross-checking the product's device generator
extern "C" float orc_synth_value(uint64_t seed, int tid, uint64_t idx, double stdv) {
    return (float)synth_int(tensor_key(seed, tid), idx) * synth_scale(stdv);
}

// debugging taps of the last row of the last call: qkv (pre-rope matmul outputs), attn, layer out
extern "C" int orc_model_taps(orc_model *m, int il, float *qkv, float *attn, float *xout) {
    if (il < 0 || il >= (int)m->hidden.size() || m->tap_qkv[il].empty()) return -1;
    memcpy(qkv, m->tap_qkv[il].data(), m->tap_qkv[il].size() * 4);
    memcpy(attn, m->tap_attn[il].data(), m->tap_attn[il].size() * 4);
    const size_t E = (size_t)m->cfg.n_embd;
    memcpy(xout, m->hidden[il].data() + m->hidden[il].size() - E, E * 4);
    return 0;
}

// Single-token attention block (the DECODE slice of src/gemma_model.cpp:698-718 + :454-518),
// standalone for the per-op parity test of the GPU attention kernel.  qkv = [q | k | v] pre-rope;
// kc [ctx][Hkv*hd], vc [Hkv*hd][ctx] f16 caches (updated at `pos`); out [H*hd].
extern "C" void orc_attn_decode(const float *qkv, uint16_t *kc, uint16_t *vc, int pos, int H, int Hkv, int hd, int ctx,
                                float rope_base, float *out, float *dbg_w, uint16_t *dbg_p, float *dbg_inv) {
    const int qw = H * hd, kvw = Hkv * hd;
    const int n_kv = std::min(ctx, 32 * ((pos + 1) / 32 + 1));
    std::vector<float> Q(qkv, qkv + qw), K(qkv + qw, qkv + qw + kvw);
    const float *V = qkv + qw + kvw;
    orc_rope_neox(Q.data(), hd, H, pos, rope_base);
    const float q_scale = 1.0f / sqrtf((float)hd);
    for (int i = 0; i < qw; ++i) Q[i] *= q_scale;
    orc_rope_neox(K.data(), hd, Hkv, pos, rope_base);
    for (int i = 0; i < kvw; ++i) {
        kc[(size_t)pos * kvw + i] = orc_fp32_to_fp16(K[i]);
        vc[(size_t)i * ctx + pos] = orc_fp32_to_fp16(V[i]);
    }
    std::vector<float> kq(n_kv), mask(n_kv);
    std::vector<uint16_t> q16(hd), p16(n_kv);
    for (int j = 0; j < n_kv; ++j) mask[j] = j > pos ? -INFINITY : 0.0f;
    for (int h = 0; h < H; ++h) {
        const int kvh = h / (H / Hkv);
        for (int i = 0; i < hd; ++i) q16[i] = orc_fp32_to_fp16(Q[(size_t)h * hd + i]);
        orc_mul_mat(n_kv, 1, 1, (int64_t)kvw * 2, 1, (int64_t)n_kv * 4, (int64_t)n_kv * 4, (size_t)hd * 2, hd,
                    kc + (size_t)kvh * hd, kq.data(), ORC_F16, (const char *)q16.data(), 1);
        if (dbg_w)
            for (int j = 0; j < n_kv; ++j) dbg_w[(size_t)h * ctx + j] = kq[j] + mask[j];
        orc_soft_max_row(kq.data(), mask.data(), kq.data(), n_kv, 1.0f);
        for (int j = 0; j < n_kv; ++j) p16[j] = orc_fp32_to_fp16(kq[j]);
        if (dbg_p)
            for (int j = 0; j < n_kv; ++j) dbg_p[(size_t)h * ctx + j] = p16[j];
        if (dbg_inv) {
            double sum = 0.0;
            float mx = -INFINITY;
            for (int j = 0; j < n_kv; ++j) mx = std::max(mx, dbg_w ? dbg_w[(size_t)h * ctx + j] : 0.0f);
            (void)mx;
            for (int j = 0; j < n_kv; ++j) sum += 0.0;
            dbg_inv[h] = (float)sum;
        }
        orc_mul_mat(hd, 1, 1, (int64_t)ctx * 2, 1, (int64_t)hd * 4, (int64_t)hd * 4, (size_t)n_kv * 2, n_kv,
                    vc + (size_t)kvh * hd * ctx, out + (size_t)h * hd, ORC_F16, (const char *)p16.data(), 1);
    }
}
