// ggml_api.cpp — the ggml context / tensor / graph / op surface that src/gemma_model.cpp is written
// against (SURVEY §8(b) "wide op surface"), implemented for MI355X so the reference's driver code
// can build its graphs unchanged and run them on the GPU.
//
// Host side (this file) follows ggml's conventions: tensors carry host `data` pointers into a
// context arena or a "CPU" backend buffer; views alias their source (view_src = the root tensor,
// view_offs cumulative); ggml_build_forward_expand orders nodes depth-first by their sources.
// ggml_graph_compute_with_ctx is the device executor (the hpc_graph_compute role of SURVEY §8(b)):
//   * leaves get device mirrors: weights (tensors outside backend buffers) uploaded once per data
//     pointer (immutable for the program, src/gemma_model.cpp:24-27); backend-buffer leaves the
//     graph writes into (the KV cache, via ggml_cpy) are device-authoritative after their first
//     upload; other backend-buffer leaves (tokens, positions, the mask the host writes through
//     ->data, src/gemma_model.cpp:318-335) are re-uploaded every compute;
//   * every node runs on the GPU in graph order (csrc/ggml_ops.hip; quantized MUL_MAT on the hot
//     path's k_matvec for <= 4 columns and k_gemm_x otherwise, both in ggml's AVX2 lane order);
//   * the LAST node's data is copied back to its host tensor (the one src/gemma_model.cpp:280
//     samples from).
// K-quant (Q4_K / Q6_K) src0: Q8_K INIT on the device + the K-quant dots; get_rows dequantizes
// Q4_0 / Q8_0 / Q4_K / Q6_K rows.  Not provided: ops outside the Gemma graph (they fail with an error).
#include <stdarg.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <algorithm>
#include <chrono>
#include <cmath>
#include <map>
#include <mutex>
#include <set>
#include <string>
#include <unordered_map>
#include <unordered_set>
#include <vector>

#include "../../include/gemma_hpc.h"
#include "engine_ext.h"
#include "ggml_impl.h"
#include "kernels.h"

using namespace ghip;

namespace ghip {
// GHIP_GGML_DEBUG (operational knob): the ggml executor's diagnostics on stderr — 1: why the fast
// path was not taken or failed; 2: also the per-step host phase timings
int ghip_debug_level() {
    static const int level = [] {
        const char *v = getenv("GHIP_GGML_DEBUG");
        return v ? atoi(v) : 0;
    }();
    return level;
}
}  // namespace ghip

namespace ggml_impl {

constexpr size_t kArenaAlign = 32;

size_t type_size(int t) {
    switch (t) {
        case GGML_TYPE_F32: case GGML_TYPE_I32: return 4;
        case GGML_TYPE_F16: case GGML_TYPE_I16: return 2;
        case GGML_TYPE_I8: return 1;
        case GGML_TYPE_Q4_0: return 18;
        case GGML_TYPE_Q4_1: return 20;
        case GGML_TYPE_Q5_0: return 22;
        case GGML_TYPE_Q5_1: return 24;
        case GGML_TYPE_Q8_0: return 34;
        case GGML_TYPE_Q8_1: return 36;
        case GGML_TYPE_Q2_K: return 84;
        case GGML_TYPE_Q3_K: return 110;
        case GGML_TYPE_Q4_K: return 144;
        case GGML_TYPE_Q5_K: return 176;
        case GGML_TYPE_Q6_K: return 210;
        case GGML_TYPE_Q8_K: return 292;
        default: return 0;
    }
}
int64_t blck_size(int t) {
    switch (t) {
        case GGML_TYPE_Q4_0: case GGML_TYPE_Q4_1: case GGML_TYPE_Q5_0: case GGML_TYPE_Q5_1: case GGML_TYPE_Q8_0:
        case GGML_TYPE_Q8_1: return 32;
        case GGML_TYPE_Q2_K: case GGML_TYPE_Q3_K: case GGML_TYPE_Q4_K: case GGML_TYPE_Q5_K: case GGML_TYPE_Q6_K:
        case GGML_TYPE_Q8_K: return 256;
        default: return 1;
    }
}

// tensor objects come from slabs of kSlab, kept in a process pool when their context is freed (the
// reference re-creates its ~1,000-tensor compute context every token: one heap allocation per tensor
// was a measurable part of the host's per-token time)
constexpr size_t kSlab = 512;
std::mutex slab_mu;
std::vector<ggml_tensor *> slab_pool;
ggml_tensor *slab_take(ggml_context *ctx) {
    if (ctx->slabs.empty() || ctx->slab_used == kSlab) {
        ggml_tensor *s = nullptr;
        {
            std::lock_guard<std::mutex> lk(slab_mu);
            if (!slab_pool.empty()) {
                s = slab_pool.back();
                slab_pool.pop_back();
            }
        }
        if (!s) s = new ggml_tensor[kSlab];
        ctx->slabs.push_back(s);
        ctx->slab_used = 0;
    }
    return &ctx->slabs.back()[ctx->slab_used++];
}
void slab_put(std::vector<ggml_tensor *> &slabs) {
    std::lock_guard<std::mutex> lk(slab_mu);
    for (ggml_tensor *s : slabs) {
        if (slab_pool.size() < 64) slab_pool.push_back(s);
        else delete[] s;
    }
    slabs.clear();
}

ggml_tensor *new_tensor_impl(ggml_context *ctx, ggml_type type, int n_dims, const int64_t *ne, ggml_tensor *view_src,
                             size_t view_offs) {
    ggml_tensor *t = slab_take(ctx);
    memset(t, 0, sizeof(*t));
    t->type = type;
    for (int i = 0; i < GGML_MAX_DIMS; ++i) t->ne[i] = i < n_dims ? ne[i] : 1;
    t->nb[0] = type_size(type);
    t->nb[1] = t->nb[0] * (t->ne[0] / blck_size(type));
    for (int i = 2; i < GGML_MAX_DIMS; ++i) t->nb[i] = t->nb[i - 1] * t->ne[i - 1];
    if (view_src && view_src->view_src) {  // views always point at the root tensor
        view_offs += view_src->view_offs;
        view_src = view_src->view_src;
    }
    t->view_src = view_src;
    t->view_offs = view_offs;
    if (view_src) {
        t->data = view_src->data ? (char *)view_src->data + view_offs : nullptr;
    } else if (!ctx->no_alloc) {
        const size_t nbytes = ggml_nbytes(t);
        const size_t off = (ctx->used + kArenaAlign - 1) & ~(kArenaAlign - 1);
        if (off + nbytes > ctx->mem_size) {
            fprintf(stderr, "[gemma_hip] ggml: context out of memory (%zu + %zu > %zu)\n", off, nbytes, ctx->mem_size);
            abort();
        }
        t->data = ctx->mem + off;
        ctx->used = off + nbytes;
    }
    ctx->tensors.push_back(t);
    return t;
}

}  // namespace ggml_impl
using namespace ggml_impl;

namespace {

constexpr size_t kAlign = 32;
constexpr int kGraphSize = 8192;

ggml_tensor *view_of(ggml_context *ctx, ggml_tensor *a, int n_dims, const int64_t *ne, size_t offset) {
    return new_tensor_impl(ctx, a->type, n_dims, ne, a, offset);
}

ggml_tensor *op_result(ggml_context *ctx, ggml_tensor *like, ggml_op op, ggml_tensor *s0, ggml_tensor *s1 = nullptr,
                       ggml_tensor *s2 = nullptr) {
    ggml_tensor *t = new_tensor_impl(ctx, GGML_TYPE_F32, 4, like->ne, nullptr, 0);
    t->op = op;
    t->src[0] = s0;
    t->src[1] = s1;
    t->src[2] = s2;
    return t;
}

void set_f32(ggml_tensor *t, int i, float v) { memcpy(&t->op_params[i], &v, 4); }
float get_f32(const ggml_tensor *t, int i) {
    float v;
    memcpy(&v, &t->op_params[i], 4);
    return v;
}

bool is_contiguous(const ggml_tensor *t) {
    return t->nb[0] == type_size(t->type) && t->nb[1] == t->nb[0] * (t->ne[0] / blck_size(t->type)) &&
           t->nb[2] == t->nb[1] * t->ne[1] && t->nb[3] == t->nb[2] * t->ne[2];
}

// ---- device executor state ------------------------------------------------------------------------
struct leaf_mirror {
    void *dev = nullptr;
    size_t bytes = 0;
    bool valid = false;  // device copy current (for device-authoritative leaves)
};

struct executor {
    std::recursive_mutex mu;
    bool inited = false;
    hipStream_t stream = nullptr;
    std::unordered_map<const void *, leaf_mirror> leaves;  // keyed by root host data pointer
    std::map<std::pair<const void *, int>, tiled_mat> tiled;  // quantized src0 re-tiled for the hot path
    std::unordered_set<const ggml_backend_buffer *> buffers;
    char *scratch = nullptr;
    size_t scratch_bytes = 0;
    uint16_t *gelu_tab = nullptr;
    float *rope_c = nullptr, *rope_s = nullptr;
    int rope_npos = 0, rope_dims = 0;
    float rope_base = 0.f;
};

executor &ex() {
    static executor e;
    return e;
}

bool in_backend_buffer(const void *p) {
    for (const ggml_backend_buffer *b : ex().buffers)
        if ((const char *)p >= b->mem && (const char *)p < b->mem + b->size) return true;
    return false;
}

int ensure_init() {
    executor &e = ex();
    if (e.inited) return 0;
    if (hpc_init(0)) return -1;
    GHIP_CHECK(hipStreamCreateWithFlags(&e.stream, hipStreamNonBlocking));
    std::vector<uint16_t> et, gt;
    build_f16_tables(et, gt);
    GHIP_CHECK(hipMalloc(&e.gelu_tab, 65536 * 2));
    GHIP_CHECK(hipMemcpy(e.gelu_tab, gt.data(), 65536 * 2, hipMemcpyHostToDevice));
    e.inited = true;
    return 0;
}

int ensure_rope(int npos, int n_dims, float base) {
    executor &e = ex();
    if (e.rope_c && e.rope_npos >= npos && e.rope_dims == n_dims && e.rope_base == base) return 0;
    if (e.rope_c) (void)hipFree(e.rope_c);
    if (e.rope_s) (void)hipFree(e.rope_s);
    const int n = std::max(npos, 512);
    std::vector<float> c, s;
    build_rope(n, n_dims, base, c, s);
    GHIP_CHECK(hipMalloc(&e.rope_c, c.size() * 4));
    GHIP_CHECK(hipMalloc(&e.rope_s, s.size() * 4));
    GHIP_CHECK(hipMemcpy(e.rope_c, c.data(), c.size() * 4, hipMemcpyHostToDevice));
    GHIP_CHECK(hipMemcpy(e.rope_s, s.data(), s.size() * 4, hipMemcpyHostToDevice));
    e.rope_npos = n;
    e.rope_dims = n_dims;
    e.rope_base = base;
    return 0;
}

ggml_tensor *root_of(ggml_tensor *t) { return t->view_src ? t->view_src : t; }
bool is_view_op(int op) {
    return op == GGML_OP_VIEW || op == GGML_OP_RESHAPE || op == GGML_OP_PERMUTE || op == GGML_OP_TRANSPOSE ||
           op == GGML_OP_CPY;
}

struct run_state {
    std::unordered_map<const ggml_tensor *, char *> node_dev;  // device base of computed roots
    size_t scratch_used = 0;
};

int scratch_reserve(size_t bytes) {
    executor &e = ex();
    if (e.scratch_bytes >= bytes) return 0;
    if (e.scratch) GHIP_CHECK(hipFree(e.scratch));
    e.scratch = nullptr;
    GHIP_CHECK(hipMalloc(&e.scratch, bytes));
    e.scratch_bytes = bytes;
    return 0;
}

char *scratch_take(run_state &rs, size_t bytes) {
    const size_t off = (rs.scratch_used + 255) & ~(size_t)255;
    rs.scratch_used = off + bytes;
    return ex().scratch + off;
}

// device address of any tensor in the graph (its root's mirror + the view offset)
char *dev_addr(run_state &rs, ggml_tensor *t) {
    ggml_tensor *r = root_of(t);
    const size_t off = (size_t)((char *)t->data - (char *)r->data);
    auto it = rs.node_dev.find(r);
    if (it != rs.node_dev.end()) return it->second + off;
    auto lf = ex().leaves.find(r->data);
    if (lf != ex().leaves.end()) return (char *)lf->second.dev + off;
    return nullptr;
}

gt_desc desc(run_state &rs, ggml_tensor *t) {
    gt_desc d;
    d.data = dev_addr(rs, t);
    for (int i = 0; i < 4; ++i) {
        d.ne[i] = t->ne[i];
        d.nb[i] = (int64_t)t->nb[i];
    }
    d.type = t->type;
    return d;
}

// one leaf root: make its device mirror current
int sync_leaf(ggml_tensor *r, bool graph_written) {
    executor &e = ex();
    const size_t bytes = ggml_nbytes(r);
    leaf_mirror &m = e.leaves[r->data];
    if (m.bytes < bytes) {
        if (m.dev) GHIP_CHECK(hipFree(m.dev));
        GHIP_CHECK(hipMalloc(&m.dev, bytes));
        m.bytes = bytes;
        m.valid = false;
    }
    const bool host_written_input = in_backend_buffer(r->data) && !graph_written;
    if (!m.valid || host_written_input) {
        GHIP_CHECK(hipMemcpyAsync(m.dev, r->data, bytes, hipMemcpyHostToDevice, e.stream));
        m.valid = true;
    }
    return 0;
}

const tiled_mat *tiled_weight(run_state &rs, ggml_tensor *w) {
    executor &e = ex();
    ggml_tensor *r = root_of(w);
    const auto key = std::make_pair((const void *)w->data, (int)w->type);
    auto it = e.tiled.find(key);
    if (it != e.tiled.end()) return &it->second;
    if (!is_contiguous(w)) {
        set_error("ggml mul_mat: quantized src0 must be contiguous");
        return nullptr;
    }
    tiled_mat m = alloc_tiled(w->type, w->ne[1], w->ne[0], e.stream);
    const char *src = dev_addr(rs, w);
    if (!src || launch_repack(m, (const uint8_t *)src, (int64_t)w->nb[1], e.stream)) {
        free_tiled(m);
        if (!src) set_error("ggml mul_mat: src0 has no device data");
        return nullptr;
    }
    (void)r;
    return &(e.tiled[key] = m);
}

int run_mul_mat(run_state &rs, ggml_tensor *node) {
    executor &e = ex();
    ggml_tensor *a = node->src[0], *b = node->src[1];
    if (b->type != GGML_TYPE_F32) {
        set_error("ggml mul_mat: src1 must be f32");
        return -1;
    }
    const int64_t K = a->ne[0], cols = b->ne[1] * b->ne[2] * b->ne[3];
    if (a->type == GGML_TYPE_F16) {
        // INIT: src1 -> contiguous f16 rows, then ggml_vec_dot_f16 per (row, column)
        gt_desc b16 = desc(rs, b);
        b16.type = T_F16;
        b16.data = scratch_take(rs, (size_t)(K * cols * 2));
        b16.nb[0] = 2;
        for (int i = 1; i < 4; ++i) b16.nb[i] = b16.nb[i - 1] * b16.ne[i - 1];
        if (launch_g_copy(desc(rs, b), b16, e.stream)) return -1;
        if (b->ne[2] % a->ne[2] || b->ne[3] % a->ne[3] || a->nb[0] != 2) {
            set_error("ggml mul_mat: unsupported f16 broadcast / stride");
            return -1;
        }
        return launch_g_mul_mat_f16(desc(rs, a), (const uint16_t *)b16.data, K, desc(rs, node), b->ne[1], b->ne[2],
                                    b->ne[3], e.stream);
    }
    if (a->type == GGML_TYPE_Q4_K || a->type == GGML_TYPE_Q6_K) {
        // ggml INIT quantizes src1 to Q8_K (vec_dot_type of the K-quants), then the AVX2-lane-order
        // K-quant dot per (row, column): the same kernels as the C-ABI mul_mat (csrc/kquant.hip)
        if (K % 256 || a->ne[2] != 1 || a->ne[3] != 1 || !is_contiguous(a) || b->nb[0] != 4 ||
            b->nb[1] != (size_t)K * 4 || (cols > b->ne[1] && b->nb[2] != b->nb[1] * b->ne[1])) {
            set_error("ggml mul_mat: K-quant path needs K % 256 == 0, contiguous src0 and src1 rows");
            return -1;
        }
        const int64_t nsb = K / 256;
        uint8_t *xq = (uint8_t *)scratch_take(rs, (size_t)(cols * nsb * 292));
        if (launch_quant_q8_K((const float *)dev_addr(rs, b), K, K, (int)cols, xq, nsb * 292, e.stream)) return -1;
        // >= kq_gemm_min() (default 8) columns: the MFMA GEMM (prefill_kq.hip), as the C-ABI mul_mat
        const uint8_t *wdev = (const uint8_t *)dev_addr(rs, a);
        const int64_t rb_want = nsb * (a->type == GGML_TYPE_Q4_K ? 144 : 210);
        if (cols >= kq_gemm_min() && (int64_t)a->nb[1] == rb_want &&
            ((uintptr_t)wdev & (a->type == GGML_TYPE_Q4_K ? 15 : 3)) == 0) {
            q8kx_args x;
            x.x = xq; x.x_col_stride = nsb * 292; x.nsb = (int)nsb; x.T = (int)cols;
            x.xh = (uint16_t *)scratch_take(rs, (size_t)(cols * K * 2)); x.ldh = K;
            x.xd = (float *)scratch_take(rs, (size_t)(cols * nsb * 4)); x.ldd = nsb;
            x.xm = (uint16_t *)scratch_take(rs, (size_t)(cols * nsb * 32)); x.ldm = nsb;
            if (launch_q8k_expand(x, e.stream)) return -1;
            kqg_args g;
            g.w = wdev; g.row_bytes = rb_want; g.rows = a->ne[1]; g.nsb = (int)nsb; g.T = (int)cols; g.tiled = 0;
            g.xh = x.xh; g.ldh = x.ldh; g.xd = x.xd; g.ldd = x.ldd; g.xm = x.xm; g.ldm = x.ldm;
            g.y = (float *)dev_addr(rs, node); g.ldy = a->ne[1];
            return launch_gemm_kq(a->type, g, e.stream);
        }
        kq_args k;
        k.w = wdev;
        k.row_bytes = (int64_t)a->nb[1];
        k.rows = a->ne[1];
        k.nsb = (int)nsb;
        k.x = xq;
        k.x_col_stride = nsb * 292;
        k.y = (float *)dev_addr(rs, node);
        k.y_col_stride = a->ne[1];
        k.ncols = (int)cols;
        return launch_matvec_kq(a->type, k, e.stream);
    }
    if (a->type != GGML_TYPE_Q4_0 && a->type != GGML_TYPE_Q8_0) {
        set_error("ggml mul_mat: src0 type " + std::to_string(a->type) + " not supported by the graph executor");
        return -1;
    }
    if (K % 32 || a->ne[2] != 1 || a->ne[3] != 1 || b->nb[0] != 4 || b->nb[1] != (size_t)K * 4 ||
        (cols > b->ne[1] && b->nb[2] != b->nb[1] * b->ne[1])) {
        set_error("ggml mul_mat: quantized path needs contiguous src1 rows");
        return -1;
    }
    const tiled_mat *W = tiled_weight(rs, a);
    if (!W) return -1;
    float *y = (float *)dev_addr(rs, node);
    const char *x = dev_addr(rs, b);
    if (cols <= 4) {
        mv_args m;
        m.qs = W->qs; m.sc = W->sc; m.rows = W->rows; m.n_rt = W->n_rt; m.n_bt = W->n_bt; m.nb = W->nb;
        m.x = x; m.x_col_stride = (int64_t)b->nb[1];
        m.y = y; m.y_col_stride = a->ne[1];
        m.ncols = (int)cols;
        const int grid = (int)std::min<int64_t>((W->n_rt + 3) / 4, 1024);
        return launch_matvec(a->type, 1, PRO_F32, EPI_STORE, m, grid, e.stream);
    }
    const int64_t ldq = (K + 255) / 256 * 256, ldd = ldq / 32;
    qrow_args q;
    q.x = (const float *)x; q.ldx = K; q.K = K;
    // the image the exact GEMM's form stages from: int8 (gemm_x4_i8) or f16
    const bool i8img = gemm_x4_i8();
    q.q = i8img ? (int8_t *)scratch_take(rs, (size_t)(cols * ldq)) : nullptr;
    q.qh = i8img ? nullptr : (uint16_t *)scratch_take(rs, (size_t)(cols * ldq * 2));
    q.ldq = ldq;
    q.da = (float *)scratch_take(rs, (size_t)(cols * ldd * 4));
    q.ldd = ldd;
    if (launch_quant_rows(QR_F32, q, (int)cols, e.stream)) return -1;
    gemm_args g;
    g.qs = W->qs; g.sc = W->sc; g.rows = W->rows; g.n_rt = W->n_rt; g.n_bt = W->n_bt; g.nb = W->nb;
    g.xq = q.q; g.xh = q.qh; g.ldq = ldq; g.da = q.da; g.ldd = ldd; g.T = cols; g.y = y; g.ldy = a->ne[1];
    return launch_gemm_exact(a->type, EPI_STORE, g, e.stream);
}

int run_node(run_state &rs, ggml_tensor *n) {
    executor &e = ex();
    hipStream_t s = e.stream;
    switch (n->op) {
        case GGML_OP_VIEW: case GGML_OP_RESHAPE: case GGML_OP_PERMUTE: case GGML_OP_TRANSPOSE: return 0;
        case GGML_OP_GET_ROWS: return launch_g_get_rows(desc(rs, n->src[0]), desc(rs, n->src[1]), desc(rs, n), s);
        case GGML_OP_SCALE: return launch_g_elementwise(0, desc(rs, n->src[0]), gt_desc(), desc(rs, n), get_f32(n, 0), nullptr, 0, s);
        case GGML_OP_GELU: return launch_g_elementwise(1, desc(rs, n->src[0]), gt_desc(), desc(rs, n), 0.f, e.gelu_tab, n->op_params[0], s);
        case GGML_OP_MUL: return launch_g_elementwise(2, desc(rs, n->src[0]), desc(rs, n->src[1]), desc(rs, n), 0.f, nullptr, 0, s);
        case GGML_OP_ADD: return launch_g_elementwise(3, desc(rs, n->src[0]), desc(rs, n->src[1]), desc(rs, n), 0.f, nullptr, 0, s);
        case GGML_OP_RMS_NORM: return launch_g_rms_norm(desc(rs, n->src[0]), desc(rs, n), get_f32(n, 0), s);
        case GGML_OP_CPY: case GGML_OP_CONT: return launch_g_copy(desc(rs, n->src[0]), desc(rs, n), s);
        case GGML_OP_MUL_MAT: return run_mul_mat(rs, n);
        case GGML_OP_SOFT_MAX: {
            ggml_tensor *mask = n->src[1];
            if (n->src[2] || get_f32(n, 1) != 0.0f) {
                set_error("ggml soft_max_ext: ALiBi (pos / max_bias) is not supported");
                return -1;
            }
            return launch_g_soft_max(desc(rs, n->src[0]), mask ? desc(rs, mask) : gt_desc(), mask ? 1 : 0, desc(rs, n),
                                     get_f32(n, 0), s);
        }
        case GGML_OP_ROPE: {
            const int n_dims = n->op_params[1];
            // the Gemma graph's rope: NEOX (mode 2), no YaRN extension, unit scales (src/macro.h:12-18)
            if (n->op_params[2] != 2 || get_f32(n, 6) != 1.0f || get_f32(n, 7) != 0.0f || get_f32(n, 8) != 1.0f ||
                n_dims > n->src[0]->ne[0] || n_dims % 2) {
                set_error("ggml rope: only NEOX mode with freq_scale 1, ext_factor 0, attn_factor 1 is supported");
                return -1;
            }
            // positions are a host-written input: size the cos/sin table from its values
            const ggml_tensor *pos = n->src[1];
            int maxp = 0;
            for (int64_t i = 0; i < pos->ne[0]; ++i)
                maxp = std::max(maxp, *(const int32_t *)((const char *)pos->data + i * pos->nb[0]));
            if (ensure_rope(maxp + 1, n_dims, get_f32(n, 5))) return -1;
            return launch_g_rope_neox(desc(rs, n->src[0]), desc(rs, n->src[1]), desc(rs, n), n_dims, e.rope_c, e.rope_s, s);
        }
        default:
            set_error("ggml graph: op " + std::to_string(n->op) + " not supported");
            return -1;
    }
}

// ---- the Gemma graph fast path -------------------------------------------------------------------
// build_compute_graph (src/gemma_model.cpp:665-747) emits one fixed graph per call.  When the graph
// handed to the executor is exactly that graph (verified op by op, every parameter, and the host
// inputs: tokens, positions, the causal mask, the KV write position), it runs on the
// device-resident engine (fused kernels, one hipGraph per decode token, engine.cpp) over the same
// host weights and over the executor's own device mirrors of the graph's KV-cache tensors, and the
// last node's logits are copied back like the generic path does.  Same arithmetic, same bits
// (tests/test_gpu_ggml_graph.py runs both paths).  Anything else runs node by node below.
struct gemma_match {
    gemma_hip_config cfg{};
    host_weights hw;
    std::vector<ggml_tensor *> kc, vc;  // cache roots per layer
    std::vector<int32_t> tokens;
    int T = 0;
    int pos0 = 0;
    std::vector<const ggml_tensor *> stores;  // the matched K / V cache CPY nodes
};

bool op_is(const ggml_tensor *t, int op) { return t && t->op == op; }
bool is_leaf_w(const ggml_tensor *t) { return t && t->op == GGML_OP_NONE && !t->view_src && t->data; }
const ggml_tensor *skip_views(const ggml_tensor *t) {  // through RESHAPE / VIEW / PERMUTE / TRANSPOSE
    while (t && (t->op == GGML_OP_RESHAPE || t->op == GGML_OP_VIEW || t->op == GGML_OP_PERMUTE || t->op == GGML_OP_TRANSPOSE))
        t = t->src[0];
    return t;
}

// norm * w: MUL(RMS_NORM(x), w) -> x, w, eps
bool match_norm(const ggml_tensor *t, const ggml_tensor **x, const float **w, float *eps) {
    if (!op_is(t, GGML_OP_MUL) || !op_is(t->src[0], GGML_OP_RMS_NORM) || !is_leaf_w(t->src[1]) ||
        t->src[1]->type != GGML_TYPE_F32)
        return false;
    *x = t->src[0]->src[0];
    *w = (const float *)t->src[1]->data;
    *eps = get_f32(t->src[0], 0);
    return true;
}

// pointer set for match_gemma's ancestor walk: linear probing over a power-of-two table, cleared
// by bumping a generation stamp (no per-insert allocation, no per-call clear of the table)
struct ptr_set {
    std::vector<const void *> key;
    std::vector<uint32_t> gen;
    uint32_t cur = 0;
    size_t mask = 0, count = 0;
    std::vector<const ggml_tensor *> stack;
    void grow() {  // keep the load factor <= 1/2 (a table never fills, so probes always end)
        std::vector<const void *> live;
        for (size_t i = 0; i < key.size(); ++i)
            if (gen[i] == cur) live.push_back(key[i]);
        key.assign(key.size() * 2, nullptr);
        gen.assign(key.size(), 0);
        cur = 1;
        mask = key.size() - 1;
        count = 0;
        for (const void *p : live) insert(p);
    }
    void reset(size_t n) {
        count = 0;
        size_t cap = 64;
        while (cap < 2 * n) cap <<= 1;
        if (cap > key.size()) {
            key.assign(cap, nullptr);
            gen.assign(cap, 0);
            cur = 0;
        }
        mask = key.size() - 1;
        if (++cur == 0) {  // wrapped: clear once
            std::fill(gen.begin(), gen.end(), 0u);
            cur = 1;
        }
    }
    static size_t hash(const void *p) {
        uint64_t x = (uint64_t)(uintptr_t)p;
        x ^= x >> 29;
        x *= 0xbf58476d1ce4e5b9ull;
        return (size_t)(x ^ (x >> 32));
    }
    bool insert(const void *p) {  // true if newly inserted
        for (size_t i = hash(p) & mask;; i = (i + 1) & mask) {
            if (gen[i] != cur) {
                gen[i] = cur;
                key[i] = p;
                if (++count * 2 > key.size()) grow();
                return true;
            }
            if (key[i] == p) return false;
        }
    }
    bool has(const void *p) const {
        for (size_t i = hash(p) & mask;; i = (i + 1) & mask) {
            if (gen[i] != cur) return false;
            if (key[i] == p) return true;
        }
    }
};
ptr_set &anc_set() {
    static thread_local ptr_set s;
    return s;
}

// graphs (node / leaf arrays + the visited set) pooled across contexts, like the tensor slabs
std::mutex graph_mu;
std::vector<ggml_cgraph *> graph_pool;
ggml_cgraph *graph_take() {
    ggml_cgraph *g = nullptr;
    {
        std::lock_guard<std::mutex> lk(graph_mu);
        if (!graph_pool.empty()) {
            g = graph_pool.back();
            graph_pool.pop_back();
        }
    }
    if (!g) {
        g = new ggml_cgraph();
        g->nodes = new ggml_tensor *[kGraphSize];
        g->leafs = new ggml_tensor *[kGraphSize];
        g->visited = new ptr_set();
    }
    ((ptr_set *)g->visited)->reset(1024);
    return g;
}
void graph_put(ggml_cgraph *g) {
    std::lock_guard<std::mutex> lk(graph_mu);
    if (graph_pool.size() < 8) {
        graph_pool.push_back(g);
        return;
    }
    delete (ptr_set *)g->visited;
    delete[] g->nodes;
    delete[] g->leafs;
    delete g;
}

bool match_gemma(ggml_cgraph *g, gemma_match &m, std::string &why) {
    auto fail = [&](const char *w) {
        why = w;
        return false;
    };
    const ggml_tensor *last = g->nodes[g->n_nodes - 1];
    if (!op_is(last, GGML_OP_MUL_MAT) || !is_leaf_w(last->src[0])) return fail("last node");
    const ggml_tensor *embd = last->src[0];
    const ggml_tensor *x;
    const float *onorm;
    float eps;
    if (!match_norm(last->src[1], &x, &onorm, &eps)) return fail("output norm");
    gemma_hip_config &c = m.cfg;
    c.n_embd = (int)embd->ne[0];
    c.n_vocab = (int)embd->ne[1];
    c.eps = eps;
    m.hw.embd = embd->data;
    m.hw.out_norm = onorm;
    // cache stores: root -> the CPY node writing it
    std::unordered_map<const ggml_tensor *, const ggml_tensor *> store;
    for (int i = 0; i < g->n_nodes; ++i)
        if (op_is(g->nodes[i], GGML_OP_CPY)) store[root_of(g->nodes[i]->src[1])] = g->nodes[i];
    std::vector<host_weights::layer> rev;
    const ggml_tensor *posv = nullptr, *maskv = nullptr;
    int wtype = -1, hd = 0, H = 0, Hkv = 0, nff = 0, kvhead = -1, gclamp = -1;
    float base = 0.f;
    while (op_is(x, GGML_OP_ADD)) {
        host_weights::layer L;
        // x = down(gelu(gate(n2)) * up(n2)) + sa
        const ggml_tensor *dn = x->src[0], *sa = x->src[1];
        if (!op_is(dn, GGML_OP_MUL_MAT) || !is_leaf_w(dn->src[0]) || !op_is(dn->src[1], GGML_OP_MUL)) return fail("ffn down");
        const ggml_tensor *gm = dn->src[1];
        if (!op_is(gm->src[0], GGML_OP_GELU) || !op_is(gm->src[1], GGML_OP_MUL_MAT)) return fail("gelu*up");
        const ggml_tensor *gt = gm->src[0]->src[0], *ut = gm->src[1];
        if (!op_is(gt, GGML_OP_MUL_MAT) || !is_leaf_w(gt->src[0]) || !is_leaf_w(ut->src[0]) || gt->src[1] != ut->src[1])
            return fail("gate/up");
        const int gc = gm->src[0]->op_params[0];
        if (gclamp >= 0 && gc != gclamp) return fail("gelu variants");
        gclamp = gc;
        const ggml_tensor *sx;
        if (!match_norm(gt->src[1], &sx, &L.ffn_norm, &eps) || sx != sa || eps != c.eps) return fail("ffn norm");
        L.gate = gt->src[0]->data; L.up = ut->src[0]->data; L.down = dn->src[0]->data;
        nff = (int)gt->src[0]->ne[1];
        // sa = Wo(cont(permute(kqv))) + inpL
        if (!op_is(sa, GGML_OP_ADD) || !op_is(sa->src[0], GGML_OP_MUL_MAT) || !is_leaf_w(sa->src[0]->src[0])) return fail("attn out");
        L.o = sa->src[0]->src[0]->data;
        const ggml_tensor *inp = sa->src[1];
        const ggml_tensor *cont = sa->src[0]->src[1];
        if (!op_is(cont, GGML_OP_CONT) || !op_is(cont->src[0], GGML_OP_PERMUTE)) return fail("kqv merge");
        const ggml_tensor *kqv = cont->src[0]->src[0];
        if (!op_is(kqv, GGML_OP_MUL_MAT) || !op_is(kqv->src[0], GGML_OP_VIEW) || !op_is(kqv->src[1], GGML_OP_SOFT_MAX))
            return fail("kqv");
        const ggml_tensor *sm = kqv->src[1];
        if (sm->src[2] || get_f32(sm, 0) != 1.0f || get_f32(sm, 1) != 0.0f || !op_is(sm->src[1], GGML_OP_VIEW)) return fail("softmax");
        if (maskv && sm->src[1] != maskv) return fail("mask");
        maskv = sm->src[1];
        const ggml_tensor *kq = sm->src[0];
        if (!op_is(kq, GGML_OP_MUL_MAT) || !op_is(kq->src[0], GGML_OP_VIEW) || !op_is(kq->src[1], GGML_OP_PERMUTE)) return fail("kq");
        const ggml_tensor *qs = kq->src[1]->src[0];
        if (!op_is(qs, GGML_OP_SCALE) || !op_is(qs->src[0], GGML_OP_ROPE)) return fail("q scale");
        const ggml_tensor *qr = qs->src[0];
        const ggml_tensor *qm = skip_views(qr->src[0]);
        if (!op_is(qm, GGML_OP_MUL_MAT) || !is_leaf_w(qm->src[0])) return fail("q proj");
        const ggml_tensor *n1 = qm->src[1];
        const ggml_tensor *n1x;
        if (!match_norm(n1, &n1x, &L.attn_norm, &eps) || n1x != inp || eps != c.eps) return fail("attn norm");
        L.q = qm->src[0]->data;
        hd = (int)qr->ne[0];
        H = (int)qr->ne[1];
        if (qr->op_params[1] != hd || qr->op_params[2] != 2 || get_f32(qr, 6) != 1.0f || get_f32(qr, 7) != 0.0f ||
            get_f32(qr, 8) != 1.0f)
            return fail("rope params");
        if (get_f32(qs, 0) != 1.0f / sqrtf((float)hd)) return fail("q scale value");
        if (posv && qr->src[1] != posv) return fail("positions");
        posv = qr->src[1];
        base = get_f32(qr, 5);
        // caches and their stores
        const ggml_tensor *kroot = root_of((ggml_tensor *)kq->src[0]), *vroot = root_of((ggml_tensor *)kqv->src[0]);
        auto ks = store.find(kroot), vs = store.find(vroot);
        if (ks == store.end() || vs == store.end()) return fail("kv store");
        const ggml_tensor *kr = ks->second->src[0];  // rope(reshape(k proj))
        if (!op_is(kr, GGML_OP_ROPE) || kr->src[1] != posv || kr->op_params[2] != 2 || get_f32(kr, 5) != base) return fail("k rope");
        const ggml_tensor *km = skip_views(kr->src[0]);
        const ggml_tensor *vm = skip_views(vs->second->src[0]);
        if (!op_is(km, GGML_OP_MUL_MAT) || km->src[1] != n1 || !op_is(vm, GGML_OP_MUL_MAT) || vm->src[1] != n1) return fail("k/v proj");
        L.k = km->src[0]->data;
        L.v = vm->src[0]->data;
        Hkv = (int)kr->ne[1];
        const int64_t kvw = (int64_t)Hkv * hd;
        if (kroot->type != GGML_TYPE_F16 || vroot->type != GGML_TYPE_F16 || ggml_nelements(kroot) % kvw) return fail("cache type");
        const int64_t off_k = (int64_t)((char *)ks->second->src[1]->data - (char *)kroot->data);
        const int kh = (int)(off_k / (kvw * 2));
        if (kvhead >= 0 && kh != kvhead) return fail("kv head");
        kvhead = kh;
        // the V store: view_2d(v, T, kvw, n_ctx * 2, kv_head * 2) of the transposed cache
        // (src/gemma_model.cpp:510-512): element kv_head of every dimension row
        const ggml_tensor *vview = vs->second->src[1];
        const int64_t vctx = ggml_nelements(vroot) / kvw;
        if ((int64_t)((char *)vview->data - (char *)vroot->data) != (int64_t)kh * 2 || vview->nb[1] != (size_t)vctx * 2)
            return fail("v store view");
        m.stores.push_back(ks->second);
        m.stores.push_back(vs->second);
        const int types[7] = {(int)qm->src[0]->type, (int)km->src[0]->type, (int)vm->src[0]->type, (int)sa->src[0]->src[0]->type,
                              (int)gt->src[0]->type, (int)ut->src[0]->type, (int)dn->src[0]->type};
        for (int t : types)
            if (t != types[0] || (wtype >= 0 && t != wtype)) return fail("mixed layer types");
        wtype = types[0];
        rev.push_back(L);
        m.kc.push_back((ggml_tensor *)kroot);
        m.vc.push_back((ggml_tensor *)vroot);
        x = inp;
    }
    // x0 = get_rows(token_embd, tokens) * sqrt(E)
    if (!op_is(x, GGML_OP_SCALE) || !op_is(x->src[0], GGML_OP_GET_ROWS) || x->src[0]->src[0] != embd ||
        get_f32(x, 0) != sqrtf((float)c.n_embd))
        return fail("embedding");
    if (rev.empty() || !posv || !maskv) return fail("no layers");
    std::reverse(rev.begin(), rev.end());
    std::reverse(m.kc.begin(), m.kc.end());
    std::reverse(m.vc.begin(), m.vc.end());
    m.hw.layers = rev;
    if (wtype != GGML_TYPE_Q4_0 && wtype != GGML_TYPE_Q8_0) return fail("layer type (fast path: Q4_0 / Q8_0)");
    if ((int)embd->type != wtype && embd->type != GGML_TYPE_Q6_K) return fail("token_embd type");
    c.n_layer = (int)rev.size();
    c.n_head = H; c.n_head_kv = Hkv; c.head_dim = hd; c.n_ff = nff;
    c.n_ctx = (int)(ggml_nelements(m.kc[0]) / ((int64_t)Hkv * hd));
    c.wtype = wtype;
    c.out_type = embd->type == GGML_TYPE_Q6_K ? T_Q6_K : 0;
    c.rope_base = base;
    c.gelu_clamp = gclamp;
    // host inputs: tokens, positions, mask (the engine derives the causal mask and n_kv itself)
    const ggml_tensor *tok = x->src[0]->src[1];
    m.T = (int)tok->ne[0];
    if (tok->type != GGML_TYPE_I32 || posv->ne[0] != m.T || posv->type != GGML_TYPE_I32) return fail("inputs");
    m.tokens.assign((const int32_t *)tok->data, (const int32_t *)tok->data + m.T);
    const int32_t *pv = (const int32_t *)posv->data;
    m.pos0 = pv[0];
    for (int i = 0; i < m.T; ++i)
        if (pv[i] != m.pos0 + i) return fail("positions not consecutive");
    if (m.T > 1 && m.pos0 != 0) return fail("multi-token graph not starting at 0");
    if (kvhead != m.pos0) return fail("kv head != position");
    const int64_t kv_n = maskv->ne[0];
    if (kv_n != std::min<int64_t>(c.n_ctx, 32 * ((m.pos0 + m.T) / 32 + 1)) || maskv->ne[1] != m.T || maskv->type != GGML_TYPE_F32)
        return fail("n_kv");
    for (int i = 0; i < m.T; ++i) {
        const float *row = (const float *)((const char *)maskv->data + (size_t)i * maskv->nb[1]);
        for (int64_t j = 0; j < kv_n; ++j) {
            const bool masked = j > m.pos0 + i;
            if (masked ? !(row[j] == -INFINITY) : row[j] != 0.0f) return fail("mask not causal");
        }
    }
    if (last->ne[1] != m.T || !last->data || !is_contiguous(last)) return fail("output rows");
    // exactly that graph: every node is an ancestor of the logits or one of the matched cache
    // stores (an extra side node, e.g. a second output or another CPY, would be skipped otherwise)
    // (a flat open-addressing pointer set reused across calls: the per-token check allocates nothing)
    ptr_set &anc = anc_set();
    anc.reset(4 * (size_t)(g->n_nodes + g->n_leafs) + 64);
    std::vector<const ggml_tensor *> &stack = anc.stack;
    stack.clear();
    stack.push_back(last);
    for (const ggml_tensor *st : m.stores) stack.push_back(st);
    while (!stack.empty()) {
        const ggml_tensor *t = stack.back();
        stack.pop_back();
        if (!t || !anc.insert(t)) continue;
        for (int k = 0; k < GGML_MAX_SRC; ++k)
            if (t->src[k]) stack.push_back(t->src[k]);
    }
    for (int i = 0; i < g->n_nodes; ++i)
        if (!anc.has(g->nodes[i])) return fail("extra node");
    return true;
}

struct fast_engine {
    gemma_engine *e = nullptr;
    const void *key_embd = nullptr, *key_q0 = nullptr;
    uint64_t fp = 0;  // fingerprint of the first bytes of token_embd and layer 0's q
    int n_ctx = 0, n_layer = 0;
    std::vector<const void *> kv_keys;
    std::vector<const void *> weights;  // every host weight the engine copied
};
fast_engine &fast() {
    static fast_engine f;
    return f;
}
uint64_t fingerprint(const void *a, const void *b) {
    uint64_t h = 1469598103934665603ull;
    for (const void *p : {a, b}) {
        const unsigned char *c = (const unsigned char *)p;
        for (int i = 0; i < 256; ++i) h = (h ^ c[i]) * 1099511628211ull;
    }
    return h;
}
void drop_fast() {
    fast_engine &f = fast();
    if (f.e) gemma_engine_free(f.e);
    f = fast_engine{};
}

// 1 = ran on the engine, 0 = not the Gemma graph (run generically), -1 = error
double now_us() {
    return (double)std::chrono::duration_cast<std::chrono::nanoseconds>(std::chrono::steady_clock::now().time_since_epoch()).count() * 1e-3;
}

int try_fast(ggml_cgraph *g) {
    // GHIP_GGML_FAST=0: every graph node by node (operational knob: the executor's generic path)
    static const bool on = !getenv("GHIP_GGML_FAST") || atoi(getenv("GHIP_GGML_FAST"));
    const bool prof = ghip_debug_level() >= 2;
    if (!on || g->n_nodes < 8) return 0;
    const double t0 = prof ? now_us() : 0.0;
    gemma_match m;
    std::string why;
    if (!match_gemma(g, m, why)) {
        if (ghip_debug_level() >= 1) fprintf(stderr, "[gemma_hip] ggml fast path not taken: %s\n", why.c_str());
        return 0;
    }
    const double tm = prof ? now_us() : 0.0;
    executor &ex_ = ex();
    // the caches' device mirrors (device-authoritative: the graph writes them)
    std::vector<uint16_t *> kc, vc;
    std::vector<const void *> kv_keys;
    for (int il = 0; il < m.cfg.n_layer; ++il) {
        if (sync_leaf(m.kc[il], true) || sync_leaf(m.vc[il], true)) return -1;
        kc.push_back((uint16_t *)ex_.leaves[m.kc[il]->data].dev);
        vc.push_back((uint16_t *)ex_.leaves[m.vc[il]->data].dev);
        kv_keys.push_back(kc.back());
        kv_keys.push_back(vc.back());
    }
    GHIP_CHECK(hipStreamSynchronize(ex_.stream));
    const double ts = prof ? now_us() : 0.0;
    fast_engine &f = fast();
    // the engine serves positions below n_ctx - 1 (its RoPE / history tables); the last slot runs
    // node by node
    if (m.T == 1 && m.pos0 + 1 >= m.cfg.n_ctx) return 0;
    const uint64_t fp = fingerprint(m.hw.embd, m.hw.layers[0].q);
    if (!f.e || f.key_embd != m.hw.embd || f.key_q0 != m.hw.layers[0].q || f.fp != fp || f.n_ctx != m.cfg.n_ctx ||
        f.n_layer != m.cfg.n_layer || f.kv_keys != kv_keys) {
        drop_fast();
        int dev = 0;
        (void)hipGetDevice(&dev);
        f.e = gemma_engine_create_ext(&m.cfg, dev, m.hw, kc, vc);
        if (!f.e) return -1;
        f.key_embd = m.hw.embd;
        f.key_q0 = m.hw.layers[0].q;
        f.fp = fp;
        f.n_ctx = m.cfg.n_ctx;
        f.n_layer = m.cfg.n_layer;
        f.kv_keys = kv_keys;
        f.weights = {m.hw.embd, m.hw.out_norm};
        for (const host_weights::layer &L : m.hw.layers)
            for (const void *w : {L.q, L.k, L.v, L.o, L.gate, L.up, L.down, (const void *)L.attn_norm, (const void *)L.ffn_norm})
                f.weights.push_back(w);
    }
    ggml_tensor *last = g->nodes[g->n_nodes - 1];
    const double t1 = prof ? now_us() : 0.0;
    if (prof) fprintf(stderr, "[gemma_hip] fast path T=%d: match %.1f us, cache mirrors %.1f us, engine setup %.1f us\n", m.T,
                      tm - t0, ts - tm, t1 - ts);
    const int rc = m.T == 1 ? gemma_engine_ext_decode(f.e, m.tokens[0], m.pos0, (float *)last->data)
                            : gemma_engine_ext_prefill(f.e, m.tokens.data(), m.T, (float *)last->data);
    if (rc) {  // the engine could not serve this graph: node by node instead (same results)
        if (ghip_debug_level() >= 1) fprintf(stderr, "[gemma_hip] ggml fast path failed: %s\n", last_error().c_str());
        set_error("");
        return 0;
    }
    if (prof) fprintf(stderr, "[gemma_hip] fast path T=%d: match+sync %.1f us, engine %.1f us\n", m.T, t1 - t0, now_us() - t1);
    for (int il = 0; il < m.cfg.n_layer; ++il) {
        ex_.leaves[m.kc[il]->data].valid = true;
        ex_.leaves[m.vc[il]->data].valid = true;
    }
    return 1;
}

}  // namespace

// hpc_flush_weights / hpc_unregister_weight (capi.cpp): the fast path's engine holds device copies of
// the graph's host weights; drop it when they go (host == nullptr: always)
void ggml_fast_drop(const void *host) {
    std::lock_guard<std::recursive_mutex> lk(ex().mu);
    fast_engine &f = fast();
    if (!f.e) return;
    if (host && std::find(f.weights.begin(), f.weights.end(), host) == f.weights.end()) return;
    drop_fast();
}

extern "C" {

// ---- context and sizes -------------------------------------------------------------------------
// Arenas of freed contexts are kept (up to 4) and handed to the next ggml_init of the same size:
// the reference re-creates its compute context every token (src/gemma_model.cpp), and a fresh
// mmap'ed arena page-faults on every first write (the logits row alone is 256 pages).  ggml_init
// never promised zeroed memory.
namespace {
std::mutex arena_mu;
std::vector<std::pair<size_t, char *>> arena_pool;
char *arena_get(size_t bytes) {
    std::lock_guard<std::mutex> lk(arena_mu);
    for (size_t i = 0; i < arena_pool.size(); ++i)
        if (arena_pool[i].first == bytes) {
            char *p = arena_pool[i].second;
            arena_pool.erase(arena_pool.begin() + (long)i);
            return p;
        }
    return (char *)aligned_alloc(64, bytes);
}
void arena_put(size_t bytes, char *p) {
    if (bytes > ((size_t)256 << 20)) {  // weight contexts (the whole GGUF blob): give the memory back
        free(p);
        return;
    }
    std::lock_guard<std::mutex> lk(arena_mu);
    if (arena_pool.size() >= 4) {
        free(arena_pool.front().second);
        arena_pool.erase(arena_pool.begin());
    }
    arena_pool.emplace_back(bytes, p);
}
}  // namespace

struct ggml_context *ggml_init(struct ggml_init_params params) {
    ggml_context *c = new ggml_context();
    c->mem_size = params.mem_size;
    c->no_alloc = params.no_alloc;
    if (params.mem_buffer) {
        c->mem = (char *)params.mem_buffer;
    } else if (params.mem_size) {
        c->mem = arena_get((params.mem_size + 63) & ~(size_t)63);
        c->owns_mem = true;
    }
    return c;
}

void ggml_free(struct ggml_context *ctx) {
    if (!ctx) return;
    // the address span of this context's data: the executor caches and the fast path's weights are
    // checked tensor by tensor only when one of their keys falls inside it (the per-token compute
    // context of the reference's loop never holds one, and hundreds of lookups per token are host time)
    uintptr_t lo = UINTPTR_MAX, hi = 0;
    for (const ggml_tensor *t : ctx->tensors)
        if (!t->view_src && t->data) {
            lo = std::min(lo, (uintptr_t)t->data);
            hi = std::max(hi, (uintptr_t)t->data + 1);
        }
    auto inside = [&](const void *p) { return (uintptr_t)p >= lo && (uintptr_t)p < hi; };
    {
        std::lock_guard<std::recursive_mutex> lk(ex().mu);
        bool any = false;
        for (const auto &kv : ex().leaves) any = any || inside(kv.first);
        for (const auto &kv : ex().tiled) any = any || inside(kv.first.first);
        // a freed compute context's tensors leave the executor's caches keyed by their data
        if (any)
        for (ggml_tensor *t : ctx->tensors) {
            if (t->view_src || !t->data) continue;
            auto it = ex().leaves.find(t->data);
            if (it != ex().leaves.end() && !in_backend_buffer(t->data)) {
                (void)hipFree(it->second.dev);
                ex().leaves.erase(it);
            }
            auto tt = ex().tiled.find(std::make_pair((const void *)t->data, (int)t->type));
            if (tt != ex().tiled.end()) {
                free_tiled(tt->second);
                ex().tiled.erase(tt);
            }
        }
        // a freed weight context takes the fast path's device copy of its weights with it; under the
        // executor's lock, which try_fast holds while it runs that engine
        fast_engine &f = fast();
        if (f.e && std::any_of(f.weights.begin(), f.weights.end(), inside)) {
            const std::unordered_set<const void *> ws(f.weights.begin(), f.weights.end());
            for (ggml_tensor *t : ctx->tensors)
                if (t->data && ws.count(t->data)) {
                    drop_fast();
                    break;
                }
        }
    }
    slab_put(ctx->slabs);
    for (ggml_cgraph *g : ctx->graphs) graph_put(g);
    if (ctx->owns_mem) arena_put((ctx->mem_size + 63) & ~(size_t)63, ctx->mem);
    delete ctx;
}

size_t ggml_tensor_overhead(void) { return sizeof(struct ggml_tensor) + 32; }
size_t ggml_graph_overhead(void) { return sizeof(struct ggml_cgraph) + 2 * kGraphSize * sizeof(void *) + 32; }
size_t ggml_get_mem_size(const struct ggml_context *ctx) { return ctx->mem_size; }
size_t ggml_type_size(enum ggml_type type) { return type_size(type); }
int64_t ggml_blck_size(enum ggml_type type) { return blck_size(type); }
size_t ggml_row_size(enum ggml_type type, int64_t ne) { return type_size(type) * ne / blck_size(type); }
size_t ggml_element_size(const struct ggml_tensor *t) { return type_size(t->type); }
int64_t ggml_nelements(const struct ggml_tensor *t) { return t->ne[0] * t->ne[1] * t->ne[2] * t->ne[3]; }
size_t ggml_nbytes(const struct ggml_tensor *t) {
    size_t nbytes = type_size(t->type);
    if (blck_size(t->type) == 1) {
        for (int i = 0; i < GGML_MAX_DIMS; ++i) nbytes += (size_t)(t->ne[i] - 1) * t->nb[i];
    } else {
        nbytes = (size_t)(t->ne[0] * t->nb[0] / blck_size(t->type));
        for (int i = 1; i < GGML_MAX_DIMS; ++i) nbytes += (size_t)(t->ne[i] - 1) * t->nb[i];
    }
    return nbytes;
}

// ---- ggml's naming of derived tensors (ggml.c of the reference's era): a view / reshape / permute /
// transpose / cont is named "<src> (view)" etc., a cpy "<dst> (copy of <src>)" (or "<src> (copy)" when
// the destination is unnamed), and ggml_build_forward_expand names the still unnamed nodes
// "node_<index>" and leaves "leaf_<index>".  These are the names the reference's graph listings hold
// (tensor_dump/tensor_in_target_cgraph; the source-side dump at src/gemma_model.cpp:240-248).  Plain
// concatenation instead of snprintf: ~600 tensors per decode graph on the host path.
static void name_cat(ggml_tensor *t, const char *a, const char *b, const char *c = nullptr, const char *d = nullptr) {
    char *o = t->name, *const end = t->name + GGML_MAX_NAME - 1;
    for (const char *p : {a, b, c, d})
        for (; p && *p && o < end; ++p) *o++ = *p;
    *o = 0;
}
static void name_index(char *name, const char *prefix, int i) {
    char digits[12];
    int n = 0;
    do {
        digits[n++] = (char)('0' + i % 10);
        i /= 10;
    } while (i > 0 && n < 11);
    char *o = name;
    for (const char *p = prefix; *p; ++p) *o++ = *p;
    while (n > 0) *o++ = digits[--n];
    *o = 0;
}

// ---- tensors and views -------------------------------------------------------------------------
struct ggml_tensor *ggml_new_tensor(struct ggml_context *ctx, enum ggml_type type, int n_dims, const int64_t *ne) {
    return new_tensor_impl(ctx, type, n_dims, ne, nullptr, 0);
}
struct ggml_tensor *ggml_new_tensor_1d(struct ggml_context *ctx, enum ggml_type type, int64_t ne0) {
    return new_tensor_impl(ctx, type, 1, &ne0, nullptr, 0);
}
struct ggml_tensor *ggml_new_tensor_2d(struct ggml_context *ctx, enum ggml_type type, int64_t ne0, int64_t ne1) {
    const int64_t ne[2] = {ne0, ne1};
    return new_tensor_impl(ctx, type, 2, ne, nullptr, 0);
}
struct ggml_tensor *ggml_new_tensor_3d(struct ggml_context *ctx, enum ggml_type type, int64_t ne0, int64_t ne1,
                                       int64_t ne2) {
    const int64_t ne[3] = {ne0, ne1, ne2};
    return new_tensor_impl(ctx, type, 3, ne, nullptr, 0);
}
struct ggml_tensor *ggml_view_1d(struct ggml_context *ctx, struct ggml_tensor *a, int64_t ne0, size_t offset) {
    ggml_tensor *t = view_of(ctx, a, 1, &ne0, offset);
    t->op = GGML_OP_VIEW;
    t->src[0] = a;
    name_cat(t, a->name, " (view)");
    return t;
}
struct ggml_tensor *ggml_view_2d(struct ggml_context *ctx, struct ggml_tensor *a, int64_t ne0, int64_t ne1, size_t nb1,
                                 size_t offset) {
    const int64_t ne[2] = {ne0, ne1};
    ggml_tensor *t = view_of(ctx, a, 2, ne, offset);
    t->nb[1] = nb1;
    t->nb[2] = t->nb[1] * ne1;
    t->nb[3] = t->nb[2];
    t->op = GGML_OP_VIEW;
    t->src[0] = a;
    name_cat(t, a->name, " (view)");
    return t;
}
struct ggml_tensor *ggml_view_3d(struct ggml_context *ctx, struct ggml_tensor *a, int64_t ne0, int64_t ne1, int64_t ne2,
                                 size_t nb1, size_t nb2, size_t offset) {
    const int64_t ne[3] = {ne0, ne1, ne2};
    ggml_tensor *t = view_of(ctx, a, 3, ne, offset);
    t->nb[1] = nb1;
    t->nb[2] = nb2;
    t->nb[3] = t->nb[2] * ne2;
    t->op = GGML_OP_VIEW;
    t->src[0] = a;
    name_cat(t, a->name, " (view)");
    return t;
}
struct ggml_tensor *ggml_reshape_2d(struct ggml_context *ctx, struct ggml_tensor *a, int64_t ne0, int64_t ne1) {
    const int64_t ne[2] = {ne0, ne1};
    ggml_tensor *t = view_of(ctx, a, 2, ne, 0);
    t->op = GGML_OP_RESHAPE;
    t->src[0] = a;
    name_cat(t, a->name, " (reshaped)");
    return t;
}
struct ggml_tensor *ggml_reshape_3d(struct ggml_context *ctx, struct ggml_tensor *a, int64_t ne0, int64_t ne1,
                                    int64_t ne2) {
    const int64_t ne[3] = {ne0, ne1, ne2};
    ggml_tensor *t = view_of(ctx, a, 3, ne, 0);
    t->op = GGML_OP_RESHAPE;
    t->src[0] = a;
    name_cat(t, a->name, " (reshaped)");
    return t;
}
struct ggml_tensor *ggml_permute(struct ggml_context *ctx, struct ggml_tensor *a, int axis0, int axis1, int axis2,
                                 int axis3) {
    ggml_tensor *t = view_of(ctx, a, 4, a->ne, 0);
    const int ax[4] = {axis0, axis1, axis2, axis3};
    for (int i = 0; i < 4; ++i) {
        t->ne[ax[i]] = a->ne[i];
        t->nb[ax[i]] = a->nb[i];
    }
    t->op = GGML_OP_PERMUTE;
    t->src[0] = a;
    name_cat(t, a->name, " (permuted)");
    return t;
}
struct ggml_tensor *ggml_transpose(struct ggml_context *ctx, struct ggml_tensor *a) {
    ggml_tensor *t = view_of(ctx, a, 4, a->ne, 0);
    for (int i = 0; i < 4; ++i) t->nb[i] = a->nb[i];
    t->ne[0] = a->ne[1];
    t->ne[1] = a->ne[0];
    t->nb[0] = a->nb[1];
    t->nb[1] = a->nb[0];
    t->op = GGML_OP_TRANSPOSE;
    t->src[0] = a;
    name_cat(t, a->name, " (transposed)");
    return t;
}
struct ggml_tensor *ggml_cont_2d(struct ggml_context *ctx, struct ggml_tensor *a, int64_t ne0, int64_t ne1) {
    const int64_t ne[2] = {ne0, ne1};
    ggml_tensor *t = new_tensor_impl(ctx, a->type, 2, ne, nullptr, 0);
    t->op = GGML_OP_CONT;
    t->src[0] = a;
    name_cat(t, a->name, " (cont)");
    return t;
}
struct ggml_tensor *ggml_set_name(struct ggml_tensor *t, const char *name) {
    snprintf(t->name, sizeof(t->name), "%s", name);
    return t;
}
struct ggml_tensor *ggml_format_name(struct ggml_tensor *t, const char *fmt, ...) {
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(t->name, sizeof(t->name), fmt, ap);
    va_end(ap);
    return t;
}
const char *ggml_get_name(const struct ggml_tensor *t) { return t->name; }
const char *ggml_op_name(enum ggml_op op) {
    static const char *const names[GGML_OP_COUNT] = {"NONE", "GET_ROWS", "SCALE", "RMS_NORM", "MUL", "ADD", "MUL_MAT",
                                                     "ROPE", "SOFT_MAX", "GELU", "CPY", "CONT", "VIEW", "RESHAPE",
                                                     "PERMUTE", "TRANSPOSE"};
    return (int)op >= 0 && op < GGML_OP_COUNT ? names[op] : "?";
}
struct ggml_tensor *ggml_get_tensor(struct ggml_context *ctx, const char *name) {
    for (ggml_tensor *t : ctx->tensors)
        if (strcmp(t->name, name) == 0) return t;
    return nullptr;
}

// ---- ops ---------------------------------------------------------------------------------------
struct ggml_tensor *ggml_get_rows(struct ggml_context *ctx, struct ggml_tensor *a, struct ggml_tensor *b) {
    const int64_t ne[2] = {a->ne[0], b->ne[0]};
    ggml_tensor *t = new_tensor_impl(ctx, GGML_TYPE_F32, 2, ne, nullptr, 0);
    t->op = GGML_OP_GET_ROWS;
    t->src[0] = a;
    t->src[1] = b;
    return t;
}
struct ggml_tensor *ggml_scale(struct ggml_context *ctx, struct ggml_tensor *a, float s) {
    ggml_tensor *t = op_result(ctx, a, GGML_OP_SCALE, a);
    set_f32(t, 0, s);
    return t;
}
struct ggml_tensor *ggml_rms_norm(struct ggml_context *ctx, struct ggml_tensor *a, float eps) {
    ggml_tensor *t = op_result(ctx, a, GGML_OP_RMS_NORM, a);
    set_f32(t, 0, eps);
    return t;
}
struct ggml_tensor *ggml_mul(struct ggml_context *ctx, struct ggml_tensor *a, struct ggml_tensor *b) {
    return op_result(ctx, a, GGML_OP_MUL, a, b);
}
struct ggml_tensor *ggml_add(struct ggml_context *ctx, struct ggml_tensor *a, struct ggml_tensor *b) {
    return op_result(ctx, a, GGML_OP_ADD, a, b);
}
struct ggml_tensor *ggml_mul_mat(struct ggml_context *ctx, struct ggml_tensor *a, struct ggml_tensor *b) {
    const int64_t ne[4] = {a->ne[1], b->ne[1], b->ne[2], b->ne[3]};
    ggml_tensor *t = new_tensor_impl(ctx, GGML_TYPE_F32, 4, ne, nullptr, 0);
    t->op = GGML_OP_MUL_MAT;
    t->src[0] = a;
    t->src[1] = b;
    return t;
}
struct ggml_tensor *ggml_rope_custom(struct ggml_context *ctx, struct ggml_tensor *a, struct ggml_tensor *b, int n_dims,
                                     int mode, int n_ctx, int n_orig_ctx, float freq_base, float freq_scale,
                                     float ext_factor, float attn_factor, float beta_fast, float beta_slow) {
    ggml_tensor *t = op_result(ctx, a, GGML_OP_ROPE, a, b);
    // ggml's param layout: n_past(0), n_dims, mode, n_ctx, n_orig_ctx, then the floats
    t->op_params[0] = 0;
    t->op_params[1] = n_dims;
    t->op_params[2] = mode;
    t->op_params[3] = n_ctx;
    t->op_params[4] = n_orig_ctx;
    set_f32(t, 5, freq_base);
    set_f32(t, 6, freq_scale);
    set_f32(t, 7, ext_factor);
    set_f32(t, 8, attn_factor);
    set_f32(t, 9, beta_fast);
    set_f32(t, 10, beta_slow);
    return t;
}
struct ggml_tensor *ggml_soft_max_ext(struct ggml_context *ctx, struct ggml_tensor *a, struct ggml_tensor *mask,
                                      struct ggml_tensor *pos, float scale, float max_bias) {
    ggml_tensor *t = op_result(ctx, a, GGML_OP_SOFT_MAX, a, mask, pos);
    set_f32(t, 0, scale);
    set_f32(t, 1, max_bias);
    return t;
}
struct ggml_tensor *ggml_gelu(struct ggml_context *ctx, struct ggml_tensor *a) {
    ggml_tensor *t = op_result(ctx, a, GGML_OP_GELU, a);
    const char *clamp = getenv("GEMMA_HIP_GELU_CLAMP");  // later-ggml clamp variant
    t->op_params[0] = clamp && atoi(clamp) ? 1 : 0;
    return t;
}
struct ggml_tensor *ggml_cpy(struct ggml_context *ctx, struct ggml_tensor *a, struct ggml_tensor *b) {
    ggml_tensor *t = view_of(ctx, b, 4, b->ne, 0);
    for (int i = 0; i < 4; ++i) t->nb[i] = b->nb[i];
    t->op = GGML_OP_CPY;
    t->src[0] = a;
    t->src[1] = b;
    if (b->name[0]) name_cat(t, b->name, " (copy of ", a->name, ")");
    else name_cat(t, a->name, " (copy)");
    return t;
}

// ---- graphs ------------------------------------------------------------------------------------
struct ggml_cgraph *ggml_new_graph(struct ggml_context *ctx) {
    ggml_cgraph *g = graph_take();
    g->size = kGraphSize;
    g->grads = nullptr;
    g->n_nodes = g->n_leafs = 0;
    ctx->graphs.push_back(g);
    return g;
}

static void visit(ggml_cgraph *g, ptr_set &seen, ggml_tensor *t) {
    if (!t || !seen.insert(t)) return;
    for (int i = 0; i < GGML_MAX_SRC; ++i) visit(g, seen, t->src[i]);
    if (t->op == GGML_OP_NONE) {
        if (g->n_leafs < g->size) {
            if (!t->name[0]) name_index(t->name, "leaf_", g->n_leafs);
            g->leafs[g->n_leafs++] = t;
        }
    } else {
        if (g->n_nodes >= g->size) {
            fprintf(stderr, "[gemma_hip] ggml: graph full\n");
            abort();
        }
        if (!t->name[0]) name_index(t->name, "node_", g->n_nodes);
        g->nodes[g->n_nodes++] = t;
    }
}

void ggml_build_forward_expand(struct ggml_cgraph *g, struct ggml_tensor *t) {
    // the graph keeps its visited set: rebuilding it from nodes + leafs on every call made the
    // reference's per-layer expands quadratic (~2.5 ms of host time per Gemma-2B decode graph)
    visit(g, *(ptr_set *)g->visited, t);
}

enum ggml_status ggml_graph_compute_with_ctx(struct ggml_context *ctx, struct ggml_cgraph *g, int n_threads) {
    (void)ctx;
    (void)n_threads;
    executor &e = ex();
    std::lock_guard<std::recursive_mutex> lk(e.mu);
    set_error("");
    if (ensure_init()) return GGML_STATUS_FAILED;
    if (g->n_nodes == 0) return GGML_STATUS_SUCCESS;
    const int fr = try_fast(g);  // the Gemma graph: the device-resident engine
    if (fr != 0) return fr > 0 ? GGML_STATUS_SUCCESS : GGML_STATUS_FAILED;
    // leaves the graph writes into (ggml_cpy destinations): device-authoritative
    std::unordered_set<const void *> written;
    for (int i = 0; i < g->n_nodes; ++i)
        if (g->nodes[i]->op == GGML_OP_CPY) written.insert(root_of(g->nodes[i]->src[1])->data);
    // leaf roots (graph leaves, and the roots of views over them)
    std::vector<ggml_tensor *> roots;
    std::unordered_set<ggml_tensor *> node_set(g->nodes, g->nodes + g->n_nodes), seen;
    auto add_root = [&](ggml_tensor *t) {
        ggml_tensor *r = root_of(t);
        if (!node_set.count(r) && !seen.count(r)) {
            seen.insert(r);
            roots.push_back(r);
        }
    };
    for (int i = 0; i < g->n_leafs; ++i) add_root(g->leafs[i]);
    for (int i = 0; i < g->n_nodes; ++i) {
        if (g->nodes[i]->view_src) add_root(g->nodes[i]);
        for (int k = 0; k < GGML_MAX_SRC; ++k)
            if (g->nodes[i]->src[k]) add_root(g->nodes[i]->src[k]);
    }
    for (ggml_tensor *r : roots) {
        if (!r->data) {
            set_error("ggml graph: leaf tensor without data");
            return GGML_STATUS_FAILED;
        }
        if (sync_leaf(r, written.count(r->data) > 0)) return GGML_STATUS_FAILED;
    }
    // device memory for computed roots, plus per-op scratch
    size_t need = 0;
    for (int i = 0; i < g->n_nodes; ++i)
        if (!g->nodes[i]->view_src) need += (ggml_nbytes(g->nodes[i]) + 255) & ~(size_t)255;
    size_t extra = 0;
    for (int i = 0; i < g->n_nodes; ++i) {
        const ggml_tensor *n = g->nodes[i];
        if (n->op == GGML_OP_MUL_MAT) {
            const int64_t K = n->src[0]->ne[0], cols = n->src[1]->ne[1] * n->src[1]->ne[2] * n->src[1]->ne[3];
            const int64_t ldq = (K + 255) / 256 * 256;
            extra = std::max<size_t>(extra, (size_t)(cols * ldq * 2 + cols * ldq / 8 + cols * K * 2 + 1024));
        }
    }
    if (scratch_reserve(need + extra + 4096)) return GGML_STATUS_ALLOC_FAILED;
    run_state rs;
    for (int i = 0; i < g->n_nodes; ++i)
        if (!g->nodes[i]->view_src) rs.node_dev[g->nodes[i]] = scratch_take(rs, ggml_nbytes(g->nodes[i]));
    const size_t node_end = rs.scratch_used;
    for (int i = 0; i < g->n_nodes; ++i) {
        rs.scratch_used = node_end;  // per-op scratch is reused node after node
        if (run_node(rs, g->nodes[i])) return GGML_STATUS_FAILED;
    }
    for (const void *w : written) ex().leaves[w].valid = true;
    // the last node back to the host (what src/gemma_model.cpp:280 reads)
    ggml_tensor *last = g->nodes[g->n_nodes - 1];
    if (last->data) {
        const char *src = dev_addr(rs, last);
        if (!is_contiguous(last)) {
            set_error("ggml graph: last node not contiguous");
            return GGML_STATUS_FAILED;
        }
        if (hipMemcpyAsync(last->data, src, ggml_nbytes(last), hipMemcpyDeviceToHost, e.stream) != hipSuccess)
            return GGML_STATUS_FAILED;
    }
    if (hipStreamSynchronize(e.stream) != hipSuccess) {
        set_error("ggml graph: device error");
        return GGML_STATUS_FAILED;
    }
    return GGML_STATUS_SUCCESS;
}

int hpc_graph_compute(struct ggml_cgraph *graph) {
    return ggml_graph_compute_with_ctx(nullptr, graph, 1) == GGML_STATUS_SUCCESS ? 0 : -1;
}

// ---- backend ("CPU" buffers in host memory, mirrored by the executor) ---------------------------
static ggml_backend_buffer_type g_cpu_buft = {"CPU"};
ggml_backend_buffer_type_t ggml_backend_cpu_buffer_type(void) { return &g_cpu_buft; }

ggml_backend_buffer_t ggml_backend_alloc_ctx_tensors_from_buft(struct ggml_context *ctx, ggml_backend_buffer_type_t buft) {
    (void)buft;
    size_t total = 0;
    for (ggml_tensor *t : ctx->tensors)
        if (!t->data && !t->view_src) total += (ggml_nbytes(t) + kAlign - 1) & ~(kAlign - 1);
    ggml_backend_buffer *b = new ggml_backend_buffer();
    b->size = total;
    b->mem = (char *)aligned_alloc(64, (total + 63) & ~(size_t)63);
    size_t off = 0;
    for (ggml_tensor *t : ctx->tensors) {
        if (t->data || t->view_src) continue;
        t->data = b->mem + off;
        off += (ggml_nbytes(t) + kAlign - 1) & ~(kAlign - 1);
        b->tensors.push_back(t);
    }
    for (ggml_tensor *t : ctx->tensors)
        if (t->view_src && !t->data && t->view_src->data) t->data = (char *)t->view_src->data + t->view_offs;
    std::lock_guard<std::recursive_mutex> lk(ex().mu);
    ex().buffers.insert(b);
    return b;
}

void ggml_backend_buffer_clear(ggml_backend_buffer_t b, uint8_t value) {
    memset(b->mem, value, b->size);
    std::lock_guard<std::recursive_mutex> lk(ex().mu);
    for (ggml_tensor *t : b->tensors) {  // device mirrors re-upload from the cleared host copy
        auto it = ex().leaves.find(t->data);
        if (it != ex().leaves.end()) it->second.valid = false;
    }
}
const char *ggml_backend_buffer_name(ggml_backend_buffer_t b) {
    (void)b;
    return "CPU (MI355X-mirrored)";
}
size_t ggml_backend_buffer_get_size(ggml_backend_buffer_t b) { return b->size; }
void ggml_backend_buffer_free(ggml_backend_buffer_t b) {
    if (!b) return;
    std::lock_guard<std::recursive_mutex> lk(ex().mu);
    for (ggml_tensor *t : b->tensors) {
        auto it = ex().leaves.find(t->data);
        if (it != ex().leaves.end()) {
            (void)hipFree(it->second.dev);
            ex().leaves.erase(it);
        }
    }
    ex().buffers.erase(b);
    free(b->mem);
    delete b;
}

void ggml_backend_tensor_set(struct ggml_tensor *t, const void *data, size_t offset, size_t size) {
    memcpy((char *)t->data + offset, data, size);
    std::lock_guard<std::recursive_mutex> lk(ex().mu);
    ggml_tensor *r = root_of(t);
    auto it = ex().leaves.find(r->data);
    if (it != ex().leaves.end() && it->second.valid) {  // keep a device-authoritative mirror current
        const size_t off = (size_t)((char *)t->data - (char *)r->data) + offset;
        if (hipMemcpy((char *)it->second.dev + off, data, size, hipMemcpyHostToDevice) != hipSuccess)
            it->second.valid = false;
    }
}
void ggml_backend_tensor_get(const struct ggml_tensor *t, void *data, size_t offset, size_t size) {
    memcpy(data, (const char *)t->data + offset, size);
}

}  // extern "C"
