// capi.cpp — the narrow drop-in: `mul_mat` with the exact src/hpc.h:22-32 signature, plus the
// device-lifecycle entry points that replace the OpenCL runtime (src/opencl.h:22-38).
//
// Reference behaviour restated (src/hpc.cpp:216-273): output addressing
// dst + (c % ne1)*nb1 + (c / ne1)*nb2 + r*4 for r < ne01, c < ne11*ne12; src0 rows at stride nb01;
// src1 already converted by ggml's INIT into `wdata` (row_size bytes per column).  Differences:
// every row is computed (on the GPU; the reference's GPU share is verify-only), the
// `vec_dot` pointer is not called, and errors are recorded instead of exit(1) when
// hpc_set_error_mode(0) is selected.
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <algorithm>
#include <map>
#include <mutex>
#include <tuple>

#include "../../include/gemma_hpc.h"
#include "ggml_impl.h"
#include "kernels.h"

namespace ghip {
tiled_mat alloc_tiled(int type, int64_t rows, int64_t K, hipStream_t s);
void free_tiled(tiled_mat &m);
}  // namespace ghip

using namespace ghip;

namespace {

struct weight_key {
    const void *host;
    int type;
    int64_t ne00, ne01;
    size_t nb01;
    bool operator<(const weight_key &o) const {
        return std::tie(host, type, ne00, ne01, nb01) < std::tie(o.host, o.type, o.ne00, o.ne01, o.nb01);
    }
};

struct hpc_state {
    bool inited = false;
    int device = 0;
    hipStream_t stream = nullptr;
    std::map<weight_key, tiled_mat> weights;
    std::map<weight_key, uint8_t *> raw_weights;  // K-quants: ggml row-major super-blocks, packed rows
    void *scratch = nullptr;
    size_t scratch_bytes = 0;
    void *host_stage = nullptr;
    size_t host_stage_bytes = 0;
    int exit_on_error = 1;
    int ks = 1;  // K split of the quantized matvec (tests exercise 1/2/4/8)
    std::recursive_mutex mu;
};

hpc_state &st() {
    static hpc_state s;
    return s;
}

void fail(const std::string &msg) {
    set_error(msg);
    if (st().exit_on_error) {
        fprintf(stderr, "[gemma_hip] mul_mat: %s\n", msg.c_str());
        exit(1);
    }
}

int ensure_scratch(size_t bytes) {
    hpc_state &s = st();
    if (s.scratch_bytes >= bytes) return 0;
    if (s.scratch) GHIP_CHECK(hipFree(s.scratch));
    s.scratch = nullptr;
    GHIP_CHECK(hipMalloc(&s.scratch, bytes));
    s.scratch_bytes = bytes;
    return 0;
}

const tiled_mat *get_weight(const weight_key &k) {
    hpc_state &s = st();
    auto it = s.weights.find(k);
    if (it != s.weights.end()) return &it->second;
    const int bb = k.type == T_Q4_0 ? 18 : 34;
    const int64_t row_bytes = k.ne00 / 32 * bb;
    uint8_t *dev_rows = nullptr;
    if (hipMalloc(&dev_rows, (size_t)(row_bytes * k.ne01)) != hipSuccess) {
        set_error("mul_mat: weight upload alloc failed");
        return nullptr;
    }
    // rows are row_bytes long at stride nb01 on the host
    if (hipMemcpy2D(dev_rows, row_bytes, k.host, k.nb01, row_bytes, k.ne01, hipMemcpyHostToDevice) != hipSuccess) {
        (void)hipFree(dev_rows);
        set_error("mul_mat: weight upload failed");
        return nullptr;
    }
    tiled_mat m = alloc_tiled(k.type, k.ne01, k.ne00, s.stream);
    if (launch_repack(m, dev_rows, row_bytes, s.stream) != 0 || hipStreamSynchronize(s.stream) != hipSuccess) {
        (void)hipFree(dev_rows);
        free_tiled(m);
        return nullptr;
    }
    (void)hipFree(dev_rows);
    return &(s.weights[k] = m);
}

// K-quant rows (Q4_K 144 B / Q6_K 210 B per 256 values) stay in ggml layout, rows packed
int64_t kq_row_bytes(int type, int64_t ne00) { return ne00 / 256 * (type == T_Q4_K ? 144 : 210); }

const uint8_t *get_raw_weight(const weight_key &k) {
    hpc_state &s = st();
    auto it = s.raw_weights.find(k);
    if (it != s.raw_weights.end()) return it->second;
    const int64_t row_bytes = kq_row_bytes(k.type, k.ne00);
    uint8_t *dev = nullptr;
    if (hipMalloc(&dev, (size_t)(row_bytes * k.ne01)) != hipSuccess) {
        set_error("mul_mat: weight upload alloc failed");
        return nullptr;
    }
    if (hipMemcpy2D(dev, row_bytes, k.host, k.nb01, row_bytes, k.ne01, hipMemcpyHostToDevice) != hipSuccess) {
        (void)hipFree(dev);
        set_error("mul_mat: weight upload failed");
        return nullptr;
    }
    return s.raw_weights[k] = dev;
}

}  // namespace

extern "C" int hpc_init(int device) {
    hpc_state &s = st();
    std::lock_guard<std::recursive_mutex> lk(s.mu);
    set_error("");
    if (s.inited) return 0;
    GHIP_CHECK(hipSetDevice(device));
    GHIP_CHECK(hipStreamCreateWithFlags(&s.stream, hipStreamNonBlocking));
    s.device = device;
    s.inited = true;
    return 0;
}

extern "C" void hpc_shutdown(void) {
    hpc_state &s = st();
    std::lock_guard<std::recursive_mutex> lk(s.mu);
    if (!s.inited) return;
    for (auto &kv : s.weights) free_tiled(kv.second);
    s.weights.clear();
    for (auto &kv : s.raw_weights) (void)hipFree(kv.second);
    s.raw_weights.clear();
    if (s.scratch) (void)hipFree(s.scratch);
    if (s.host_stage) (void)hipHostFree(s.host_stage);
    s.scratch = s.host_stage = nullptr;
    s.scratch_bytes = s.host_stage_bytes = 0;
    (void)hipStreamDestroy(s.stream);
    s.stream = nullptr;
    s.inited = false;
}

extern "C" int hpc_last_error(char *buf, size_t len) {
    const std::string &e = last_error();
    if (buf && len) {
        const size_t n = e.size() < len - 1 ? e.size() : len - 1;
        memcpy(buf, e.data(), n);
        buf[n] = 0;
    }
    return (int)e.size();
}

extern "C" void hpc_set_error_mode(int exit_on_error) { st().exit_on_error = exit_on_error; }

extern "C" int hpc_weight_cache_entries(void) { return (int)(st().weights.size() + st().raw_weights.size()); }

// drops every cached device copy of the host weight at `host` (any type/shape); returns how many.
// The cache is keyed by the host pointer: a caller that frees or rewrites a src0 buffer calls this
// first, or a later buffer at the same address would be served the stale device copy.
extern "C" int hpc_unregister_weight(const void *host) {
    ggml_fast_drop(host);
    hpc_state &s = st();
    std::lock_guard<std::recursive_mutex> lk(s.mu);
    if (s.inited) (void)hipStreamSynchronize(s.stream);  // no launch may still read a freed copy
    int n = 0;
    for (auto it = s.weights.begin(); it != s.weights.end();) {
        if (it->first.host == host) {
            free_tiled(it->second);
            it = s.weights.erase(it);
            ++n;
        } else {
            ++it;
        }
    }
    for (auto it = s.raw_weights.begin(); it != s.raw_weights.end();) {
        if (it->first.host == host) {
            (void)hipFree(it->second);
            it = s.raw_weights.erase(it);
            ++n;
        } else {
            ++it;
        }
    }
    return n;
}

extern "C" void hpc_flush_weights(void) {
    ggml_fast_drop(nullptr);
    hpc_state &s = st();
    std::lock_guard<std::recursive_mutex> lk(s.mu);
    if (s.inited) (void)hipStreamSynchronize(s.stream);
    for (auto &kv : s.weights) free_tiled(kv.second);
    s.weights.clear();
    for (auto &kv : s.raw_weights) (void)hipFree(kv.second);
    s.raw_weights.clear();
}

extern "C" void hpc_set_matvec_ks(int ks) { st().ks = ks > 0 ? ks : 1; }

namespace ghip {
// the tiled device copy of a registered (or already mul_mat'ed) Q4_0 / Q8_0 host weight with rows
// of K values, any row count: the ggml fast path's engine copies its weights from here, device to
// device, instead of uploading them from the host a second time
// Only dense registrations qualify (nb01 = the row size of (type, K): upload_rows copies rows as
// if they were contiguous; a strided view sharing the base pointer would hand it the wrong rows),
// and of those the one with the most rows.
bool registered_tiled(const void *host, int type, int64_t K, tiled_mat *out) {
    hpc_state &s = st();
    std::lock_guard<std::recursive_mutex> lk(s.mu);
    const size_t dense = (size_t)(K / 32) * (type == T_Q4_0 ? 18 : 34);
    const tiled_mat *best = nullptr;
    int64_t best_rows = -1;
    for (const auto &kv : s.weights)
        if (kv.first.host == host && kv.first.type == type && kv.first.ne00 == K && (size_t)kv.first.nb01 == dense &&
            kv.first.ne01 > best_rows) {
            best = &kv.second;
            best_rows = kv.first.ne01;
        }
    if (!best) return false;
    *out = *best;
    return true;
}
}  // namespace ghip

extern "C" int hpc_register_weight(const void *host, int type, int64_t ne00, int64_t ne01, size_t nb01) {
    hpc_state &s = st();
    std::lock_guard<std::recursive_mutex> lk(s.mu);
    if (hpc_init(s.device)) return -1;
    if (type == T_Q4_K || type == T_Q6_K) {
        if (ne00 % 256) {
            set_error("hpc_register_weight: K-quant rows need ne00 % 256 == 0");
            return -1;
        }
        return get_raw_weight({host, type, ne00, ne01, nb01}) ? 0 : -1;
    }
    if ((type != T_Q4_0 && type != T_Q8_0) || ne00 % 32) {
        set_error("hpc_register_weight: unsupported type/shape");
        return -1;
    }
    return get_weight({host, type, ne00, ne01, nb01}) ? 0 : -1;
}

extern "C" void hpc_set_kq_gemm_min(int min_cols) { set_kq_gemm_min(min_cols); }
extern "C" void hpc_set_gemm_x4(int on) { set_gemm_x4(on); }

extern "C" void mul_mat(int64_t ne01, int64_t ne11, int64_t ne12, int64_t nb01, int64_t ne1, int64_t nb1, int64_t nb2,
                        size_t row_size, int64_t shared_edge, struct ggml_tensor *src0, struct ggml_tensor *src1,
                        struct ggml_tensor *dst, ggml_vec_dot_t vec_dot, enum ggml_type src0_type,
                        const char *wdata) {
    (void)src1;
    (void)vec_dot;
    hpc_state &s = st();
    std::lock_guard<std::recursive_mutex> lk(s.mu);
    set_error("");
    if (hpc_init(s.device)) return fail(last_error());
    const int64_t col_num = ne11 * ne12;
    if (col_num <= 0 || ne01 <= 0) return;
    const int type = (int)src0_type;
    float *dev_dst = nullptr;
    const char *dev_w = nullptr;
    const size_t dst_bytes = (size_t)(ne01 * col_num) * 4;
    const size_t w_bytes = (size_t)col_num * row_size;
    if (type == T_Q4_0 || type == T_Q8_0) {
        if (shared_edge % 32) return fail("quantized mul_mat needs shared_edge % 32 == 0");
        const tiled_mat *W = get_weight({src0->data, type, shared_edge, ne01, (size_t)nb01});
        if (!W) return fail(last_error());
        if (ensure_scratch(dst_bytes + w_bytes + 256)) return fail(last_error());
        dev_dst = (float *)s.scratch;
        dev_w = (const char *)s.scratch + ((dst_bytes + 255) & ~(size_t)255);
        if (hipMemcpyAsync((void *)dev_w, wdata, w_bytes, hipMemcpyHostToDevice, s.stream) != hipSuccess)
            return fail("mul_mat: wdata upload failed");
        mv_args a;
        a.qs = W->qs; a.sc = W->sc; a.rows = W->rows; a.n_rt = W->n_rt; a.n_bt = W->n_bt; a.nb = W->nb;
        a.x = dev_w; a.x_col_stride = (int64_t)row_size;
        a.y = dev_dst; a.y_col_stride = ne01;
        a.ncols = (int)col_num;
        int ks = s.ks;
        if (ks == KS_RR && !matvec_rr_supported(type, W->n_bt)) ks = 8;
        while (ks > 1 && ks != KS_RR && (W->n_bt % ks || matvec_lds_bytes(type, ks, W->n_bt, W->n_bt / ks) > 160 * 1024)) ks >>= 1;
        const int grid = ks > 1 ? (int)std::min<int64_t>(W->n_rt, 1024) : (int)std::min<int64_t>((W->n_rt + 3) / 4, 1024);
        if (launch_matvec(type, ks, PRO_Q8, EPI_STORE, a, grid, s.stream)) return fail(last_error());
    } else if (type == T_Q4_K || type == T_Q6_K) {
        // vec_dot_type Q8_K: wdata holds col_num Q8_K rows (row_size = K/256 * 292 bytes)
        if (shared_edge % 256 || row_size != (size_t)(shared_edge / 256 * 292))
            return fail("K-quant mul_mat needs shared_edge % 256 == 0 and Q8_K wdata rows");
        const uint8_t *W = get_raw_weight({src0->data, type, shared_edge, ne01, (size_t)nb01});
        if (!W) return fail(last_error());
        // >= kq_gemm_min() (default 8) columns: the MFMA GEMM (prefill_kq.hip) against the f16 image
        // of the Q8_K columns; fewer: the dot4 matvec / T-column kernel
        const bool mfma = col_num >= kq_gemm_min();
        const int64_t nsb = shared_edge / 256;
        auto al = [](size_t b) { return (b + 255) & ~(size_t)255; };
        const size_t xh_bytes = mfma ? (size_t)col_num * shared_edge * 2 : 0, xd_bytes = mfma ? (size_t)col_num * nsb * 4 : 0;
        const size_t xm_bytes = mfma ? (size_t)col_num * nsb * 32 : 0;
        if (ensure_scratch(al(dst_bytes) + al(w_bytes) + al(xh_bytes) + al(xd_bytes) + xm_bytes + 256)) return fail(last_error());
        dev_dst = (float *)s.scratch;
        dev_w = (const char *)s.scratch + al(dst_bytes);
        if (hipMemcpyAsync((void *)dev_w, wdata, w_bytes, hipMemcpyHostToDevice, s.stream) != hipSuccess)
            return fail("mul_mat: wdata upload failed");
        if (mfma) {
            uint8_t *base = (uint8_t *)dev_w + al(w_bytes);
            q8kx_args x;
            x.x = (const uint8_t *)dev_w; x.x_col_stride = (int64_t)row_size; x.nsb = (int)nsb; x.T = (int)col_num;
            x.xh = (uint16_t *)base; x.ldh = shared_edge;
            x.xd = (float *)(base + al(xh_bytes)); x.ldd = nsb;
            x.xm = (uint16_t *)(base + al(xh_bytes) + al(xd_bytes)); x.ldm = nsb;
            if (launch_q8k_expand(x, s.stream)) return fail(last_error());
            kqg_args g;
            g.w = W; g.row_bytes = kq_row_bytes(type, shared_edge); g.rows = ne01; g.nsb = (int)nsb; g.T = (int)col_num;
            g.tiled = 0;
            g.xh = x.xh; g.ldh = x.ldh; g.xd = x.xd; g.ldd = x.ldd; g.xm = x.xm; g.ldm = x.ldm;
            g.y = dev_dst; g.ldy = ne01;
            if (launch_gemm_kq(type, g, s.stream)) return fail(last_error());
        } else {
        kq_args a;
        a.w = W; a.row_bytes = kq_row_bytes(type, shared_edge); a.rows = ne01; a.nsb = (int)(shared_edge / 256);
        a.x = (const uint8_t *)dev_w; a.x_col_stride = (int64_t)row_size;
        a.y = dev_dst; a.y_col_stride = ne01; a.ncols = (int)col_num;
        if (launch_matvec_kq(type, a, s.stream)) return fail(last_error());
        }
    } else if (type == T_F16) {
        // src0 (e.g. a KV-cache view) changes between calls: upload the ne01 rows every time
        const size_t K = (size_t)shared_edge;
        const size_t src_bytes = (size_t)ne01 * K * 2;
        if (ensure_scratch(dst_bytes + w_bytes + src_bytes + 512)) return fail(last_error());
        dev_dst = (float *)s.scratch;
        dev_w = (const char *)s.scratch + ((dst_bytes + 255) & ~(size_t)255);
        uint16_t *dev_src = (uint16_t *)(dev_w + ((w_bytes + 255) & ~(size_t)255));
        if (hipMemcpy2DAsync(dev_src, K * 2, src0->data, (size_t)nb01, K * 2, (size_t)ne01, hipMemcpyHostToDevice,
                             s.stream) != hipSuccess)
            return fail("mul_mat: src0 upload failed");
        if (hipMemcpyAsync((void *)dev_w, wdata, w_bytes, hipMemcpyHostToDevice, s.stream) != hipSuccess)
            return fail("mul_mat: wdata upload failed");
        if (launch_mul_mat_f16(dev_src, (int64_t)K, ne01, (const uint16_t *)dev_w, (int64_t)(row_size / 2), col_num,
                               (int64_t)K, dev_dst, s.stream))
            return fail(last_error());
    } else {
        // src/hpc.cpp:132-143,162-166: no kernel for this type
        return fail("kernel is null (unsupported src0 type " + std::to_string(type) + ")");
    }
    // copy back with the reference's dst addressing
    if (s.host_stage_bytes < dst_bytes) {
        if (s.host_stage) (void)hipHostFree(s.host_stage);
        if (hipHostMalloc(&s.host_stage, dst_bytes, 0) != hipSuccess) return fail("mul_mat: host stage alloc failed");
        s.host_stage_bytes = dst_bytes;
    }
    if (hipMemcpyAsync(s.host_stage, dev_dst, dst_bytes, hipMemcpyDeviceToHost, s.stream) != hipSuccess ||
        hipStreamSynchronize(s.stream) != hipSuccess)
        return fail("mul_mat: result download failed");
    const float *res = (const float *)s.host_stage;
    char *d = (char *)dst->data;
    for (int64_t c = 0; c < col_num; ++c)
        memcpy(d + (c % ne1) * nb1 + (c / ne1) * nb2, res + c * ne01, (size_t)ne01 * 4);
}

// ---- per-op test entry for the prefill GEMM (tests/test_gpu_prefill.py) -------------------------
// W: ggml row-major blocks [rows][K/32] of `type`; X: [T][K] f32.  Quantizes X like ggml's INIT
// (Q8_0, AVX2 semantics) and runs the int8 MFMA GEMM: Y[T][rows].  xq/da (optional) return the
// activation image for a bit-exact check of the quantizer.
static int test_gemm(bool exact, int type, int64_t rows, int64_t K, int64_t T, const void *W, const float *X, float *Y,
                     int8_t *xq_out, float *da_out) {
    set_error("");
    if ((type != T_Q4_0 && type != T_Q8_0) || K % 32 || rows <= 0 || T <= 0) {
        set_error("gemma_test_gemm: bad arguments");
        return -1;
    }
    const int bb = type == T_Q4_0 ? 18 : 34;
    const int64_t row_bytes = K / 32 * bb, ldq = (K + 255) / 256 * 256, ldd = ldq / 32;
    uint8_t *d_rows = nullptr;
    float *d_x = nullptr, *d_y = nullptr, *d_da = nullptr;
    int8_t *d_q = nullptr;
    uint16_t *d_h = nullptr;
    GHIP_CHECK(hipMalloc(&d_rows, (size_t)(row_bytes * rows)));
    GHIP_CHECK(hipMalloc(&d_x, (size_t)(T * K * 4)));
    GHIP_CHECK(hipMalloc(&d_y, (size_t)(T * rows * 4)));
    GHIP_CHECK(hipMalloc(&d_q, (size_t)(T * ldq)));
    GHIP_CHECK(hipMalloc(&d_da, (size_t)(T * ldd * 4)));
    GHIP_CHECK(hipMalloc(&d_h, (size_t)(T * ldq * 2)));
    GHIP_CHECK(hipMemcpy(d_rows, W, (size_t)(row_bytes * rows), hipMemcpyHostToDevice));
    GHIP_CHECK(hipMemcpy(d_x, X, (size_t)(T * K * 4), hipMemcpyHostToDevice));
    tiled_mat m = alloc_tiled(type, rows, K, nullptr);
    int r = launch_repack(m, d_rows, row_bytes, nullptr);
    qrow_args qa;
    qa.x = d_x; qa.ldx = K; qa.K = K; qa.q = d_q; qa.qh = exact ? d_h : nullptr; qa.ldq = ldq; qa.da = d_da; qa.ldd = ldd;
    if (r == 0) r = launch_quant_rows(QR_F32, qa, (int)T, nullptr);
    gemm_args g;
    g.qs = m.qs; g.sc = m.sc; g.rows = rows; g.n_rt = m.n_rt; g.n_bt = m.n_bt; g.nb = m.nb;
    g.xq = d_q; g.xh = d_h; g.ldq = ldq; g.da = d_da; g.ldd = ldd; g.T = T; g.y = d_y; g.ldy = rows;
    if (r == 0) r = exact ? launch_gemm_exact(type, EPI_STORE, g, nullptr) : launch_gemm_q(type, EPI_STORE, g, nullptr);
    if (r == 0) GHIP_CHECK(hipDeviceSynchronize());
    if (r == 0) {
        GHIP_CHECK(hipMemcpy(Y, d_y, (size_t)(T * rows * 4), hipMemcpyDeviceToHost));
        if (xq_out)
            GHIP_CHECK(hipMemcpy2D(xq_out, (size_t)K, d_q, (size_t)ldq, (size_t)K, (size_t)T, hipMemcpyDeviceToHost));
        if (da_out)
            GHIP_CHECK(hipMemcpy2D(da_out, (size_t)(K / 32 * 4), d_da, (size_t)(ldd * 4), (size_t)(K / 32 * 4), (size_t)T,
                                   hipMemcpyDeviceToHost));
    }
    free_tiled(m);
    void *bufs[] = {d_rows, d_x, d_y, d_q, d_da, d_h};
    for (void *p : bufs) (void)hipFree(p);
    return r;
}

extern "C" int gemma_test_gemm(int type, int64_t rows, int64_t K, int64_t T, const void *W, const float *X, float *Y,
                               int8_t *xq_out, float *da_out) {
    return test_gemm(false, type, rows, K, T, W, X, Y, xq_out, da_out);
}

extern "C" int gemma_test_gemm_exact(int type, int64_t rows, int64_t K, int64_t T, const void *W, const float *X,
                                     float *Y, int8_t *xq_out, float *da_out) {
    return test_gemm(true, type, rows, K, T, W, X, Y, xq_out, da_out);
}

// ---- K-quant matvec timing (bench.py): random bytes of the right shape, `iters` launches timed
// with hipEvents on one stream; returns avg µs and the algorithmic bytes per launch
extern "C" double gemma_kq_time(int type, int64_t rows, int64_t K, int iters, double *algo_bytes) {
    set_error("");
    if ((type != T_Q4_K && type != T_Q6_K) || K % 256 || rows <= 0 || iters <= 0) {
        set_error("gemma_kq_time: bad arguments");
        return -1.0;
    }
    const int64_t rb = kq_row_bytes(type, K), nsb = K / 256;
    const size_t wbytes = (size_t)(rb * rows);
    // rotate over enough copies that each launch reads cold weights (> the 256 MiB Infinity Cache)
    const int copies = (int)std::max<int64_t>(1, std::min<int64_t>(16, (int64_t)(768ull << 20) / (int64_t)wbytes));
    uint8_t *w = nullptr, *x = nullptr;
    float *y = nullptr;
    if (hipMalloc(&w, wbytes * copies) != hipSuccess || hipMalloc(&x, (size_t)nsb * 292) != hipSuccess ||
        hipMalloc(&y, (size_t)rows * 4) != hipSuccess) {
        set_error("gemma_kq_time: alloc failed");
        return -1.0;
    }
    // valid-looking data: bytes 0x11 with small fp16 scales (value does not change the timing)
    (void)hipMemset(w, 0x11, wbytes * copies);
    (void)hipMemset(x, 0x01, (size_t)nsb * 292);
    hipStream_t s;
    (void)hipStreamCreate(&s);
    kq_args a;
    a.row_bytes = rb; a.rows = rows; a.nsb = (int)nsb; a.x = x; a.x_col_stride = nsb * 292; a.y = y; a.y_col_stride = rows;
    // the engine's lane-contiguous layout (the bytes are arbitrary either way)
    a.tiled = type == T_Q4_K || K % 2048 == 0;
    int r = 0;
    for (int i = 0; i < 3 && !r; ++i) { a.w = w + (size_t)(i % copies) * wbytes; r = launch_matvec_kq(type, a, s); }
    hipEvent_t e0, e1;
    (void)hipEventCreate(&e0);
    (void)hipEventCreate(&e1);
    (void)hipEventRecord(e0, s);
    for (int i = 0; i < iters && !r; ++i) {
        a.w = w + (size_t)(i % copies) * wbytes;
        r = launch_matvec_kq(type, a, s);
    }
    (void)hipEventRecord(e1, s);
    (void)hipEventSynchronize(e1);
    float ms = 0.f;
    (void)hipEventElapsedTime(&ms, e0, e1);
    (void)hipEventDestroy(e0);
    (void)hipEventDestroy(e1);
    (void)hipStreamDestroy(s);
    (void)hipFree(w);
    (void)hipFree(x);
    (void)hipFree(y);
    if (r) return -1.0;
    if (algo_bytes) *algo_bytes = (double)wbytes + (double)nsb * 292 + (double)rows * 4;
    return (double)ms * 1e3 / iters;
}
