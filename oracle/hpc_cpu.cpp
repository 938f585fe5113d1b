// hpc_cpu.cpp — ORACLE (test infrastructure only; see oracle.h header).
//
// Restates the reference's CPU hot path:
//   * src/thread_pool.{h,cpp}: a mutex + condition-variable task queue returning futures,
//     created with N_THREADS_MUL_MAT_CPU = 4 workers (src/macro.h:21, src/app.cpp:35);
//   * src/hpc.cpp:216-273 `mul_mat`: cpu_row_num = ceil(ne01*ratio/N)*N, row_per_core =
//     cpu_row_num/N, one `mul_mat_sub` task per worker, then future.get() on each;
//   * src/hpc.cpp:15-41 `mul_mat_sub`: rows outer, columns inner, one vec_dot per output with
//     dst address (c % ne1)*nb1 + (c / ne1)*nb2 + r*4.
// ratio is fixed at 1.0 (every row on the CPU): the shipped 0.9 split leaves GPU rows unwritten
// because the OpenCL kernels only verify, so 1.0 is the only valid reference path.
#include <atomic>
#include <chrono>
#include <condition_variable>
#include <functional>
#include <future>
#include <memory>
#include <mutex>
#include <queue>
#include <thread>
#include <vector>

#include <math.h>
#include <string.h>

#include "oracle.h"

namespace {

class task_pool {
  public:
    explicit task_pool(int n) {
        for (int i = 0; i < n; ++i)
            workers_.emplace_back([this] {
                for (;;) {
                    std::function<void()> task;
                    {
                        std::unique_lock<std::mutex> lk(mu_);
                        cv_.wait(lk, [this] { return stop_ || !tasks_.empty(); });
                        if (stop_ && tasks_.empty()) return;
                        task = std::move(tasks_.front());
                        tasks_.pop();
                    }
                    task();
                }
            });
    }
    ~task_pool() {
        {
            std::lock_guard<std::mutex> lk(mu_);
            stop_ = true;
        }
        cv_.notify_all();
        for (auto &w : workers_) w.join();
    }
    std::future<void> submit(std::function<void()> fn) {
        auto t = std::make_shared<std::packaged_task<void()>>(std::move(fn));
        std::future<void> f = t->get_future();
        {
            std::lock_guard<std::mutex> lk(mu_);
            tasks_.emplace([t] { (*t)(); });
        }
        cv_.notify_one();
        return f;
    }
    int size() const { return (int)workers_.size(); }

  private:
    std::vector<std::thread> workers_;
    std::queue<std::function<void()>> tasks_;
    std::mutex mu_;
    std::condition_variable cv_;
    bool stop_ = false;
};

// Fork-join pool for the bench's "fixed" leg (NOT the reference's design): workers spin on a
// generation counter (then yield), the caller runs share 0 itself, completion is one atomic count.
// No allocation, lock or futex per mul_mat; the reference pool above pays a packaged_task, a
// mutex round trip and a condvar wake per task, N tasks per call, ~415 calls per decode token.
std::mutex &g_pool_mu_spin() {
    static std::mutex m;
    return m;
}

class spin_pool {
  public:
    explicit spin_pool(int n) : n_(n) {
        for (int i = 1; i < n; ++i)
            workers_.emplace_back([this, i] {
                unsigned seen = 0;
                for (;;) {
                    unsigned g;
                    int spins = 0;
                    while ((g = gen_.load(std::memory_order_acquire)) == seen) {
                        if (++spins > 20000) std::this_thread::yield();
                    }
                    seen = g;
                    if (stop_.load(std::memory_order_relaxed)) return;
                    (*fn_)(i);
                    done_.fetch_add(1, std::memory_order_acq_rel);
                }
            });
    }
    ~spin_pool() {
        stop_.store(true);
        gen_.fetch_add(1, std::memory_order_release);
        for (auto &w : workers_) w.join();
    }
    void run(const std::function<void(int)> &fn) {
        fn_ = &fn;
        done_.store(0, std::memory_order_relaxed);
        gen_.fetch_add(1, std::memory_order_release);
        fn(0);
        while (done_.load(std::memory_order_acquire) != n_ - 1) {
        }
    }
    int size() const { return n_; }

  private:
    int n_;
    std::vector<std::thread> workers_;
    const std::function<void(int)> *fn_ = nullptr;
    std::atomic<unsigned> gen_{0};
    std::atomic<int> done_{0};
    std::atomic<bool> stop_{false};
};

int g_threads = 4;  // src/macro.h:21 N_THREADS_MUL_MAT_CPU
int g_pool_kind = 0;  // 0 = reference task pool, 1 = spin fork-join pool (bench "fixed" leg)
std::unique_ptr<spin_pool> g_spin;

spin_pool &spool() {
    std::lock_guard<std::mutex> lk(g_pool_mu_spin());
    if (!g_spin || g_spin->size() != g_threads) {
        g_spin.reset();
        g_spin = std::make_unique<spin_pool>(g_threads);
    }
    return *g_spin;
}

// mul_mat profile (orc_prof): [0] calls, [1] wall ns, [2] sum over calls of the slowest share's
// compute ns, [3]-[5] the same three for the F16 (attention) calls alone.
std::atomic<int64_t> g_prof[6];
bool g_prof_on = false;

inline int64_t now_ns() {
    return std::chrono::duration_cast<std::chrono::nanoseconds>(
               std::chrono::steady_clock::now().time_since_epoch()).count();
}
std::unique_ptr<task_pool> g_pool;
std::mutex g_pool_mu;

task_pool &pool() {
    std::lock_guard<std::mutex> lk(g_pool_mu);
    if (!g_pool || g_pool->size() != g_threads) {
        g_pool.reset();
        g_pool = std::make_unique<task_pool>(g_threads);
    }
    return *g_pool;
}

typedef void (*vec_dot_fn)(int, float *, const void *, const void *);

void f16_dot_ordered(int n, float *s, const void *x, const void *y) {
    orc_vec_dot_f16(n, s, (const uint16_t *)x, (const uint16_t *)y);
}
void f16_dot_avx2(int n, float *s, const void *x, const void *y) {
    orc_vec_dot_f16_avx2(n, s, (const uint16_t *)x, (const uint16_t *)y);
}

vec_dot_fn pick_vec_dot(int type, int avx2) {
    switch (type) {
        case ORC_Q4_0: return avx2 ? orc_vec_dot_q4_0_q8_0_avx2 : orc_vec_dot_q4_0_q8_0;
        case ORC_Q8_0: return avx2 ? orc_vec_dot_q8_0_q8_0_avx2 : orc_vec_dot_q8_0_q8_0;
        case ORC_F16: return avx2 ? f16_dot_avx2 : f16_dot_ordered;
        case ORC_Q4_K: return avx2 ? orc_vec_dot_q4_K_q8_K_avx2 : orc_vec_dot_q4_K_q8_K;
        case ORC_Q6_K: return avx2 ? orc_vec_dot_q6_K_q8_K_avx2 : orc_vec_dot_q6_K_q8_K;
    }
    return nullptr;
}

// src/hpc.cpp:15-41 (block = MUL_MAT_BLOCK_SIZE = 1, src/macro.h:23)
void mul_mat_sub(int64_t start_row, int64_t end_row, int64_t shared_edge, int64_t col_num, int64_t ne01,
                 int64_t ne1, int64_t nb01, int64_t nb1, int64_t nb2, int64_t row_size, const char *src0,
                 const char *src1, char *dst, vec_dot_fn vec_dot) {
    for (int64_t r = start_row; r < end_row && r < ne01; ++r) {
        for (int64_t c = 0; c < col_num; ++c) {
            const int64_t mat_i = c / ne1, mat_col_i = c % ne1;
            float *dst_col = (float *)(dst + mat_col_i * nb1 + mat_i * nb2);
            vec_dot((int)shared_edge, &dst_col[r], src0 + r * nb01, src1 + c * row_size);
        }
    }
}

}  // namespace

extern "C" void orc_set_threads(int n) { g_threads = n > 0 ? n : 1; }

extern "C" void orc_mul_mat(int64_t ne01, int64_t ne11, int64_t ne12, int64_t nb01, int64_t ne1, int64_t nb1,
                            int64_t nb2, size_t row_size, int64_t shared_edge, const void *src0, void *dst,
                            int src0_type, const char *wdata, int use_avx2) {
    vec_dot_fn vd = pick_vec_dot(src0_type, use_avx2);
    if (!vd) return;
    const int64_t col_num = ne11 * ne12;
    const int N = g_threads;
    const int64_t cpu_row_num = (int64_t)ceil(((double)ne01 * 1.0) / (double)N) * N;
    const int64_t row_per_core = cpu_row_num / N;
    const int64_t t0 = g_prof_on ? now_ns() : 0;
    std::atomic<int64_t> slowest{0};
    auto share = [&, row_per_core](int t) {
        const int64_t a = g_prof_on ? now_ns() : 0;
        const int64_t s = t * row_per_core, e = (t + 1) * row_per_core;
        mul_mat_sub(s, e, shared_edge, col_num, ne01, ne1, nb01, nb1, nb2, (int64_t)row_size,
                    (const char *)src0, wdata, (char *)dst, vd);
        if (g_prof_on) {
            const int64_t d = now_ns() - a;
            int64_t cur = slowest.load();
            while (d > cur && !slowest.compare_exchange_weak(cur, d)) {
            }
        }
    };
    if (N == 1) {
        share(0);
    } else if (g_pool_kind == 1) {
        spool().run(share);
    } else {
        task_pool &p = pool();
        std::vector<std::future<void>> futs;
        for (int t = 0; t < N; ++t) futs.push_back(p.submit([&share, t] { share(t); }));
        for (auto &f : futs) f.get();
    }
    if (g_prof_on) {
        const int64_t w = now_ns() - t0, k = src0_type == ORC_F16 ? 3 : 0;
        g_prof[k] += 1;
        g_prof[k + 1] += w;
        g_prof[k + 2] += slowest.load();
    }
}

// bench.py cpu_baseline diagnostics: pool kind (0 reference task pool, 1 spin fork-join) and the
// mul_mat profile (see g_prof); out[6] = {calls, wall_s, slowest-share_s, f16 calls, f16 wall_s,
// f16 slowest-share_s}.
extern "C" void orc_set_pool(int kind) { g_pool_kind = kind == 1 ? 1 : 0; }
extern "C" void orc_prof(int enable, double *out) {
    if (out) {
        for (int i = 0; i < 6; ++i) out[i] = (i % 3 == 0) ? (double)g_prof[i].load() : g_prof[i].load() * 1e-9;
    }
    for (auto &c : g_prof) c = 0;
    g_prof_on = enable != 0;
}

// ggml MUL_MAT INIT [ext]: every src1 row (ne10 f32) -> vec_dot_type row.
extern "C" void orc_mul_mat_init(int src0_type, const float *src1, int64_t k, int64_t n_cols,
                                 int64_t col_stride_f, void *wdata) {
    char *w = (char *)wdata;
    if (src0_type == ORC_F16) {
        for (int64_t c = 0; c < n_cols; ++c) {
            uint16_t *o = (uint16_t *)(w + c * k * 2);
            for (int64_t i = 0; i < k; ++i) o[i] = orc_fp32_to_fp16(src1[c * col_stride_f + i]);
        }
    } else if (src0_type == ORC_Q4_K || src0_type == ORC_Q6_K) {  // vec_dot_type Q8_K
        const size_t rs = orc_row_size(ORC_Q8_K, k);
        for (int64_t c = 0; c < n_cols; ++c) orc_quantize_row_q8_K(src1 + c * col_stride_f, w + c * rs, (int)k);
    } else {
        const size_t rs = orc_row_size(ORC_Q8_0, k);
        for (int64_t c = 0; c < n_cols; ++c) orc_quantize_row_q8_0(src1 + c * col_stride_f, w + c * rs, (int)k);
    }
}
