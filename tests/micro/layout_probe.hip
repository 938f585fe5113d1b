// Does the tiled-weight order matter for a matvec-shaped stream?  2048 waves each read N_IT items of
// 1 KiB (U in flight).  "rt-major": wave w's items are contiguous (tile = w*N_IT + k, the current
// [row tile][block tile] layout); "bt-major": tile = k*N_W + w (all waves at step k read one
// contiguous 2 MiB span).  Cold: rotating over >1 GiB.
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdint.h>
#include <vector>
typedef uint32_t u4v __attribute__((ext_vector_type(4)));

template <int U, bool BT_MAJOR>
__global__ void __launch_bounds__(256) k_probe(const u4v *__restrict__ p, int n_it, int n_w, uint32_t *out) {
    const int lane = threadIdx.x & 63, w = blockIdx.x * 4 + (threadIdx.x >> 6);
    uint32_t acc = 0;
    for (int k0 = 0; k0 < n_it; k0 += U) {
        u4v v[U];
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const int k = k0 + u;
            const int64_t tile = BT_MAJOR ? (int64_t)k * n_w + w : (int64_t)w * n_it + k;
            v[u] = __builtin_nontemporal_load(p + tile * 64 + lane);
        }
#pragma unroll
        for (int u = 0; u < U; ++u) acc ^= v[u].x ^ v[u].y ^ v[u].z ^ v[u].w;
    }
    if (acc == 0x12345678u) out[0] = acc;
}

int main() {
    uint32_t *out;
    (void)hipMalloc(&out, 4);
    hipEvent_t a, b;
    (void)hipEventCreate(&a);
    (void)hipEventCreate(&b);
    const int n_w = 2048;
    for (int n_it : {8, 16, 32}) {
        const size_t S = (size_t)n_w * n_it * 1024;
        const int nb = (int)((2048ull << 20) / S) + 1;
        std::vector<u4v *> bufs(nb);
        for (auto &q : bufs) { (void)hipMalloc(&q, S); (void)hipMemset(q, 1, S); }
        for (int bt : {0, 1}) {
            auto launch = [&](int i) {
                if (bt) hipLaunchKernelGGL((k_probe<8, true>), dim3(n_w / 4), dim3(256), 0, 0, bufs[i % nb], n_it, n_w, out);
                else hipLaunchKernelGGL((k_probe<8, false>), dim3(n_w / 4), dim3(256), 0, 0, bufs[i % nb], n_it, n_w, out);
            };
            for (int i = 0; i < nb; ++i) launch(i);
            const int iters = 4 * nb;
            (void)hipEventRecord(a, 0);
            for (int i = 0; i < iters; ++i) launch(i);
            (void)hipEventRecord(b, 0);
            (void)hipEventSynchronize(b);
            float ms = 0;
            (void)hipEventElapsedTime(&ms, a, b);
            const double us = ms * 1000.0 / iters;
            printf("MB %.1f items/wave %d %s: %.2f us %.0f GB/s\n", S / 1048576.0, n_it, bt ? "bt-major" : "rt-major", us,
                   S / (us * 1e-6) / 1e9);
        }
        for (auto q : bufs) (void)hipFree(q);
    }
    return 0;
}
