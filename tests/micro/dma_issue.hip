// Microbenchmark: issue cost of LDS-DMA (global_load_lds_dwordx4) per wave instruction, as the
// persistent token kernel (csrc/token.hip) issues its ring refills.  One workgroup per CU, W waves,
// each issues N tile refills (1 KiB + optional 128 B scale DMA) into a private LDS ring; stamps
// around the issue loop and around the drain.  hipcc --offload-arch=gfx950 -O3 dma_issue.hip
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdint.h>
#include <vector>
#include <algorithm>

__device__ __forceinline__ void dma16(const void *g, uint32_t lds_addr) {
    const uint32_t lds = __builtin_amdgcn_readfirstlane(lds_addr);
    unsigned keep;
    asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, off nt\n\ts_mov_b32 m0, %0"
                 : "=&s"(keep) : "v"(g), "s"(lds) : "memory");
}

template <int MODE>
__global__ void __launch_bounds__(512) k(const uint8_t *w, size_t per_cu, unsigned long long *out, int n) {
    extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
    const int lane = threadIdx.x & 63, wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const uint8_t *base = w + (size_t)blockIdx.x * per_cu + (size_t)wave * n * 1152;
    const uint32_t ring = (uint32_t)(uintptr_t)smem + wave * 8 * 1152;
    unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
    for (int i = 0; i < n; ++i) {
        const uint32_t dst = ring + (i & 7) * 1152;
        dma16(base + (size_t)i * 1152 + lane * 16, dst);
        if (MODE & 1) { if (lane < 8) dma16(base + (size_t)i * 1152 + 1024 + lane * 16, dst + 1024); }
        if (MODE & 2) asm volatile("s_waitcnt vmcnt(14)" ::: "memory");  // keep 7 tiles in flight
    }
    unsigned long long t1 = __builtin_amdgcn_s_memrealtime();
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    unsigned long long t2 = __builtin_amdgcn_s_memrealtime();
    if (lane == 0) {
        out[(blockIdx.x * 8 + wave) * 2 + 0] = t1 - t0;
        out[(blockIdx.x * 8 + wave) * 2 + 1] = t2 - t0;
    }
}

int main() {
    const int ncu = 256, n = 64;
    const size_t per_cu = (size_t)8 * n * 1152;
    uint8_t *w; unsigned long long *o;
    hipMalloc(&w, per_cu * ncu + 4096);
    hipMemset(w, 1, per_cu * ncu);
    hipMalloc(&o, ncu * 8 * 2 * 8);
    std::vector<unsigned long long> h(ncu * 8 * 2);
    auto run = [&](auto kern, const char *name, int waves) {
        hipFuncSetAttribute((const void *)kern, hipFuncAttributeMaxDynamicSharedMemorySize, 8 * 8 * 1152);
        for (int rep = 0; rep < 3; ++rep) {
            hipLaunchKernelGGL(kern, dim3(ncu), dim3(64 * waves), 8 * 8 * 1152, 0, w, per_cu, o, n);
            hipDeviceSynchronize();
        }
        hipMemcpy(h.data(), o, h.size() * 8, hipMemcpyDeviceToHost);
        std::vector<double> is, dr;
        for (int i = 0; i < ncu * waves; ++i) {
            const int b = i / waves, wv = i % waves;
            is.push_back(h[(b * 8 + wv) * 2] / 100.0);
            dr.push_back(h[(b * 8 + wv) * 2 + 1] / 100.0);
        }
        std::sort(is.begin(), is.end()); std::sort(dr.begin(), dr.end());
        const double bytes = (double)waves * n * ((name[0] == 's') ? 1152 : 1024);
        printf("%-28s waves %d: issue loop median %.2f us (%.3f us per tile), to drain median %.2f us (%.1f GB/s per CU)\n",
               name, waves, is[is.size() / 2], is[is.size() / 2] / n, dr[dr.size() / 2], bytes / (dr[dr.size() / 2] * 1e3));
    };
    for (int waves : {1, 4, 8}) {
        run(k<0>, "quants only", waves);
        run(k<1>, "scales too", waves);
        run(k<3>, "scales + vmcnt(14)", waves);
    }
    return 0;
}
