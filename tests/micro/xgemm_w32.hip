// Compute-only ceiling of the exact GEMM's W32 block step (k_gemm_x, W32, 16-row x 32-token wave):
// 4 x v_mfma_f32_32x32x16_f16 from register operands, then 8 d products and 64 lane-chain fmafs.
// Cycles per block per wave (s_memtime) and ns per block per SIMD at 1, 2, 3 waves per SIMD.
// Build twice (default, -fno-slp-vectorize) to compare packed / scalar f32 VALU beside the MFMAs.
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdint.h>
typedef _Float16 h8 __attribute__((ext_vector_type(8)));
typedef float f16v __attribute__((ext_vector_type(16)));

__global__ void __launch_bounds__(256) k(float *out, unsigned long long *cyc, int iters, float s) {
    h8 a[2][2], b[2];
#pragma unroll
    for (int q = 0; q < 2; ++q)
#pragma unroll
        for (int h = 0; h < 2; ++h) a[q][h] = (h8)(_Float16)(threadIdx.x & 3) + (_Float16)(q + h);
    b[0] = (h8)(_Float16)1; b[1] = (h8)(_Float16)2;
    float dw[2][4], da = s;
#pragma unroll
    for (int q = 0; q < 2; ++q)
#pragma unroll
        for (int j = 0; j < 4; ++j) dw[q][j] = s * (q * 4 + j + 1);
    float acc[2][4][8] = {};
    const f16v z = {};
    unsigned long long t0 = __builtin_readcyclecounter();
    for (int it = 0; it < iters; ++it) {
        f16v d[2][2];
#pragma unroll
        for (int q = 0; q < 2; ++q)
#pragma unroll
            for (int h = 0; h < 2; ++h) d[q][h] = __builtin_amdgcn_mfma_f32_32x32x16_f16(a[q][h], b[h], z, 0, 0, 0);
#pragma unroll
        for (int q = 0; q < 2; ++q)
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                const float dd = dw[q][j] * da;
#pragma unroll
                for (int i = 0; i < 4; ++i) {
                    acc[q][j][i] = __builtin_fmaf(dd, d[q][0][4 * j + i], acc[q][j][i]);
                    acc[q][j][4 + i] = __builtin_fmaf(dd, d[q][1][4 * j + i], acc[q][j][4 + i]);
                }
            }
        da = da * 1.0000001f;  // keeps the products loop-variant
    }
    unsigned long long t1 = __builtin_readcyclecounter();
    float v = 0;
#pragma unroll
    for (int q = 0; q < 2; ++q)
#pragma unroll
        for (int j = 0; j < 4; ++j)
#pragma unroll
            for (int i = 0; i < 8; ++i) v += acc[q][j][i];
    out[blockIdx.x * blockDim.x + threadIdx.x] = v;
    if (threadIdx.x == 0) cyc[blockIdx.x] = t1 - t0;
}

int main() {
    float *o; unsigned long long *c;
    hipMalloc(&o, 4096 * 256 * 4); hipMalloc(&c, 4096 * 8);
    const int iters = 4000;
    for (int w : {1, 2, 3}) {
        const int blocks = 256 * w;  // 4 waves per block: w waves per SIMD on every CU
        hipLaunchKernelGGL(k, dim3(blocks), dim3(256), 0, 0, o, c, iters, 1.0f);
        hipEvent_t e0, e1; hipEventCreate(&e0); hipEventCreate(&e1);
        hipEventRecord(e0);
        hipLaunchKernelGGL(k, dim3(blocks), dim3(256), 0, 0, o, c, iters, 1.0f);
        hipEventRecord(e1); hipEventSynchronize(e1);
        float ms; hipEventElapsedTime(&ms, e0, e1);
        unsigned long long h; hipMemcpy(&h, c, 8, hipMemcpyDeviceToHost);
        printf("waves/SIMD %d: %.1f cyc per block per wave (own clock), %.2f ns per block per SIMD (wall)\n", w,
               (double)h / iters, ms * 1e6 / ((double)iters * w));
    }
    return 0;
}
