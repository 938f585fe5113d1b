// Compute-only ceiling of the exact GEMM's inner block (k_gemm_x): 16 MFMA 16x16x32 f16 with
// register operands, then 16 mul + 64 fmaf into 64 lane-chain accumulators.  Cycles per block per
// wave at 1..3 waves per SIMD; VARIANT 1 = the fmafs of block i interleaved with block i+1's MFMAs.
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdint.h>
typedef _Float16 h8 __attribute__((ext_vector_type(8)));
typedef float f4 __attribute__((ext_vector_type(4)));

template <int VAR>
__global__ void __launch_bounds__(256) k(float *out, unsigned long long *cyc, int iters, float s) {
    h8 a[8], b[2];
#pragma unroll
    for (int i = 0; i < 8; ++i) a[i] = (h8)(_Float16)(threadIdx.x & 3) + (_Float16)i;
    b[0] = (h8)(_Float16)1; b[1] = (h8)(_Float16)2;
    float dw[8], da[2];
#pragma unroll
    for (int i = 0; i < 8; ++i) dw[i] = s * (i + 1);
    da[0] = s; da[1] = 2 * s;
    float acc[8][2][4] = {};
    f4 dd[8][2];
    const f4 z = {0, 0, 0, 0};
    unsigned long long t0 = __builtin_readcyclecounter();
    if (VAR == 1) {
#pragma unroll
        for (int rt = 0; rt < 8; ++rt)
#pragma unroll
            for (int ct = 0; ct < 2; ++ct) dd[rt][ct] = __builtin_amdgcn_mfma_f32_16x16x32_f16(a[rt], b[ct], z, 0, 0, 0);
    }
    for (int it = 0; it < iters; ++it) {
        if (VAR == 0) {
#pragma unroll
            for (int rt = 0; rt < 8; ++rt)
#pragma unroll
                for (int ct = 0; ct < 2; ++ct) dd[rt][ct] = __builtin_amdgcn_mfma_f32_16x16x32_f16(a[rt], b[ct], z, 0, 0, 0);
#pragma unroll
            for (int rt = 0; rt < 8; ++rt)
#pragma unroll
                for (int ct = 0; ct < 2; ++ct) {
                    const float d = dw[rt] * da[ct];
#pragma unroll
                    for (int v = 0; v < 4; ++v) acc[rt][ct][v] = __builtin_fmaf(d, dd[rt][ct][v], acc[rt][ct][v]);
                }
        } else {
            // consume the previous block's results while this block's MFMAs run
#pragma unroll
            for (int rt = 0; rt < 8; ++rt)
#pragma unroll
                for (int ct = 0; ct < 2; ++ct) {
                    const f4 prev = dd[rt][ct];
                    dd[rt][ct] = __builtin_amdgcn_mfma_f32_16x16x32_f16(a[rt], b[ct], z, 0, 0, 0);
                    const float d = dw[rt] * da[ct];
#pragma unroll
                    for (int v = 0; v < 4; ++v) acc[rt][ct][v] = __builtin_fmaf(d, prev[v], acc[rt][ct][v]);
                }
        }
        a[0][0] += (_Float16)1;  // keep the loop from being hoisted
    }
    unsigned long long t1 = __builtin_readcyclecounter();
    float r = 0;
#pragma unroll
    for (int rt = 0; rt < 8; ++rt)
#pragma unroll
        for (int ct = 0; ct < 2; ++ct)
#pragma unroll
            for (int v = 0; v < 4; ++v) r += acc[rt][ct][v] + dd[rt][ct][v];
    out[blockIdx.x * 256 + threadIdx.x] = r;
    if (threadIdx.x == 0) cyc[blockIdx.x] = t1 - t0;
}

template <typename K>
void run(const char *name, K kern, int wps) {
    float *o; unsigned long long *c;
    const int blocks = 256 * wps;
    (void)hipMalloc(&o, blocks * 256 * 4); (void)hipMalloc(&c, blocks * 8);
    const int iters = 4000;
    hipLaunchKernelGGL(kern, dim3(blocks), dim3(256), 0, 0, o, c, iters, 1e-3f);
    hipEvent_t e0, e1; (void)hipEventCreate(&e0); (void)hipEventCreate(&e1);
    (void)hipEventRecord(e0);
    hipLaunchKernelGGL(kern, dim3(blocks), dim3(256), 0, 0, o, c, iters, 1e-3f);
    (void)hipEventRecord(e1); (void)hipEventSynchronize(e1);
    float ms; (void)hipEventElapsedTime(&ms, e0, e1);
    unsigned long long h; (void)hipMemcpy(&h, c, 8, hipMemcpyDeviceToHost);
    printf("%-12s waves/SIMD %d: %.1f cyc per block (wave clock); chip %.3f ms -> %.1f ns per block per SIMD, %.2f ns per MFMA\n",
           name, wps, (double)h / iters, ms, ms * 1e6 / (iters * wps), ms * 1e6 / (iters * wps * 16));
    (void)hipFree(o); (void)hipFree(c);
}

int main() {
    for (int w : {1, 2, 3}) {
        run("mfma_then_fma", k<0>, w);
        run("pipelined", k<1>, w);
    }
    return 0;
}
