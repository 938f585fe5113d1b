// Back-to-back issue rate of the f16 MFMA shapes on gfx950 (and v_fma_mix_f32 / v_pk_fma_f32 for
// comparison): cycles per instruction on one SIMD, 4 independent accumulators per wave, 1 or 2
// waves per SIMD.  Used to price "MFMA as a batched fma" (one product per output per step) for the
// exact attention.  build: hipcc --offload-arch=gfx950 -O3 mfma_rates.hip -o mfma_rates
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>

typedef _Float16 h4 __attribute__((ext_vector_type(4)));
typedef _Float16 h8 __attribute__((ext_vector_type(8)));
typedef float f4 __attribute__((ext_vector_type(4)));
typedef float f16v __attribute__((ext_vector_type(16)));

template <int OP>
__global__ void k(float *out, unsigned long long *cyc, int iters) {
    const _Float16 x = (_Float16)(float)(threadIdx.x & 7);
    h4 a4 = {x, x, x, x};
    h8 a8 = {x, x, x, x, x, x, x, x};
    f4 c4[4] = {};
    f16v c16[4] = {};
    float s[8] = {};
    typedef float v2f __attribute__((ext_vector_type(2)));
    v2f p[8] = {};
    const unsigned long long t0 = __builtin_readcyclecounter();
    for (int it = 0; it < iters; ++it) {
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            if (OP == 0) c4[i] = __builtin_amdgcn_mfma_f32_16x16x16f16(a4, a4, c4[i], 0, 0, 0);
            if (OP == 1) c16[i] = __builtin_amdgcn_mfma_f32_32x32x8f16(a4, a4, c16[i], 0, 0, 0);
            if (OP == 2) c4[i] = __builtin_amdgcn_mfma_f32_4x4x4f16(a4, a4, c4[i], 0, 0, 0);
            if (OP == 3) c4[i] = __builtin_amdgcn_mfma_f32_16x16x32_f16(a8, a8, c4[i], 0, 0, 0);
            if (OP == 4) c16[i] = __builtin_amdgcn_mfma_f32_32x32x16_f16(a8, a8, c16[i], 0, 0, 0);
            if (OP == 5) {
                asm volatile("v_fma_mix_f32 %0, %1, %2, %0 op_sel_hi:[1,1,0]" : "+v"(s[2 * i]) : "v"(a4[0]), "v"(a4[1]));
                asm volatile("v_fma_mix_f32 %0, %1, %2, %0 op_sel_hi:[1,1,0]" : "+v"(s[2 * i + 1]) : "v"(a4[0]), "v"(a4[1]));
            }
            if (OP == 6) {
                asm volatile("v_pk_fma_f32 %0, %1, %2, %0" : "+v"(p[2 * i]) : "v"(p[7]), "v"(p[6]));
                asm volatile("v_pk_fma_f32 %0, %1, %2, %0" : "+v"(p[2 * i + 1]) : "v"(p[7]), "v"(p[6]));
            }
        }
    }
    const unsigned long long t1 = __builtin_readcyclecounter();
    float acc = 0.0f;
#pragma unroll
    for (int i = 0; i < 4; ++i) acc += c4[i][0] + c16[i][0] + s[2 * i] + s[2 * i + 1] + p[2 * i].x + p[2 * i + 1].y;
    out[blockIdx.x * blockDim.x + threadIdx.x] = acc;
    if (threadIdx.x == 0) cyc[blockIdx.x] = t1 - t0;
}

template <typename K>
void run(const char *name, K kern, int per_iter, int outputs_per_instr, int waves_per_simd) {
    float *o;
    unsigned long long *c;
    const int blocks = 256 * waves_per_simd;  // 256-thread blocks: 4 waves each, one block per CU per wave/SIMD
    hipMalloc(&o, blocks * 256 * 4);
    hipMalloc(&c, blocks * 8);
    const int iters = 4000;
    hipLaunchKernelGGL(kern, dim3(blocks), dim3(256), 0, 0, o, c, iters);
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    hipEventRecord(e0);
    hipLaunchKernelGGL(kern, dim3(blocks), dim3(256), 0, 0, o, c, iters);
    hipEventRecord(e1);
    hipEventSynchronize(e1);
    float ms;
    hipEventElapsedTime(&ms, e0, e1);
    unsigned long long h;
    hipMemcpy(&h, c, 8, hipMemcpyDeviceToHost);
    const double instr = (double)iters * per_iter;
    const double ns = ms * 1e6 / (instr * waves_per_simd);  // per SIMD-instruction
    printf("%-22s waves/SIMD %d: %6.2f cyc/instr (own clock), %.3f ns per SIMD-instr, %.1f fma-outputs/ns/SIMD\n", name,
           waves_per_simd, (double)h / instr, ns, outputs_per_instr / ns);
    hipFree(o);
    hipFree(c);
}

int main() {
    for (int w : {1, 2}) {
        run("mfma 16x16x16 f16", k<0>, 4, 256, w);
        run("mfma 32x32x8 f16", k<1>, 4, 1024, w);
        run("mfma 4x4x4(16b) f16", k<2>, 4, 256, w);
        run("mfma 16x16x32 f16", k<3>, 4, 256, w);
        run("mfma 32x32x16 f16", k<4>, 4, 1024, w);
        run("v_fma_mix_f32", k<5>, 8, 64, w);
        run("v_pk_fma_f32", k<6>, 8, 128, w);
    }
    return 0;
}
