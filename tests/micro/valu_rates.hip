// Throughput of the exact-prefill GEMM's VALU ops on gfx950: cycles per wave-instruction with
// `waves` waves per SIMD, 16 independent chains per wave (s_memtime around the loop).
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdint.h>

#define REP16(X) X(0) X(1) X(2) X(3) X(4) X(5) X(6) X(7) X(8) X(9) X(10) X(11) X(12) X(13) X(14) X(15)

template <int OP>
__global__ void k(uint32_t *out, unsigned long long *cyc, int iters, uint32_t seed) {
    uint32_t r[16];
#pragma unroll
    for (int i = 0; i < 16; ++i) r[i] = seed * (threadIdx.x + i + 1);
    const uint32_t a = seed ^ threadIdx.x, b = seed + 7;
    unsigned long long t0 = __builtin_readcyclecounter();
    for (int it = 0; it < iters; ++it) {
#define OPX(i)                                                                                         \
    if (OP == 0) asm volatile("v_dot4_i32_i8 %0, %1, %2, %0" : "+v"(r[i]) : "v"(a), "v"(b));           \
    if (OP == 1) asm volatile("v_cvt_f32_i32 %0, %0" : "+v"(r[i]));                                   \
    if (OP == 2) asm volatile("v_fma_f32 %0, %1, %2, %0" : "+v"(r[i]) : "v"(a), "v"(b));             \
    if (OP == 3) asm volatile("v_mul_f32 %0, %1, %0" : "+v"(r[i]) : "v"(a));                          \
    if (OP == 4) asm volatile("v_dot4c_i32_i8 %0, %1, %2" : "+v"(r[i]) : "v"(a), "v"(b));             \
    if (OP == 5) asm volatile("v_add_f32 %0, %1, %0" : "+v"(r[i]) : "v"(a));                          \
    if (OP == 6) asm volatile("v_sub_u32 %0, %1, %0" : "+v"(r[i]) : "v"(a));                          \
    if (OP == 7) asm volatile("v_fma_mix_f32 %0, %1, %2, %0 op_sel_hi:[1,1,0]" : "+v"(r[i]) : "v"(a), "v"(b)); \
    if (OP == 8) asm volatile("v_cvt_f32_f16 %0, %1" : "=v"(r[i]) : "v"(r[i]));                       \
    if (OP == 9) asm volatile("v_dot2_f32_f16 %0, %1, %2, %0" : "+v"(r[i]) : "v"(a), "v"(b));
        REP16(OPX)
    }
    unsigned long long t1 = __builtin_readcyclecounter();
    uint32_t acc = 0;
#pragma unroll
    for (int i = 0; i < 16; ++i) acc ^= r[i];
    out[blockIdx.x * blockDim.x + threadIdx.x] = acc;
    if (threadIdx.x == 0) cyc[blockIdx.x] = t1 - t0;
}

template <int OP>
__global__ void kpk(uint32_t *out, unsigned long long *cyc, int iters, uint32_t seed) {
    typedef float v2f __attribute__((ext_vector_type(2)));
    v2f r[8];
#pragma unroll
    for (int i = 0; i < 8; ++i) r[i] = v2f{(float)(seed + i), (float)threadIdx.x};
    v2f a = {1.0001f, 0.9999f}, b = {0.5f, 0.25f};
    unsigned long long t0 = __builtin_readcyclecounter();
    for (int it = 0; it < iters; ++it) {
#pragma unroll
        for (int i = 0; i < 8; ++i) {
            if (OP == 0) asm volatile("v_pk_fma_f32 %0, %1, %2, %0" : "+v"(r[i]) : "v"(a), "v"(b));
            if (OP == 1) asm volatile("v_pk_mul_f32 %0, %1, %0" : "+v"(r[i]) : "v"(a));
            if (OP == 2) asm volatile("v_pk_add_f32 %0, %1, %0" : "+v"(r[i]) : "v"(a));
        }
    }
    unsigned long long t1 = __builtin_readcyclecounter();
    float acc = 0;
#pragma unroll
    for (int i = 0; i < 8; ++i) acc += r[i].x + r[i].y;
    out[blockIdx.x * blockDim.x + threadIdx.x] = __builtin_bit_cast(uint32_t, acc);
    if (threadIdx.x == 0) cyc[blockIdx.x] = t1 - t0;
}

template <typename K>
void run(const char *name, K kern, int ninstr_per_iter, int waves_per_simd) {
    uint32_t *o; unsigned long long *c;
    const int blocks = 256 * 4 * waves_per_simd / 4;  // 256-thread blocks: 4 waves each
    hipMalloc(&o, blocks * 256 * 4); hipMalloc(&c, blocks * 8);
    const int iters = 2000;
    hipLaunchKernelGGL(kern, dim3(blocks), dim3(256), 0, 0, o, c, iters, 3u);
    hipEvent_t e0, e1; hipEventCreate(&e0); hipEventCreate(&e1);
    hipEventRecord(e0);
    hipLaunchKernelGGL(kern, dim3(blocks), dim3(256), 0, 0, o, c, iters, 5u);
    hipEventRecord(e1); hipEventSynchronize(e1);
    float ms; hipEventElapsedTime(&ms, e0, e1);
    unsigned long long h; hipMemcpy(&h, c, 8, hipMemcpyDeviceToHost);
    const double instr = (double)iters * ninstr_per_iter;
    // per SIMD: waves_per_simd waves each issue `instr` wave-instructions
    printf("%-16s waves/SIMD %d: %.2f cyc/instr (wave's own clock), chip %.3f ms -> %.2f ns per SIMD-instr\n", name,
           waves_per_simd, (double)h / instr, ms, ms * 1e6 / (instr * waves_per_simd));
    hipFree(o); hipFree(c);
}

int main() {
    for (int w : {1, 2, 4}) {
        run("dot4_i32_i8", k<0>, 16, w);
        run("dot4c_i32_i8", k<4>, 16, w);
        run("cvt_f32_i32", k<1>, 16, w);
        run("fma_f32", k<2>, 16, w);
        run("mul_f32", k<3>, 16, w);
        run("add_f32", k<5>, 16, w);
        run("sub_u32", k<6>, 16, w);
        run("fma_mix_f32", k<7>, 16, w);
        run("cvt_f32_f16", k<8>, 16, w);
        run("dot2_f32_f16", k<9>, 16, w);
        run("pk_fma_f32", kpk<0>, 8, w);
        run("pk_mul_f32", kpk<1>, 8, w);
        run("pk_add_f32", kpk<2>, 8, w);
    }
    return 0;
}
