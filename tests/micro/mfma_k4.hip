// The K = 4 multi-block f16 MFMAs on gfx950 (VERDICT r5 "Next round" #3): register layout of
// v_mfma_f32_32x32x4_2b_f16 and v_mfma_f32_16x16x4_4b_f16, exactness of their 4-term integer sums
// (Q4_0 nibble - 8 times Q8_0 int8: the AVX2 lane sum isum_l of ggml's vec_dot_q4_0_q8_0), and their
// issue rate against v_mfma_f32_32x32x16_f16 (the exact prefill GEMM's current instruction, 3/4 of
// whose products are masked zeros).  One block of a K = 4 form = one AVX2 lane l: A = the 4 weights
// 4l..4l+3 of 32 (16) rows, B = the same 4 activations of 32 (16) tokens, every product useful.
// build: hipcc --offload-arch=gfx950 -O3 mfma_k4.hip -o mfma_k4
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>

typedef _Float16 h4 __attribute__((ext_vector_type(4)));
typedef _Float16 h8 __attribute__((ext_vector_type(8)));
typedef float f4 __attribute__((ext_vector_type(4)));
typedef float f16v __attribute__((ext_vector_type(16)));
typedef float f32v __attribute__((ext_vector_type(32)));

// ---- layout: A / B operands given per lane, D written out per (lane, reg)
__global__ void k_layout32(const float *A, const float *B, float *D) {
    const int L = threadIdx.x;
    h4 a, b;
    for (int k = 0; k < 4; ++k) a[k] = (_Float16)A[L * 4 + k], b[k] = (_Float16)B[L * 4 + k];
    f32v d = {};
    d = __builtin_amdgcn_mfma_f32_32x32x4f16(a, b, d, 0, 0, 0);
    for (int r = 0; r < 32; ++r) D[L * 32 + r] = d[r];
}
__global__ void k_layout16(const float *A, const float *B, float *D) {
    const int L = threadIdx.x;
    h4 a, b;
    for (int k = 0; k < 4; ++k) a[k] = (_Float16)A[L * 4 + k], b[k] = (_Float16)B[L * 4 + k];
    f16v d = {};
    d = __builtin_amdgcn_mfma_f32_16x16x4f16(a, b, d, 0, 0, 0);
    for (int r = 0; r < 16; ++r) D[L * 16 + r] = d[r];
}

// ---- rate: NACC independent accumulators per wave, back to back
template <int OP, int NACC>
__global__ void k_rate(float *out, int iters) {
    const _Float16 x = (_Float16)(float)(threadIdx.x & 7);
    h4 a4 = {x, x, x, x};
    h8 a8 = {x, x, x, x, x, x, x, x};
    f32v c32[NACC] = {};
    f16v c16[NACC] = {};
    for (int it = 0; it < iters; ++it) {
#pragma unroll
        for (int i = 0; i < NACC; ++i) {
            if (OP == 0) c32[i] = __builtin_amdgcn_mfma_f32_32x32x4f16(a4, a4, c32[i], 0, 0, 0);
            if (OP == 1) c16[i] = __builtin_amdgcn_mfma_f32_16x16x4f16(a4, a4, c16[i], 0, 0, 0);
            if (OP == 2) c16[i] = __builtin_amdgcn_mfma_f32_32x32x16_f16(a8, a8, c16[i], 0, 0, 0);
        }
    }
    float acc = 0.0f;
#pragma unroll
    for (int i = 0; i < NACC; ++i) acc += c32[i][0] + c16[i][0];
    out[blockIdx.x * blockDim.x + threadIdx.x] = acc;
}

template <typename K>
double rate(K kern, int per_iter, int waves_per_simd) {
    float *o;
    const int blocks = 256 * waves_per_simd;
    hipMalloc(&o, (size_t)blocks * 256 * 4);
    const int iters = 2000;
    hipLaunchKernelGGL(kern, dim3(blocks), dim3(256), 0, 0, o, iters);
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    hipEventRecord(e0);
    hipLaunchKernelGGL(kern, dim3(blocks), dim3(256), 0, 0, o, iters);
    hipEventRecord(e1);
    hipEventSynchronize(e1);
    float ms;
    hipEventElapsedTime(&ms, e0, e1);
    hipFree(o);
    return ms * 1e6 / ((double)iters * per_iter * waves_per_simd);  // ns per SIMD-instruction
}

static uint32_t rng = 12345;
static int rnd(int lo, int hi) {
    rng = rng * 1664525u + 1013904223u;
    return lo + (int)((rng >> 8) % (uint32_t)(hi - lo + 1));
}

int main() {
    float *A, *B, *D;
    hipMallocManaged(&A, 64 * 4 * 4);
    hipMallocManaged(&B, 64 * 4 * 4);
    hipMallocManaged(&D, 64 * 32 * 4);
    // 32x32x4_2b: A lane L holds 4 K values of one (block, row); B one (block, col).  Probe: A = row id
    // in k = 0 only, B = 1 in k = 0 -> D = the row (+ 64 * block) of A that lane L / reg r sees
    for (int pass = 0; pass < 3; ++pass) {
        for (int L = 0; L < 64; ++L)
            for (int k = 0; k < 4; ++k) {
                A[L * 4 + k] = pass == 0 ? (k == 0 ? (float)(L + 1) : 0.f) : pass == 1 ? (k == 0 ? 1.f : 0.f) : (float)(k + 1);
                B[L * 4 + k] = pass == 0 ? (k == 0 ? 1.f : 0.f) : pass == 1 ? (k == 0 ? (float)(L + 1) : 0.f) : (k == 2 ? 1.f : 0.f);
            }
        hipLaunchKernelGGL(k_layout32, dim3(1), dim3(64), 0, 0, A, B, D);
        hipDeviceSynchronize();
        printf("32x32x4_2b pass %d (%s): lane 0..2, 31..33, 63 x regs 0..31\n", pass,
               pass == 0 ? "A lane+1 that feeds (lane, reg)" : pass == 1 ? "B lane+1" : "K pairing: A=k+1, B=[k==2] -> 3");
        for (int L : {0, 1, 2, 31, 32, 33, 63}) {
            printf("  L%2d:", L);
            for (int r = 0; r < 32; ++r) printf(" %3.0f", D[L * 32 + r]);
            printf("\n");
        }
    }
    for (int pass = 0; pass < 2; ++pass) {
        for (int L = 0; L < 64; ++L)
            for (int k = 0; k < 4; ++k) {
                A[L * 4 + k] = pass == 0 ? (k == 0 ? (float)(L + 1) : 0.f) : (k == 0 ? 1.f : 0.f);
                B[L * 4 + k] = pass == 0 ? (k == 0 ? 1.f : 0.f) : (k == 0 ? (float)(L + 1) : 0.f);
            }
        hipLaunchKernelGGL(k_layout16, dim3(1), dim3(64), 0, 0, A, B, D);
        hipDeviceSynchronize();
        printf("16x16x4_4b pass %d (%s): lanes x regs 0..15\n", pass, pass == 0 ? "A lane+1" : "B lane+1");
        for (int L : {0, 1, 15, 16, 17, 31, 32, 48, 63}) {
            printf("  L%2d:", L);
            for (int r = 0; r < 16; ++r) printf(" %3.0f", D[L * 16 + r]);
            printf("\n");
        }
    }
    // exactness: random Q4_0 (nibble - 8) x int8 lane sums, every output against the integer sum
    int bad = 0, total = 0;
    for (int trial = 0; trial < 200; ++trial) {
        int ai[64][4], bi[64][4];
        for (int L = 0; L < 64; ++L)
            for (int k = 0; k < 4; ++k) {
                ai[L][k] = rnd(-8, 7);
                bi[L][k] = trial == 0 ? (k & 1 ? -128 : 127) : rnd(-128, 127);
                if (trial == 0) ai[L][k] = -8;
                A[L * 4 + k] = (float)ai[L][k];
                B[L * 4 + k] = (float)bi[L][k];
            }
        hipLaunchKernelGGL(k_layout32, dim3(1), dim3(64), 0, 0, A, B, D);
        hipDeviceSynchronize();
        // expected with the layout (row = A lane, col = B lane, same block): compare the multiset
        // of outputs per block with the integer products (layout-free check)
        long sum_dev = 0, sum_ref = 0, sq_dev = 0, sq_ref = 0;
        for (int L = 0; L < 64; ++L)
            for (int r = 0; r < 32; ++r) {
                const float v = D[L * 32 + r];
                if (v != (float)(long)v) ++bad;
                sum_dev += (long)v;
                sq_dev += (long)v * (long)v;
                ++total;
            }
        for (int b = 0; b < 2; ++b)
            for (int i = 0; i < 32; ++i)
                for (int j = 0; j < 32; ++j) {
                    long s = 0;
                    for (int k = 0; k < 4; ++k) s += (long)ai[b * 32 + i][k] * bi[b * 32 + j][k];
                    sum_ref += s;
                    sq_ref += s * s;
                }
        if (sum_dev != sum_ref || sq_dev != sq_ref) ++bad;
    }
    printf("exactness: %d bad of %d outputs / 200 trials (integral and sum/sum-of-squares equal to the integer lane sums)\n",
           bad, total);
    for (int w : {1, 2, 3, 4}) {
        printf("waves/SIMD %d: 32x32x4_2b %.2f ns  16x16x4_4b %.2f ns  32x32x16 %.2f ns per SIMD-instruction (4 acc)\n", w,
               rate(k_rate<0, 4>, 4, w), rate(k_rate<1, 4>, 4, w), rate(k_rate<2, 4>, 4, w));
    }
    printf("useful MACs: 32x32x4_2b 8192, 16x16x4_4b 4096, 32x32x16 16384 (4096 useful in the lane-masked GEMM)\n");
    return 0;
}
