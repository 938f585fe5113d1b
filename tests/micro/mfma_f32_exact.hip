// Are the f32-input MFMAs (v_mfma_f32_16x16x4_f32, v_mfma_f32_32x32x2_f32) an fmaf chain over K?
// The exact prefill attention's vec_dot_f16 is 32 fmaf chains per output; if one MFMA
// step equals fmaf(a_K-1, b_K-1, ... fmaf(a_0, b_0, c)) bit for bit, a chain's consecutive terms can
// ride the K dimension.  Operands are f16 values widened to f32 (q16 / k16 / P16 / v16: products are
// exact in f32), random bit patterns (wide exponents, f16 denormals, signed zeros; no inf / nan) and
// N(0, 1)-like values, chained over 1 / 8 / 64 MFMAs (D fed back as C).  Hypotheses counted per output:
//   H1 fmaf chain in K order 0..K-1;  H2 fmaf chain in reverse K order;  H3 c + (sum of the K
//   products, one rounding);  H4 (c + p0 + ... computed as pairwise (p0+p1)+(p2+p3) then + c).
// build: hipcc --offload-arch=gfx950 -O3 mfma_f32_exact.hip -o mfma_f32_exact
#include <hip/hip_runtime.h>
#include <math.h>
#include <stdint.h>
#include <stdio.h>

typedef float f4v __attribute__((ext_vector_type(4)));
typedef float f16v __attribute__((ext_vector_type(16)));

__device__ uint32_t hash(uint32_t x) {
    x ^= x >> 16; x *= 0x7feb352d; x ^= x >> 15; x *= 0x846ca68b; x ^= x >> 16;
    return x;
}
__device__ float rnd(uint32_t r, int mode) {
    uint32_t b = r & 0xFFFF;
    if ((b & 0x7C00) == 0x7C00) b &= 0xBFFF;                   // no inf / nan
    if (mode == 1) b = (b & 0x8000) | (0x3000 + (b & 0x0FFF));  // |x| in [2^-3, 2^1): attention-like
    if (mode == 2) b = (b & 0x8000) | 0x3C00 | (b & 0x3FF);     // [1, 2)
    return (float)__builtin_bit_cast(_Float16, (uint16_t)b);
}

template <int K>
__device__ void refs(const float *a, const float *b, float c, float out[4]) {
    float h1 = c;
    for (int k = 0; k < K; ++k) h1 = __builtin_fmaf(a[k], b[k], h1);
    float h2 = c;
    for (int k = K - 1; k >= 0; --k) h2 = __builtin_fmaf(a[k], b[k], h2);
    double s = 0.0;
    for (int k = 0; k < K; ++k) s += (double)a[k] * (double)b[k];
    const float h3 = (float)((double)c + s);
    float h4;
    if (K == 4) h4 = ((a[0] * b[0] + a[1] * b[1]) + (a[2] * b[2] + a[3] * b[3])) + c;
    else h4 = (a[0] * b[0] + a[1] * b[1]) + c;
    out[0] = h1; out[1] = h2; out[2] = h3; out[3] = h4;
}

// 16x16x4: A lane l -> A[l % 16][l / 16]; B lane l -> B[l / 16][l % 16]; D[4 (l / 16) + i][l % 16]
__global__ void k16(int steps, uint32_t seed, int mode, unsigned *bad) {
    const int lane = threadIdx.x, blk = blockIdx.x;
    f4v acc = {0, 0, 0, 0};
    float ref[4][4] = {};
    for (int s = 0; s < steps; ++s) {
        auto A = [&](int m, int k) { return rnd(hash(seed ^ (blk * 7919u + s * 131u + m * 17u + k)), mode); };
        auto B = [&](int k, int n) { return rnd(hash(seed * 3u + blk * 104729u + s * 977u + k * 37u + n * 5u), (mode + k) % 3); };
        acc = __builtin_amdgcn_mfma_f32_16x16x4f32(A(lane % 16, lane / 16), B(lane / 16, lane % 16), acc, 0, 0, 0);
        const int n = lane % 16;
        for (int i = 0; i < 4; ++i) {
            const int m = 4 * (lane / 16) + i;
            float a[4], b[4];
            for (int k = 0; k < 4; ++k) { a[k] = A(m, k); b[k] = B(k, n); }
            for (int h = 0; h < 4; ++h) {
                float o[4];
                refs<4>(a, b, ref[h][i], o);
                ref[h][i] = o[h];
            }
        }
    }
    for (int h = 0; h < 4; ++h)
        for (int i = 0; i < 4; ++i)
            if (__builtin_bit_cast(uint32_t, acc[i]) != __builtin_bit_cast(uint32_t, ref[h][i])) atomicAdd(bad + h, 1u);
}

// 32x32x2: A lane l -> A[l % 32][l / 32]; B lane l -> B[l / 32][l % 32]; D reg r of lane l:
// row (r & 3) + 8 (r >> 2) + 4 (l / 32), column l % 32
__global__ void k32(int steps, uint32_t seed, int mode, unsigned *bad) {
    const int lane = threadIdx.x, blk = blockIdx.x;
    f16v acc = {};
    float ref[4][16] = {};
    for (int s = 0; s < steps; ++s) {
        auto A = [&](int m, int k) { return rnd(hash(seed ^ (blk * 7919u + s * 131u + m * 17u + k)), mode); };
        auto B = [&](int k, int n) { return rnd(hash(seed * 3u + blk * 104729u + s * 977u + k * 37u + n * 5u), (mode + k) % 3); };
        acc = __builtin_amdgcn_mfma_f32_32x32x2f32(A(lane % 32, lane / 32), B(lane / 32, lane % 32), acc, 0, 0, 0);
        const int n = lane % 32;
        for (int r = 0; r < 16; ++r) {
            const int m = (r & 3) + 8 * (r >> 2) + 4 * (lane / 32);
            float a[2] = {A(m, 0), A(m, 1)}, b[2] = {B(0, n), B(1, n)};
            for (int h = 0; h < 4; ++h) {
                float o[4];
                refs<2>(a, b, ref[h][r], o);
                ref[h][r] = o[h];
            }
        }
    }
    for (int h = 0; h < 4; ++h)
        for (int r = 0; r < 16; ++r)
            if (__builtin_bit_cast(uint32_t, acc[r]) != __builtin_bit_cast(uint32_t, ref[h][r])) atomicAdd(bad + h, 1u);
}

int main() {
    unsigned *bad;
    hipMalloc(&bad, 16);
    const int nblk = 2048;
    for (int shape = 0; shape < 2; ++shape)
        for (int mode = 0; mode < 3; ++mode)
            for (int steps : {1, 8, 64}) {
                hipMemset(bad, 0, 16);
                if (shape == 0) hipLaunchKernelGGL(k16, dim3(nblk), dim3(64), 0, 0, steps, 777u + steps + mode, mode, bad);
                else hipLaunchKernelGGL(k32, dim3(nblk), dim3(64), 0, 0, steps, 777u + steps + mode, mode, bad);
                unsigned h[4];
                hipMemcpy(h, bad, 16, hipMemcpyDeviceToHost);
                const unsigned tot = nblk * 64u * (shape == 0 ? 4u : 16u);
                printf("%s mode %d steps %2d: of %u outputs, differ from H1 fmaf-chain %u, H2 reverse chain %u, "
                       "H3 one rounding %u, H4 pairwise %u\n", shape == 0 ? "16x16x4f32" : "32x32x2f32", mode, steps, tot,
                       h[0], h[1], h[2], h[3]);
            }
    return 0;
}
