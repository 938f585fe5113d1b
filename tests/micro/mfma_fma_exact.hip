// Is v_mfma_f32_32x32x8_f16 with ONE nonzero product per output a correctly rounded fma?  For every
// output D[m][n] = A[m][p(m)] * B[p(m)][n] + C[m][n] (the other K positions of row m are zero), the
// result is compared bit for bit with fmaf((float)a, (float)b, c) (= v_fma_mix_f32, the exact
// attention's vec_dot_f16 step).  Operands: random f16 bit patterns (normals, denormals, zeros of
// both signs; no inf/nan) and accumulators from previous steps (chains of 64 steps, as the KQV).
// build: hipcc --offload-arch=gfx950 -O3 mfma_fma_exact.hip -o mfma_fma_exact
#include <hip/hip_runtime.h>
#include <math.h>
#include <stdint.h>
#include <stdio.h>

typedef _Float16 h4 __attribute__((ext_vector_type(4)));
typedef float f16v __attribute__((ext_vector_type(16)));

__device__ uint32_t hash(uint32_t x) {
    x ^= x >> 16; x *= 0x7feb352d; x ^= x >> 15; x *= 0x846ca68b; x ^= x >> 16;
    return x;
}
__device__ _Float16 rnd_h(uint32_t r, int mode) {
    uint32_t b = r & 0xFFFF;
    if ((b & 0x7C00) == 0x7C00) b &= 0xBFFF;         // no inf / nan
    if (mode == 1) b = (b & 0x83FF);                  // denormals / zeros
    if (mode == 2) b = (b & 0x8000) | 0x3C00 | (b & 0x3FF);  // [1, 2)
    return __builtin_bit_cast(_Float16, (uint16_t)b);
}

// one wave: 32 rows m = (slot q = m >> 3, l = m & 7), p(m) = l; lane (m, kg) holds A[m][4kg..4kg+3]
__global__ void k(int steps, uint32_t seed, unsigned *bad, float *sample) {
    const int lane = threadIdx.x, m = lane & 31, kg = lane >> 5, l = m & 7;
    const int blk = blockIdx.x;
    f16v acc = {};
    float ref[16];
    for (int r = 0; r < 16; ++r) ref[r] = 0.0f;
    unsigned nbad = 0;
    for (int s = 0; s < steps; ++s) {
        const int mode = (blk + s) % 3;
        // A: row m's value a(m) at position l
        const _Float16 a = rnd_h(hash(seed ^ (blk * 7919 + s * 131 + m)), mode);
        h4 av = {0, 0, 0, 0};
        if ((l >> 2) == kg) av[l & 3] = a;
        // B: column n = lane & 31, rows 4kg..4kg+3: b(p, n)
        h4 bv;
        for (int i = 0; i < 4; ++i) bv[i] = rnd_h(hash(seed * 3 + blk * 104729 + s * 977 + (4 * kg + i) * 37 + (lane & 31)), (mode + i) % 3);
        acc = __builtin_amdgcn_mfma_f32_32x32x8f16(av, bv, acc, 0, 0, 0);
        // reference: D register r of lane (n, g): row mr = (r & 3) + 8 (r >> 2) + 4 g, p = mr & 7
        const int n = lane & 31, g = lane >> 5;
        for (int r = 0; r < 16; ++r) {
            const int mr = (r & 3) + 8 * (r >> 2) + 4 * g, p = mr & 7;
            const _Float16 ar = rnd_h(hash(seed ^ (blk * 7919 + s * 131 + mr)), mode);
            const _Float16 br = rnd_h(hash(seed * 3 + blk * 104729 + s * 977 + p * 37 + n), (mode + (p & 3)) % 3);
            ref[r] = __builtin_fmaf((float)ar, (float)br, ref[r]);
        }
    }
    for (int r = 0; r < 16; ++r)
        if (__builtin_bit_cast(uint32_t, acc[r]) != __builtin_bit_cast(uint32_t, ref[r])) {
            ++nbad;
            if (acc[r] == ref[r]) atomicAdd(bad + 2, 1u);  // equal as floats: +0 / -0
            if (sample && atomicAdd(bad + 1, 1u) == 0) { sample[0] = acc[r]; sample[1] = ref[r]; }
        }
    atomicAdd(bad, nbad);
}

int main() {
    unsigned *bad;
    float *smp;
    hipMalloc(&bad, 16);
    hipMalloc(&smp, 8);
    for (int steps : {1, 8, 64}) {
        hipMemset(bad, 0, 16);
        hipLaunchKernelGGL(k, dim3(4096), dim3(64), 0, 0, steps, 12345u + steps, bad, smp);
        unsigned h[3];
        float s[2];
        hipMemcpy(h, bad, 12, hipMemcpyDeviceToHost);
        hipMemcpy(s, smp, 8, hipMemcpyDeviceToHost);
        printf("steps %2d: %u of %u outputs differ from fmaf%s", steps, h[0], 4096u * 64u * 16u, h[0] ? "" : "\n");
        if (h[0]) printf(" (%u equal as floats; e.g. mfma %.9g %08x vs fmaf %.9g %08x)\n", h[2], s[0], *(unsigned *)&s[0], s[1], *(unsigned *)&s[1]);
    }
    return 0;
}
