// Which (m, n) each f32-MFMA output register holds, found by search: for every lane / register of
// one v_mfma_f32_16x16x4_f32 (and 32x32x2_f32) the kernel looks for the (m, n) whose fmaf chain over
// K (H1) equals the register bit for bit, and prints the map and the number of registers with no
// H1 match (the exactness question of mfma_f32_exact.hip, independent of a layout guess).
// build: hipcc --offload-arch=gfx950 -O3 mfma_f32_layout.hip -o mfma_f32_layout
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>

typedef float f4v __attribute__((ext_vector_type(4)));
typedef float f16v __attribute__((ext_vector_type(16)));

__device__ uint32_t hash(uint32_t x) {
    x ^= x >> 16; x *= 0x7feb352d; x ^= x >> 15; x *= 0x846ca68b; x ^= x >> 16;
    return x;
}
__device__ float rnd(uint32_t r) {
    uint32_t b = r & 0xFFFF;
    if ((b & 0x7C00) == 0x7C00) b &= 0xBFFF;
    return (float)__builtin_bit_cast(_Float16, (uint16_t)b);
}
template <int M, int K>
__device__ float Aval(uint32_t seed, int blk, int m, int k) { return rnd(hash(seed ^ (blk * 7919u + m * 17u + k * 1000003u))); }
template <int M, int K>
__device__ float Bval(uint32_t seed, int blk, int k, int n) { return rnd(hash(seed * 3u + blk * 104729u + k * 37u + n * 5u + 77u)); }

template <int M, int K, int NR>
__device__ void search(const float *acc, uint32_t seed, int blk, int *map, unsigned *nomatch, unsigned *nochain) {
    const int lane = threadIdx.x;
    for (int r = 0; r < NR; ++r) {
        const uint32_t want = __builtin_bit_cast(uint32_t, acc[r]);
        int found = -1;
        bool any_sum = false;
        for (int m = 0; m < M && found < 0; ++m)
            for (int n = 0; n < M; ++n) {
                float h1 = 0.0f;
                double s = 0.0;
                for (int k = 0; k < K; ++k) {
                    h1 = __builtin_fmaf(Aval<M, K>(seed, blk, m, k), Bval<M, K>(seed, blk, k, n), h1);
                    s += (double)Aval<M, K>(seed, blk, m, k) * (double)Bval<M, K>(seed, blk, k, n);
                }
                if (__builtin_bit_cast(uint32_t, h1) == want) { found = m * M + n; break; }
                if (fabs((double)acc[r] - s) <= 1e-6 * fabs(s) + 1e-30) any_sum = true;
            }
        if (blk == 0) map[lane * NR + r] = found;
        if (found < 0) {
            atomicAdd(nomatch, 1u);
            if (!any_sum) atomicAdd(nochain, 1u);
        }
    }
}

__global__ void k16(uint32_t seed, int *map, unsigned *cnt) {
    const int lane = threadIdx.x, blk = blockIdx.x;
    f4v z = {0, 0, 0, 0};
    f4v d = __builtin_amdgcn_mfma_f32_16x16x4f32(Aval<16, 4>(seed, blk, lane % 16, lane / 16),
                                                 Bval<16, 4>(seed, blk, lane / 16, lane % 16), z, 0, 0, 0);
    float acc[4] = {d[0], d[1], d[2], d[3]};
    search<16, 4, 4>(acc, seed, blk, map, cnt, cnt + 1);
}
__global__ void k32(uint32_t seed, int *map, unsigned *cnt) {
    const int lane = threadIdx.x, blk = blockIdx.x;
    f16v z = {};
    f16v d = __builtin_amdgcn_mfma_f32_32x32x2f32(Aval<32, 2>(seed, blk, lane % 32, lane / 32),
                                                  Bval<32, 2>(seed, blk, lane / 32, lane % 32), z, 0, 0, 0);
    float acc[16];
    for (int r = 0; r < 16; ++r) acc[r] = d[r];
    search<32, 2, 16>(acc, seed, blk, map, cnt, cnt + 1);
}

int main() {
    int *map;
    unsigned *cnt;
    hipMalloc(&map, 64 * 16 * 4);
    hipMalloc(&cnt, 8);
    for (int shape = 0; shape < 2; ++shape) {
        const int NR = shape == 0 ? 4 : 16, M = shape == 0 ? 16 : 32, nblk = 256;
        hipMemset(cnt, 0, 8);
        hipMemset(map, 0xff, 64 * 16 * 4);
        if (shape == 0) hipLaunchKernelGGL(k16, dim3(nblk), dim3(64), 0, 0, 12345u, map, cnt);
        else hipLaunchKernelGGL(k32, dim3(nblk), dim3(64), 0, 0, 12345u, map, cnt);
        int h[64 * 16];
        unsigned c[2];
        hipMemcpy(h, map, sizeof h, hipMemcpyDeviceToHost);
        hipMemcpy(c, cnt, 8, hipMemcpyDeviceToHost);
        printf("%s: %u of %u registers match no (m, n) fmaf chain (%u of those not even the exact sum)\n",
               shape == 0 ? "16x16x4f32" : "32x32x2f32", c[0], nblk * 64 * NR, c[1]);
        printf("  map (lane: r -> m,n) for block 0, lanes 0,1,15,16,31,32,63:\n");
        for (int lane : {0, 1, 15, 16, 31, 32, 63}) {
            printf("   lane %2d:", lane);
            for (int r = 0; r < NR; ++r) {
                const int v = h[lane * NR + r];
                if (v < 0) printf(" ?");
                else printf(" %d,%d", v / M, v % M);
            }
            printf("\n");
        }
    }
    return 0;
}
