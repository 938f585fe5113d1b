// Micro-benchmark (diagnostic, not product): cycles of a 448-long dependent fmaf chain on one wave,
// (a) operands in registers, (b) operands streamed from LDS like the matvec carry.
#include <hip/hip_runtime.h>
#include <stdio.h>

__global__ void chain_reg(float *out, long long *cyc, float seed) {
    float acc = seed, d = seed * 0.5f, s = seed * 0.25f;
    long long t0 = clock64();
#pragma unroll 16
    for (int i = 0; i < 448; ++i) acc = __builtin_fmaf(d, s, acc);
    long long t1 = clock64();
    out[threadIdx.x] = acc;
    if (threadIdx.x == 0) cyc[0] = t1 - t0;
}

template <int G>
__global__ void __launch_bounds__(512) chain_lds(float *out, long long *cyc, int total, int sbp) {
    extern __shared__ float4 sm[];
    const int lane = threadIdx.x & 63, rr = lane >> 3;
    float *st_s = (float *)sm, *st_d = st_s + 64 * sbp;
    for (int i = threadIdx.x; i < 72 * sbp; i += blockDim.x) st_s[i] = 1.0f + i * 1e-7f;
    __syncthreads();
    if (threadIdx.x >= 64) return;
    const float4 *ps = (const float4 *)(st_s + (size_t)lane * sbp);
    const float4 *pd = (const float4 *)(st_d + (size_t)rr * sbp);
    float acc = 0.f;
    long long t0 = clock64();
    float4 as[G], ad[G], bs[G], bd[G];
    _Pragma("unroll") for (int r = 0; r < G; ++r) { as[r] = ps[r]; ad[r] = pd[r]; bs[r] = ps[G + r]; bd[r] = pd[G + r]; }
    for (int c = 0; c < total; c += 2 * G) {
        asm volatile("" ::: "memory");
        _Pragma("unroll") for (int r = 0; r < G; ++r) {
            acc = __builtin_fmaf(ad[r].x, as[r].x, acc); acc = __builtin_fmaf(ad[r].y, as[r].y, acc);
            acc = __builtin_fmaf(ad[r].z, as[r].z, acc); acc = __builtin_fmaf(ad[r].w, as[r].w, acc);
        }
        asm volatile("" ::: "memory");
        if (c + 2 * G < total) _Pragma("unroll") for (int r = 0; r < G; ++r) { as[r] = ps[c + 2 * G + r]; ad[r] = pd[c + 2 * G + r]; }
        asm volatile("" ::: "memory");
        _Pragma("unroll") for (int r = 0; r < G; ++r) {
            acc = __builtin_fmaf(bd[r].x, bs[r].x, acc); acc = __builtin_fmaf(bd[r].y, bs[r].y, acc);
            acc = __builtin_fmaf(bd[r].z, bs[r].z, acc); acc = __builtin_fmaf(bd[r].w, bs[r].w, acc);
        }
        asm volatile("" ::: "memory");
        if (c + 3 * G < total) _Pragma("unroll") for (int r = 0; r < G; ++r) { bs[r] = ps[c + 3 * G + r]; bd[r] = pd[c + 3 * G + r]; }
    }
    long long t1 = clock64();
    out[threadIdx.x] = acc;
    if (threadIdx.x == 0) cyc[0] = t1 - t0;
}

int main() {
    float *out; long long *cyc, h;
    hipMalloc(&out, 4096); hipMalloc(&cyc, 8);
    for (int rep = 0; rep < 3; ++rep) {
        hipLaunchKernelGGL(chain_reg, 1, 64, 0, 0, out, cyc, 1.0f);
        hipMemcpy(&h, cyc, 8, hipMemcpyDeviceToHost);
        printf("reg chain 448 fma: %lld cycles (%.2f / fma)\n", h, h / 448.0);
    }
    const int sbp = 452, total = 112;
    for (int rep = 0; rep < 2; ++rep) {
        hipLaunchKernelGGL(chain_lds<4>, 1, 512, 72 * sbp * 4, 0, out, cyc, total, sbp);
        hipMemcpy(&h, cyc, 8, hipMemcpyDeviceToHost);
        printf("lds chain 448 fma G=4: %lld cycles (%.2f / fma)\n", h, h / 448.0);
        hipLaunchKernelGGL(chain_lds<7>, 1, 512, 72 * sbp * 4, 0, out, cyc, total, sbp);
        hipMemcpy(&h, cyc, 8, hipMemcpyDeviceToHost);
        printf("lds chain 448 fma G=7: %lld cycles (%.2f / fma)\n", h, h / 448.0);
        hipLaunchKernelGGL(chain_lds<8>, 1, 512, 72 * sbp * 4, 0, out, cyc, total, sbp);
        hipMemcpy(&h, cyc, 8, hipMemcpyDeviceToHost);
        printf("lds chain 448 fma G=8: %lld cycles (%.2f / fma)\n", h, h / 448.0);
        hipLaunchKernelGGL(chain_lds<14>, 1, 512, 72 * sbp * 4, 0, out, cyc, total, sbp);
        hipMemcpy(&h, cyc, 8, hipMemcpyDeviceToHost);
        printf("lds chain 448 fma G=14: %lld cycles (%.2f / fma)\n", h, h / 448.0);
    }
    int wg;
    hipDeviceGetAttribute(&wg, hipDeviceAttributeClockRate, 0);
    printf("clock rate attr %d kHz\n", wg);
    return 0;
}
