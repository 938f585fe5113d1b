// Micro-benchmark (diagnostic, not product): what bounds the ordered carry chain?
// NW carrier waves, LANES active lanes each, 448-step fmaf chain over LDS-stashed (d, s).
#include <hip/hip_runtime.h>
#include <stdio.h>

template <int NW, int LANES, int MODE>  // MODE 0: d,s from LDS; 1: s from LDS, d reg; 2: reads only; 3: s only, no d
__global__ void __launch_bounds__(512) kern(float *out, long long *cyc, int total, int sbp) {
    extern __shared__ float4 sm[];
    float *st_s = (float *)sm, *st_d = st_s + 64 * sbp;
    for (int i = threadIdx.x; i < 72 * sbp; i += blockDim.x) st_s[i] = 1.0f + i * 1e-7f;
    __syncthreads();
    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
    if (wave >= NW || lane >= LANES) return;
    const int gl = wave * LANES + lane;
    const float4 *ps = (const float4 *)(st_s + (size_t)gl * sbp);
    const float4 *pd = (const float4 *)(st_d + (size_t)(gl >> 3) * sbp);
    float acc = 0.f;
    constexpr int G = 4;
    long long t0 = clock64();
    float4 as[G], ad[G], bs[G], bd[G];
    const float4 dreg = make_float4(0.5f, 0.25f, 0.125f, 1.5f);
#pragma unroll
    for (int r = 0; r < G; ++r) { as[r] = ps[r]; bs[r] = ps[G + r]; if (MODE == 0 || MODE == 2) { ad[r] = pd[r]; bd[r] = pd[G + r]; } else { ad[r] = dreg; bd[r] = dreg; } }
    for (int c = 0; c < total; c += 2 * G) {
        asm volatile("" ::: "memory");
#pragma unroll
        for (int r = 0; r < G; ++r) {
            if (MODE == 2) { acc += as[r].x + ad[r].w; continue; }
            acc = __builtin_fmaf(ad[r].x, as[r].x, acc); acc = __builtin_fmaf(ad[r].y, as[r].y, acc);
            acc = __builtin_fmaf(ad[r].z, as[r].z, acc); acc = __builtin_fmaf(ad[r].w, as[r].w, acc);
        }
        asm volatile("" ::: "memory");
        if (c + 2 * G < total) {
#pragma unroll
            for (int r = 0; r < G; ++r) { as[r] = ps[c + 2 * G + r]; if (MODE == 0 || MODE == 2) ad[r] = pd[c + 2 * G + r]; }
        }
        asm volatile("" ::: "memory");
#pragma unroll
        for (int r = 0; r < G; ++r) {
            if (MODE == 2) { acc += bs[r].x + bd[r].w; continue; }
            acc = __builtin_fmaf(bd[r].x, bs[r].x, acc); acc = __builtin_fmaf(bd[r].y, bs[r].y, acc);
            acc = __builtin_fmaf(bd[r].z, bs[r].z, acc); acc = __builtin_fmaf(bd[r].w, bs[r].w, acc);
        }
        asm volatile("" ::: "memory");
        if (c + 3 * G < total) {
#pragma unroll
            for (int r = 0; r < G; ++r) { bs[r] = ps[c + 3 * G + r]; if (MODE == 0 || MODE == 2) bd[r] = pd[c + 3 * G + r]; }
        }
    }
    long long t1 = clock64();
    out[threadIdx.x] = acc;
    if (lane == 0) cyc[wave] = t1 - t0;
}

template <int NW, int LANES, int MODE>
void run(const char *name, float *out, long long *cyc) {
    const int sbp = 452, total = 112;
    long long h[8];
    hipFuncSetAttribute((const void *)kern<NW, LANES, MODE>, hipFuncAttributeMaxDynamicSharedMemorySize, 72 * sbp * 4);
    for (int rep = 0; rep < 3; ++rep) {
        hipLaunchKernelGGL((kern<NW, LANES, MODE>), 1, 512, 72 * sbp * 4, 0, out, cyc, total, sbp);
        hipMemcpy(h, cyc, 8 * NW, hipMemcpyDeviceToHost);
    }
    long long mx = 0;
    for (int w = 0; w < NW; ++w) mx = h[w] > mx ? h[w] : mx;
    printf("%-40s max over waves %6lld cycles = %6.2f / step\n", name, mx, mx / 448.0);
}

int main() {
    float *out; long long *cyc;
    (void)hipMalloc(&out, 4096); (void)hipMalloc(&cyc, 64);
    run<1, 64, 0>("1 wave x64 lanes, d+s LDS", out, cyc);
    run<1, 64, 1>("1 wave x64 lanes, s LDS, d reg", out, cyc);
    run<1, 64, 2>("1 wave x64 lanes, reads only (d+s)", out, cyc);
    run<1, 32, 0>("1 wave x32 lanes, d+s LDS", out, cyc);
    run<2, 32, 0>("2 waves x32 lanes, d+s LDS", out, cyc);
    run<4, 16, 0>("4 waves x16 lanes, d+s LDS", out, cyc);
    run<8, 8, 0>("8 waves x8 lanes, d+s LDS", out, cyc);
    run<1, 16, 0>("1 wave x16 lanes, d+s LDS", out, cyc);
    run<1, 8, 1>("1 wave x8 lanes, s LDS, d reg", out, cyc);
    return 0;
}
