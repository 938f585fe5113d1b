// Diagnostic (not product): which device exp formulations reproduce ggml's fp16 exp table
// (fp16(glibc expf(x)), x = every non-positive finite f16)?
#include <hip/hip_runtime.h>
#include <hip/hip_fp16.h>
#include <math.h>
#include <stdio.h>
#include <string.h>

__device__ __forceinline__ unsigned short f2h_bits(float f) { return __half_as_ushort(__float2half_rn(f)); }
__device__ __forceinline__ float h2f_bits(unsigned short h) { return __half2float(__ushort_as_half(h)); }

__global__ void variants(unsigned short *out) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= 65536) return;
    const float x = h2f_bits((unsigned short)i);
    out[0 * 65536 + i] = f2h_bits((float)exp((double)x));
    out[1 * 65536 + i] = f2h_bits(expf(x));
    out[2 * 65536 + i] = f2h_bits(__expf(x));
    out[3 * 65536 + i] = f2h_bits(exp2f(x * 1.44269504088896341f));
}

static unsigned short host_f2h(float f) {  // RNE float -> half bits
    unsigned int u; memcpy(&u, &f, 4);
    unsigned int sign = (u >> 16) & 0x8000; int e = (int)((u >> 23) & 0xFF) - 127 + 15; unsigned int m = u & 0x7FFFFF;
    if (((u >> 23) & 0xFF) == 0xFF) return sign | 0x7C00 | (m ? 0x200 : 0);
    if (e >= 31) return sign | 0x7C00;
    if (e <= 0) {
        if (e < -10) return sign;
        m |= 0x800000; int shift = 14 - e; unsigned int r = m >> shift, rem = m & ((1u << shift) - 1), half = 1u << (shift - 1);
        if (rem > half || (rem == half && (r & 1))) r++;
        return sign | r;
    }
    unsigned int r = (e << 10) | (m >> 13), rem = m & 0x1FFF;
    if (rem > 0x1000 || (rem == 0x1000 && (r & 1))) r++;
    return sign | r;
}
static float host_h2f(unsigned short h) {
    unsigned int s = (h & 0x8000) << 16, e = (h >> 10) & 0x1F, m = h & 0x3FF, u;
    if (e == 0) { if (!m) u = s; else { int k = 0; while (!(m & 0x400)) { m <<= 1; k++; } m &= 0x3FF; u = s | ((113 - k) << 23) | (m << 13); } }
    else if (e == 31) u = s | 0x7F800000 | (m << 13);
    else u = s | ((e + 112) << 23) | (m << 13);
    float f; memcpy(&f, &u, 4); return f;
}

int main() {
    unsigned short *d, *h = new unsigned short[4 * 65536];
    (void)hipMalloc(&d, 4 * 65536 * 2);
    hipLaunchKernelGGL(variants, 256, 256, 0, 0, d);
    (void)hipMemcpy(h, d, 4 * 65536 * 2, hipMemcpyDeviceToHost);
    const char *names[4] = {"exp(double)", "expf", "__expf", "exp2f(x*log2e)"};
    for (int v = 0; v < 4; ++v) {
        int bad = 0, n = 0;
        for (int i = 0; i < 65536; ++i) {
            const float x = host_h2f((unsigned short)i);
            if (!(x <= 0.0f) || isinf(x)) continue;
            ++n;
            if (h[v * 65536 + i] != host_f2h(expf(x))) ++bad;
        }
        printf("%-16s mismatches %d / %d\n", names[v], bad, n);
    }
    return 0;
}
