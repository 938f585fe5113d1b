// ggml_ops.hip — device kernels of the ggml-compatible graph executor (csrc/ggml_api.cpp): the
// generic, strided forms of the ops src/gemma_model.cpp builds (SURVEY §8(b) "wide op surface"),
// each with the ggml CPU arithmetic the oracle restates.  The quantized
// MUL_MAT reuses the hot-path kernels (k_matvec / k_gemm_x); these cover the rest.
#include <algorithm>

#include "device_util.h"
#include "kernels.h"

namespace ghip {
namespace {

__device__ __forceinline__ void unflat(int64_t f, const int64_t ne[4], int64_t i[4]) {
    i[0] = f % ne[0];
    f /= ne[0];
    i[1] = f % ne[1];
    f /= ne[1];
    i[2] = f % ne[2];
    i[3] = f / ne[2];
}
__device__ __forceinline__ int64_t offs(const int64_t i[4], const int64_t nb[4]) {
    return i[0] * nb[0] + i[1] * nb[1] + i[2] * nb[2] + i[3] * nb[3];
}
__device__ __forceinline__ float ld_elem(const gt_desc &t, int64_t off) {
    const char *p = t.data + off;
    return t.type == T_F16 ? h2f(*(const uint16_t *)p) : *(const float *)p;
}

// GET_ROWS of a quantized / f32 / f16 matrix (ggml dequantize_row_*: (float)(q - 8) * d for Q4_0,
// (float)q * d for Q8_0)
__global__ void k_g_get_rows(gt_desc src, gt_desc idx, gt_desc dst) {
    const int64_t r = blockIdx.x, n = dst.ne[0];
    const int64_t row = *(const int32_t *)(idx.data + r * idx.nb[0]);
    const char *srow = src.data + row * src.nb[1];
    float *d = (float *)(dst.data + r * dst.nb[1]);
    for (int64_t i = threadIdx.x; i < n; i += blockDim.x) {
        float v;
        if (src.type == T_Q4_0) {
            const uint8_t *blk = (const uint8_t *)srow + (i >> 5) * 18;
            const int e = (int)(i & 31);
            const uint8_t b = blk[2 + (e & 15)];
            const int q = (e < 16 ? (b & 15) : (b >> 4)) - 8;
            v = (float)q * pin(h2f(*(const uint16_t *)blk));
        } else if (src.type == T_Q8_0) {
            const uint8_t *blk = (const uint8_t *)srow + (i >> 5) * 34;
            v = (float)(int8_t)blk[2 + (i & 31)] * pin(h2f(*(const uint16_t *)blk));
        } else if (src.type == T_Q4_K) {
            // dequantize_row_q4_K: per 64 values j, d1 = d*sc, m1 = dmin*m, y = d1*q - m1 (no FMA:
            // oracle/kquants_cpu.cpp orc_dequantize_row_q4_K)
            const uint8_t *blk = (const uint8_t *)srow + (i >> 8) * 144;
            const int e = (int)(i & 255), j = e >> 6, hi = (e >> 5) & 1, is = 2 * j + hi;
            const uint8_t *sc = blk + 4;
            int scv, mv;
            if (is < 4) {
                scv = sc[is] & 63;
                mv = sc[is + 4] & 63;
            } else {
                scv = (sc[is + 4] & 0xF) | ((sc[is - 4] >> 6) << 4);
                mv = (sc[is + 4] >> 4) | ((sc[is] >> 6) << 4);
            }
            const uint8_t qb = blk[16 + j * 32 + (e & 31)];
            const float d1 = pin(h2f(*(const uint16_t *)blk) * (float)scv);
            const float m1 = pin(h2f(*(const uint16_t *)(blk + 2)) * (float)mv);
            v = pin(d1 * (float)(hi ? qb >> 4 : qb & 15)) - m1;
        } else if (src.type == T_Q6_K) {
            // dequantize_row_q6_K: y = d*sc*(q6 - 32), left to right
            const uint8_t *blk = (const uint8_t *)srow + (i >> 8) * 210;
            const int e = (int)(i & 255), n = e >> 7, g = (e >> 5) & 3, l = e & 31;
            const uint8_t *ql = blk + n * 64, *qh = blk + 128 + n * 32;
            const int lo = (g & 1) ? ql[l + 32] : ql[l];
            const int q = (((g & 2) ? lo >> 4 : lo & 15) | (((qh[l] >> (2 * g)) & 3) << 4)) - 32;
            const int8_t scv = ((const int8_t *)(blk + 192))[n * 8 + l / 16 + 2 * g];
            v = pin(h2f(*(const uint16_t *)(blk + 208)) * (float)scv) * (float)q;
        } else if (src.type == T_F16) {
            v = h2f(((const uint16_t *)srow)[i]);
        } else {
            v = ((const float *)srow)[i];
        }
        d[i] = v;
    }
}

// elementwise: SCALE (a*s), GELU (fp16 table), MUL (a*b), ADD (a+b); b broadcast by repetition
enum { EW_SCALE = 0, EW_GELU = 1, EW_MUL = 2, EW_ADD = 3 };
__global__ void k_g_elementwise(int op, gt_desc a, gt_desc b, gt_desc dst, float s, const uint16_t *gelu_tab,
                                int gelu_clamp) {
    const int64_t n = dst.ne[0] * dst.ne[1] * dst.ne[2] * dst.ne[3];
    for (int64_t f = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; f < n; f += (int64_t)gridDim.x * blockDim.x) {
        int64_t i[4];
        unflat(f, dst.ne, i);
        const float x = ld_elem(a, offs(i, a.nb));
        float y;
        if (op == EW_SCALE) {
            y = x * s;
        } else if (op == EW_GELU) {
            if (gelu_clamp && x <= -10.0f) y = 0.0f;
            else if (gelu_clamp && x >= 10.0f) y = x;
            else y = h2f(gelu_tab[f2h(x)]);
        } else {
            const int64_t j[4] = {i[0] % b.ne[0], i[1] % b.ne[1], i[2] % b.ne[2], i[3] % b.ne[3]};
            const float z = ld_elem(b, offs(j, b.nb));
            y = op == EW_MUL ? x * z : x + z;
        }
        *(float *)(dst.data + offs(i, dst.nb)) = y;
    }
}

// RMS_NORM per row: sum of (double)(x*x) (a fixed tree, proven equal to ggml's sequential sum by
// rms_mean_certain or replaced by that sum),
// mean = (float)(sum/n), y = x * (1/sqrtf(mean + eps))
__global__ void __launch_bounds__(256) k_g_rms_norm(gt_desc a, gt_desc dst, float eps) {
    const int64_t r = blockIdx.x, n = a.ne[0];
    int64_t i[4] = {0, r % a.ne[1], (r / a.ne[1]) % a.ne[2], r / (a.ne[1] * a.ne[2])};
    const char *src = a.data + offs(i, a.nb);
    char *out = dst.data + offs(i, dst.nb);
    double part = 0.0;
    for (int64_t k = threadIdx.x; k < n; k += 256) {
        const float x = *(const float *)(src + k * a.nb[0]);
        part += (double)(x * x);
    }
    __shared__ double red[4];
    part = wave_sum_f64(part);  // any order: the mean is certified below
    if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = part;
    __syncthreads();
    const double q = div_by_n((red[0] + red[1]) + (red[2] + red[3]), n);
    float mean = (float)q;
    if (__builtin_expect(!rms_mean_certain(q, n), 0))  // workgroup-uniform; rare: ggml's own order
        mean = (float)(seq_sumsq_wave(n, [&](int64_t i0, float v[8]) {
                           for (int j = 0; j < 8; ++j)
                               v[j] = i0 + j < n ? *(const float *)(src + (i0 + j) * a.nb[0]) : 0.0f;
                       }) / (double)n);
    const float scale = 1.0f / sqrtf(mean + eps);
    for (int64_t k = threadIdx.x; k < n; k += 256)
        *(float *)(out + k * dst.nb[0]) = *(const float *)(src + k * a.nb[0]) * scale;
}

// ROPE NEOX (mode 2): rows of ne0 for (head i1, token i2) at position pos[i2]; pairs (k, k + n_dims/2)
// rotated by the host-built cos/sin table [pos][n_dims/2] (iterated theta, libm cosf/sinf)
__global__ void k_g_rope_neox(gt_desc a, gt_desc pos, gt_desc dst, int n_dims, const float *cs, const float *sn) {
    const int64_t r = blockIdx.x;  // row over (i1, i2, i3)
    int64_t i[4] = {0, r % a.ne[1], (r / a.ne[1]) % a.ne[2], r / (a.ne[1] * a.ne[2])};
    const int p = *(const int32_t *)(pos.data + i[2] * pos.nb[0]);
    const char *src = a.data + offs(i, a.nb);
    char *out = dst.data + offs(i, dst.nb);
    const int half = n_dims / 2;
    for (int64_t k = threadIdx.x; k < a.ne[0]; k += blockDim.x) {
        float y;
        if (k < half) {
            const float x0 = *(const float *)(src + k * a.nb[0]), x1 = *(const float *)(src + (k + half) * a.nb[0]);
            const float c = cs[(int64_t)p * half + k], s = sn[(int64_t)p * half + k];
            const float p0 = x0 * c, p1 = x1 * s;
            y = p0 - p1;
        } else if (k < n_dims) {
            const float x0 = *(const float *)(src + (k - half) * a.nb[0]), x1 = *(const float *)(src + k * a.nb[0]);
            const float c = cs[(int64_t)p * half + k - half], s = sn[(int64_t)p * half + k - half];
            const float p2 = x0 * s, p3 = x1 * c;
            y = p2 + p3;
        } else {
            y = *(const float *)(src + k * a.nb[0]);
        }
        *(float *)(out + k * dst.nb[0]) = y;
    }
}

// SOFT_MAX (ext): w = x*scale (+ mask[row % ne01]); max; e = f16-table exp(f16(w - max)) (w = -inf
// -> 0); the sum of the fp16 e values is exact as an integer sum of e*2^24 (= ggml's double sum);
// y = e * (float)(1/sum)
__global__ void __launch_bounds__(256) k_g_soft_max(gt_desc a, gt_desc mask, int has_mask, gt_desc dst, float scale) {
    const int64_t r = blockIdx.x, n = a.ne[0];
    int64_t i[4] = {0, r % a.ne[1], (r / a.ne[1]) % a.ne[2], r / (a.ne[1] * a.ne[2])};
    const char *src = a.data + offs(i, a.nb);
    char *out = dst.data + offs(i, dst.nb);
    const char *mrow = has_mask ? mask.data + (i[1] % mask.ne[1]) * mask.nb[1] : nullptr;
    auto w_at = [&](int64_t k) {
        float w = *(const float *)(src + k * a.nb[0]) * scale;
        if (mrow) w = w + *(const float *)(mrow + k * mask.nb[0]);
        return w;
    };
    __shared__ float redf[4];
    __shared__ unsigned long long redu[4];
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    float mx = -INFINITY;
    for (int64_t k = threadIdx.x; k < n; k += 256) mx = fmaxf(mx, w_at(k));
    mx = wave_max(mx);
    if (lane == 0) redf[wave] = mx;
    __syncthreads();
    mx = fmaxf(fmaxf(redf[0], redf[1]), fmaxf(redf[2], redf[3]));
    unsigned long long isum = 0;
    for (int64_t k = threadIdx.x; k < n; k += 256) {
        const float w = w_at(k);
        const float e = w != -INFINITY ? h2f(exp_f16_of(f2h(w - mx))) : 0.0f;
        isum += (unsigned long long)(uint32_t)(e * 16777216.0f);  // e*2^24 <= 2^24: exact in u32 (one v_cvt_u32_f32)
    }
    isum = wave_sum_u64(isum);
    if (lane == 0) redu[wave] = isum;
    __syncthreads();
    const double sum = (double)(redu[0] + redu[1] + redu[2] + redu[3]) * (1.0 / 16777216.0);
    const float v = (float)(1.0 / sum);
    for (int64_t k = threadIdx.x; k < n; k += 256) {
        const float w = w_at(k);
        const float e = w != -INFINITY ? h2f(exp_f16_of(f2h(w - mx))) : 0.0f;
        *(float *)(out + k * dst.nb[0]) = e * v;
    }
}

// CPY / CONT / the F16 INIT of MUL_MAT: element f of src (row-major logical order) -> element f of
// dst, f32 <-> f16 (RNE)
__global__ void k_g_copy(gt_desc src, gt_desc dst) {
    const int64_t n = src.ne[0] * src.ne[1] * src.ne[2] * src.ne[3];
    for (int64_t f = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; f < n; f += (int64_t)gridDim.x * blockDim.x) {
        int64_t is[4], id[4];
        unflat(f, src.ne, is);
        unflat(f, dst.ne, id);
        const char *ps = src.data + offs(is, src.nb);
        char *pd = dst.data + offs(id, dst.nb);
        if (src.type == T_F16 && dst.type == T_F16) *(uint16_t *)pd = *(const uint16_t *)ps;
        else {
            const float v = ld_elem(src, ps - src.data);
            if (dst.type == T_F16) *(uint16_t *)pd = (uint16_t)f2h(v);
            else *(float *)pd = v;
        }
    }
}

// ggml_vec_dot_f16 (AVX/F16C): 4 x 8 fp32 accumulators over steps of 32, reduce
// ((acc0+acc2)+(acc1+acc3)) lane-wise, then the 8-lane hadd tree; leftovers in double
__device__ __forceinline__ float dot_f16_ggml(const uint16_t *x, const uint16_t *y, int64_t K) {
    float acc[4][8];
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 8; ++j) acc[i][j] = 0.0f;
    const int64_t np = K & ~(int64_t)31;
    for (int64_t i = 0; i < np; i += 32)
#pragma unroll
        for (int j = 0; j < 4; ++j)
#pragma unroll
            for (int l = 0; l < 8; ++l) acc[j][l] = __builtin_fmaf(h2f(x[i + j * 8 + l]), h2f(y[i + j * 8 + l]), acc[j][l]);
    float x0[8];
#pragma unroll
    for (int l = 0; l < 8; ++l) {
        const float a = acc[0][l] + acc[2][l], b = acc[1][l] + acc[3][l];
        x0[l] = a + b;
    }
    float t0[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) t0[i] = x0[i] + x0[i + 4];
    double sumf = (double)((t0[0] + t0[1]) + (t0[2] + t0[3]));
    for (int64_t i = np; i < K; ++i) sumf += (double)(h2f(x[i]) * h2f(y[i]));
    return (float)sumf;
}

// MUL_MAT with F16 src0 (K / V cache views) and src1 already converted to contiguous f16 rows
// (ggml's INIT): dst[i01, i11, i12, i13] = dot(src0[:, i01, i12 / r2, i13 / r3], src1row(i11, i12, i13))
__global__ void k_g_mul_mat_f16(gt_desc a, const uint16_t *b16, int64_t ne10, gt_desc dst, int64_t ne11, int64_t ne12,
                                int64_t ne13) {
    const int64_t n = a.ne[1] * ne11 * ne12 * ne13;
    const int64_t gid = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (gid >= n) return;
    const int64_t i01 = gid % a.ne[1];
    int64_t c = gid / a.ne[1];
    const int64_t i11 = c % ne11;
    c /= ne11;
    const int64_t i12 = c % ne12, i13 = c / ne12;
    const int64_t r2 = ne12 / a.ne[2], r3 = ne13 / a.ne[3];
    const uint16_t *x = (const uint16_t *)(a.data + i01 * a.nb[1] + (i12 / r2) * a.nb[2] + (i13 / r3) * a.nb[3]);
    const uint16_t *y = b16 + ((i13 * ne12 + i12) * ne11 + i11) * ne10;
    *(float *)(dst.data + i01 * dst.nb[0] + i11 * dst.nb[1] + i12 * dst.nb[2] + i13 * dst.nb[3]) = dot_f16_ggml(x, y, ne10);
}

unsigned blocks_for(int64_t n, int per) { return (unsigned)std::min<int64_t>((n + per - 1) / per, 65535 * 8); }

}  // namespace

int launch_g_get_rows(const gt_desc &src, const gt_desc &idx, const gt_desc &dst, hipStream_t s) {
    hipLaunchKernelGGL(k_g_get_rows, dim3((unsigned)dst.ne[1]), dim3(256), 0, s, src, idx, dst);
    GHIP_CHECK(hipGetLastError());
    return 0;
}
int launch_g_elementwise(int op, const gt_desc &a, const gt_desc &b, const gt_desc &dst, float scale,
                         const uint16_t *gelu_tab, int gelu_clamp, hipStream_t s) {
    const int64_t n = dst.ne[0] * dst.ne[1] * dst.ne[2] * dst.ne[3];
    hipLaunchKernelGGL(k_g_elementwise, dim3(blocks_for(n, 256)), dim3(256), 0, s, op, a, b, dst, scale, gelu_tab, gelu_clamp);
    GHIP_CHECK(hipGetLastError());
    return 0;
}
int launch_g_rms_norm(const gt_desc &a, const gt_desc &dst, float eps, hipStream_t s) {
    hipLaunchKernelGGL(k_g_rms_norm, dim3((unsigned)(a.ne[1] * a.ne[2] * a.ne[3])), dim3(256), 0, s, a, dst, eps);
    GHIP_CHECK(hipGetLastError());
    return 0;
}
int launch_g_rope_neox(const gt_desc &a, const gt_desc &pos, const gt_desc &dst, int n_dims, const float *cs,
                       const float *sn, hipStream_t s) {
    hipLaunchKernelGGL(k_g_rope_neox, dim3((unsigned)(a.ne[1] * a.ne[2] * a.ne[3])), dim3(128), 0, s, a, pos, dst, n_dims, cs, sn);
    GHIP_CHECK(hipGetLastError());
    return 0;
}
int launch_g_soft_max(const gt_desc &a, const gt_desc &mask, int has_mask, const gt_desc &dst, float scale, hipStream_t s) {
    hipLaunchKernelGGL(k_g_soft_max, dim3((unsigned)(a.ne[1] * a.ne[2] * a.ne[3])), dim3(256), 0, s, a, mask, has_mask, dst, scale);
    GHIP_CHECK(hipGetLastError());
    return 0;
}
int launch_g_copy(const gt_desc &src, const gt_desc &dst, hipStream_t s) {
    const int64_t n = src.ne[0] * src.ne[1] * src.ne[2] * src.ne[3];
    hipLaunchKernelGGL(k_g_copy, dim3(blocks_for(n, 256)), dim3(256), 0, s, src, dst);
    GHIP_CHECK(hipGetLastError());
    return 0;
}
int launch_g_mul_mat_f16(const gt_desc &a, const uint16_t *b16, int64_t ne10, const gt_desc &dst, int64_t ne11,
                         int64_t ne12, int64_t ne13, hipStream_t s) {
    const int64_t n = a.ne[1] * ne11 * ne12 * ne13;
    hipLaunchKernelGGL(k_g_mul_mat_f16, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s, a, b16, ne10, dst, ne11, ne12, ne13);
    GHIP_CHECK(hipGetLastError());
    return 0;
}

}  // namespace ghip
