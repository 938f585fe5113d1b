// ggml_semantics.cpp — ORACLE (test infrastructure only; see oracle.h header).
//
// Clean-room restatement of the ggml (Feb–Mar 2024, AVX2/F16C host) CPU arithmetic that the
// reference's MUL_MAT hot path and its neighbouring graph ops run.  The ggml fork is not
// vendored, so every function cites the SURVEY Appendix A item it follows
// plus the reference call site that reaches it.  Compiled with -ffp-contract=off: every a*b+c
// below is two roundings unless written as fmaf().
//
// PARITY: unpinned against ggml itself (no ggml source/tests here); pinned only by the analytic
// known-answer tests and the HF-transformers wiring golden.
#include "oracle.h"

#include <immintrin.h>
#include <math.h>
#include <string.h>

#include <algorithm>

namespace {

struct block_q4_0 { uint16_t d; uint8_t qs[16]; };  // 18 B / 32 values
struct block_q8_0 { uint16_t d; int8_t qs[32]; };   // 34 B / 32 values
static_assert(sizeof(block_q4_0) == 18, "q4_0 size");
static_assert(sizeof(block_q8_0) == 34, "q8_0 size");

uint16_t g_exp_f16[1 << 16];
uint16_t g_gelu_f16[1 << 16];
int g_tables_ready = 0;
int g_gelu_clamp = 0;

inline uint32_t fbits(float f) { uint32_t u; memcpy(&u, &f, 4); return u; }
inline float bitsf(uint32_t u) { float f; memcpy(&f, &u, 4); return f; }

}  // namespace

// ---------------------------------------------------------------- fp16 (RNE)
// Portable restatements (_sw) and the F16C forms ggml's x86 build uses (GGML_FP16_TO_FP32 /
// GGML_FP32_TO_FP16 = _cvtsh_ss / _cvtss_sh); test_oracle_kat checks they agree bitwise.
extern "C" float orc_fp16_to_fp32_sw(uint16_t h) {
    const uint32_t sign = (uint32_t)(h & 0x8000) << 16;
    uint32_t exp = (h >> 10) & 0x1f, mant = h & 0x3ff;
    if (exp == 0) {
        if (mant == 0) return bitsf(sign);
        // subnormal: value = mant * 2^-24 (exact in fp32)
        float v = (float)mant * 5.9604644775390625e-08f;
        return sign ? -v : v;
    }
    if (exp == 31) return bitsf(sign | 0x7f800000u | (mant << 13));
    return bitsf(sign | ((exp + 112) << 23) | (mant << 13));
}

extern "C" uint16_t orc_fp32_to_fp16_sw(float f) {
    const uint32_t x = fbits(f);
    const uint16_t sign = (uint16_t)((x >> 16) & 0x8000);
    const uint32_t ax = x & 0x7fffffffu;
    if (ax >= 0x7f800000u) {                       // inf / nan
        return (uint16_t)(sign | 0x7c00 | (ax > 0x7f800000u ? (0x200 | ((ax >> 13) & 0x3ff)) : 0));
    }
    if (ax >= 0x477ff000u) return (uint16_t)(sign | 0x7c00);  // rounds to >= 65536 -> inf
    if (ax < 0x38800000u) {                        // result subnormal (or zero) in fp16
        if (ax < 0x33000000u) return sign;         // < 2^-25: rounds to 0 (ties-to-even at 2^-25)
        const uint32_t e = ax >> 23;               // 102..112
        const uint32_t m = (ax & 0x7fffff) | 0x800000;
        const uint32_t shift = 126 - e;            // value = m * 2^(e-150); unit 2^-24
        uint32_t q = m >> shift;
        const uint32_t rem = m & ((1u << shift) - 1), half = 1u << (shift - 1);
        if (rem > half || (rem == half && (q & 1))) q++;
        return (uint16_t)(sign | q);
    }
    // normal: re-bias exponent, round mantissa 23 -> 10 bits RNE (carry may bump exponent)
    uint32_t r = ((ax >> 13) - (112u << 10));
    const uint32_t rem = ax & 0x1fff;
    if (rem > 0x1000 || (rem == 0x1000 && (r & 1))) r++;
    return (uint16_t)(sign | r);
}

extern "C" float orc_fp16_to_fp32(uint16_t h) { return _cvtsh_ss(h); }
extern "C" uint16_t orc_fp32_to_fp16(float f) { return (uint16_t)_cvtss_sh(f, _MM_FROUND_TO_NEAREST_INT); }

// mismatches between the F16C and portable forms: every fp16 pattern, and every `stride`-th fp32
// bit pattern plus each exponent's rounding boundaries (ties, +-1 ulp around them)
extern "C" int64_t orc_fp16_selfcheck(uint32_t stride) {
    int64_t bad = 0;
    for (uint32_t h = 0; h < 65536; ++h) {  // F16C quiets signalling NaNs; NaN-ness must match
        const float a = orc_fp16_to_fp32((uint16_t)h), b = orc_fp16_to_fp32_sw((uint16_t)h);
        bad += (a != a && b != b) ? 0 : fbits(a) != fbits(b);
    }
    auto one = [&](uint32_t u) { bad += orc_fp32_to_fp16(bitsf(u)) != orc_fp32_to_fp16_sw(bitsf(u)); };
    for (uint64_t u = 0; u <= 0xffffffffull; u += stride ? stride : 1) one((uint32_t)u);
    for (uint32_t sgn = 0; sgn < 2; ++sgn)
        for (uint32_t e = 0; e < 256; ++e)
            for (uint32_t m = 0; m < (1u << 13); m += 0x1000 / 8) {
                const uint32_t base = (sgn << 31) | (e << 23);
                for (uint32_t hi = 0; hi < 1024; hi += 37)
                    for (int d = -1; d <= 1; ++d) one(base | ((((hi << 13) | m) + d) & 0x7fffff));
            }
    return bad;
}

// ---------------------------------------------------------------- fp16 lookup tables
// ggml_init fills table_exp_f16[h] = f16(expf(f32(h))) and
// table_gelu_f16[h] = f16(gelu_f32(f32(h))) for every fp16 bit pattern h.
static float gelu_f32(float x) {
    const float GELU_COEF_A = 0.044715f;
    const float SQRT_2_OVER_PI = 0.79788456080286535587989211986876f;
    // 0.5f*x*(1.0f + tanhf(SQRT_2_OVER_PI*x*(1.0f + GELU_COEF_A*x*x)))  (no contraction)
    float inner = 1.0f + GELU_COEF_A * x * x;
    float t = tanhf(SQRT_2_OVER_PI * x * inner);
    return 0.5f * x * (1.0f + t);
}

extern "C" void orc_init_tables(int gelu_clamp) {
    g_gelu_clamp = gelu_clamp;
    if (g_tables_ready) return;
    for (int i = 0; i < (1 << 16); ++i) {
        const float f = orc_fp16_to_fp32((uint16_t)i);
        g_exp_f16[i] = orc_fp32_to_fp16(expf(f));
        g_gelu_f16[i] = orc_fp32_to_fp16(gelu_f32(f));
    }
    g_tables_ready = 1;
}
extern "C" const uint16_t *orc_table_exp_f16(void) { orc_init_tables(g_gelu_clamp); return g_exp_f16; }
extern "C" const uint16_t *orc_table_gelu_f16(void) { orc_init_tables(g_gelu_clamp); return g_gelu_f16; }

// ---------------------------------------------------------------- quantizers
// SURVEY A.1 quantize_row_q4_0_reference: signed max of largest |x|, d = max/-8,
// id = d ? 1/d : 0, q = min(15, (int8)(x*id + 8.5f)); element j<16 low nibble, j>=16 high.
extern "C" void orc_quantize_row_q4_0_ref(const float *x, void *vy, int k) {
    block_q4_0 *y = (block_q4_0 *)vy;
    const int nb = k / 32;
    for (int i = 0; i < nb; i++) {
        float amax = 0.0f, max = 0.0f;
        for (int j = 0; j < 32; j++) {
            const float v = x[i * 32 + j];
            if (amax < fabsf(v)) { amax = fabsf(v); max = v; }
        }
        const float d = max / -8;
        const float id = d != 0.0f ? 1.0f / d : 0.0f;
        y[i].d = orc_fp32_to_fp16(d);
        for (int j = 0; j < 16; ++j) {
            const float x0 = x[i * 32 + j] * id;
            const float x1 = x[i * 32 + 16 + j] * id;
            const float t0 = x0 + 8.5f, t1 = x1 + 8.5f;
            const uint8_t xi0 = (uint8_t)std::min(15, (int)(int8_t)(int)t0);
            const uint8_t xi1 = (uint8_t)std::min(15, (int)(int8_t)(int)t1);
            y[i].qs[j] = (uint8_t)(xi0 | (xi1 << 4));
        }
    }
}

// SURVEY A.1 quantize_row_q8_0_reference: d = amax/127, id = d ? 1/d : 0, q = roundf(x*id)
extern "C" void orc_quantize_row_q8_0_ref(const float *x, void *vy, int k) {
    block_q8_0 *y = (block_q8_0 *)vy;
    const int nb = k / 32;
    for (int i = 0; i < nb; i++) {
        float amax = 0.0f;
        for (int j = 0; j < 32; j++) amax = std::max(amax, fabsf(x[i * 32 + j]));
        const float d = amax / 127.0f;
        const float id = d != 0.0f ? 1.0f / d : 0.0f;
        y[i].d = orc_fp32_to_fp16(d);
        for (int j = 0; j < 32; ++j) y[i].qs[j] = (int8_t)roundf(x[i * 32 + j] * id);
    }
}

// SURVEY A.2 quantize_row_q8_0 (AVX2 path, what MUL_MAT INIT runs on the author's host):
// amax = max|x|; d = amax/127.f stored fp16 RNE; id = amax ? 127.f/amax : 0 (NOT 1/d);
// q = round-half-even(x*id).  Restated for the activation vector quantized once per matvec
// (the INIT phase that feeds src/hpc.cpp:216's `wdata`).
extern "C" void orc_quantize_row_q8_0(const float *x, void *vy, int k) {
    block_q8_0 *y = (block_q8_0 *)vy;
    const int nb = k / 32;
    for (int i = 0; i < nb; i++) {
        float amax = 0.0f;
        for (int j = 0; j < 32; j++) amax = std::max(amax, fabsf(x[i * 32 + j]));
        const float d = amax / 127.f;
        y[i].d = orc_fp32_to_fp16(d);
        const float id = (amax != 0.0f) ? 127.f / amax : 0.0f;
        for (int j = 0; j < 32; ++j) y[i].qs[j] = (int8_t)(int)nearbyintf(x[i * 32 + j] * id);
    }
}

extern "C" void orc_dequantize_row_q4_0(const void *vx, float *y, int k) {
    const block_q4_0 *x = (const block_q4_0 *)vx;
    for (int i = 0; i < k / 32; i++) {
        const float d = orc_fp16_to_fp32(x[i].d);
        for (int j = 0; j < 16; ++j) {
            const int x0 = (x[i].qs[j] & 0x0F) - 8, x1 = (x[i].qs[j] >> 4) - 8;
            y[i * 32 + j] = x0 * d;
            y[i * 32 + j + 16] = x1 * d;
        }
    }
}

extern "C" void orc_dequantize_row_q8_0(const void *vx, float *y, int k) {
    const block_q8_0 *x = (const block_q8_0 *)vx;
    for (int i = 0; i < k / 32; i++) {
        const float d = orc_fp16_to_fp32(x[i].d);
        for (int j = 0; j < 32; ++j) y[i * 32 + j] = x[i].qs[j] * d;
    }
}

extern "C" size_t orc_row_size(int type, int64_t ne) {
    switch (type) {
        case ORC_F32: return (size_t)ne * 4;
        case ORC_F16: return (size_t)ne * 2;
        case ORC_Q4_0: return (size_t)(ne / 32) * 18;
        case ORC_Q8_0: return (size_t)(ne / 32) * 34;
        case ORC_Q4_K: return (size_t)(ne / 256) * 144;
        case ORC_Q6_K: return (size_t)(ne / 256) * 210;
        case ORC_Q8_K: return (size_t)(ne / 256) * 292;
    }
    return 0;
}

// ---------------------------------------------------------------- vec_dot (ordered)
// per block i, d = f32(x.d)*f32(y.d) (one fp32 multiply); 8 lanes, lane l = exact
// int32 sum of elements 4l..4l+3; acc_l = fmaf(d, (float)lane_l, acc_l); final
// ((a0+a4)+(a2+a6)) + ((a1+a5)+(a3+a7))  (hsum_float_8).  Called per (row, col) from
// src/hpc.cpp:35-36 through the vec_dot function pointer.
static inline float hsum8(const float a[8]) {
    const float r0 = a[0] + a[4], r1 = a[1] + a[5], r2 = a[2] + a[6], r3 = a[3] + a[7];
    const float s0 = r0 + r2, s1 = r1 + r3;
    return s0 + s1;
}

extern "C" void orc_block_lane_sums(int wtype, const void *wb, const void *ab, int32_t lanes[8]) {
    const block_q8_0 *a = (const block_q8_0 *)ab;
    int8_t w[32];
    if (wtype == ORC_Q4_0) {
        const block_q4_0 *x = (const block_q4_0 *)wb;
        for (int j = 0; j < 16; ++j) {
            w[j] = (int8_t)((x->qs[j] & 0x0F) - 8);
            w[j + 16] = (int8_t)((x->qs[j] >> 4) - 8);
        }
    } else {
        memcpy(w, ((const block_q8_0 *)wb)->qs, 32);
    }
    for (int l = 0; l < 8; ++l) {
        int32_t s = 0;
        for (int k = 0; k < 4; ++k) s += (int32_t)w[4 * l + k] * (int32_t)a->qs[4 * l + k];
        lanes[l] = s;
    }
}

template <int WTYPE>
static void vec_dot_quant_ordered(int n, float *s, const void *vx, const void *vy) {
    const int nb = n / 32;
    const size_t wbytes = WTYPE == ORC_Q4_0 ? sizeof(block_q4_0) : sizeof(block_q8_0);
    const block_q8_0 *y = (const block_q8_0 *)vy;
    float acc[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    for (int i = 0; i < nb; ++i) {
        const uint8_t *xb = (const uint8_t *)vx + (size_t)i * wbytes;
        uint16_t xd; memcpy(&xd, xb, 2);
        const float d = orc_fp16_to_fp32(xd) * orc_fp16_to_fp32(y[i].d);
        int32_t lanes[8];
        orc_block_lane_sums(WTYPE, xb, &y[i], lanes);
        for (int l = 0; l < 8; ++l) acc[l] = fmaf(d, (float)lanes[l], acc[l]);
    }
    *s = hsum8(acc);
}

extern "C" void orc_vec_dot_q4_0_q8_0(int n, float *s, const void *vx, const void *vy) {
    vec_dot_quant_ordered<ORC_Q4_0>(n, s, vx, vy);
}
extern "C" void orc_vec_dot_q8_0_q8_0(int n, float *s, const void *vx, const void *vy) {
    vec_dot_quant_ordered<ORC_Q8_0>(n, s, vx, vy);
}

// SURVEY A.4 ggml_vec_dot_f16 (AVX + F16C + FMA): 4 accumulators x 8 lanes over steps of 32;
// sum[j] = fmaf(x, y, sum[j]) with element index i*32 + j*8 + lane; reduce sum0+=sum2,
// sum1+=sum3, sum0+=sum1; fold 128-bit halves; hadd twice; tail (none for n%32==0) in double.
// Call sites: the KQ and KQV mul_mats (src/gemma_model.cpp:474, 485) -> src/hpc.cpp:35-36.
static float reduce_f16_acc(float acc[4][8]) {
    float x0[8];
    for (int l = 0; l < 8; ++l) {
        const float a = acc[0][l] + acc[2][l];
        const float b = acc[1][l] + acc[3][l];
        x0[l] = a + b;
    }
    float t0[4];
    for (int i = 0; i < 4; ++i) t0[i] = x0[i] + x0[i + 4];
    const float h0 = t0[0] + t0[1], h1 = t0[2] + t0[3];
    return h0 + h1;
}

extern "C" void orc_vec_dot_f16(int n, float *s, const uint16_t *x, const uint16_t *y) {
    const int np = n & ~31;
    float acc[4][8] = {{0}};
    for (int i = 0; i < np; i += 32)
        for (int j = 0; j < 4; ++j)
            for (int l = 0; l < 8; ++l) {
                const int e = i + j * 8 + l;
                acc[j][l] = fmaf(orc_fp16_to_fp32(x[e]), orc_fp16_to_fp32(y[e]), acc[j][l]);
            }
    double sumf = reduce_f16_acc(acc);
    for (int i = np; i < n; ++i) sumf += (double)(orc_fp16_to_fp32(x[i]) * orc_fp16_to_fp32(y[i]));
    *s = (float)sumf;
}

// ---------------------------------------------------------------- vec_dot (AVX2, timing path)
// Same arithmetic with intrinsics (bit-identical to the ordered versions above; tested).
static inline __m256 mul_sum_i8_pairs_float(__m256i x, __m256i y) {
    const __m256i ax = _mm256_sign_epi8(x, x);
    const __m256i sy = _mm256_sign_epi8(y, x);
    const __m256i dot = _mm256_maddubs_epi16(ax, sy);
    const __m256i summed = _mm256_madd_epi16(_mm256_set1_epi16(1), dot);
    return _mm256_cvtepi32_ps(summed);
}
static inline float hsum_float_8(__m256 x) {
    __m128 res = _mm256_extractf128_ps(x, 1);
    res = _mm_add_ps(res, _mm256_castps256_ps128(x));
    res = _mm_add_ps(res, _mm_movehl_ps(res, res));
    res = _mm_add_ss(res, _mm_movehdup_ps(res));
    return _mm_cvtss_f32(res);
}

extern "C" void orc_vec_dot_q4_0_q8_0_avx2(int n, float *s, const void *vx, const void *vy) {
    const block_q4_0 *x = (const block_q4_0 *)vx;
    const block_q8_0 *y = (const block_q8_0 *)vy;
    const int nb = n / 32;
    __m256 acc = _mm256_setzero_ps();
    for (int i = 0; i < nb; ++i) {
        const __m256 d = _mm256_set1_ps(_cvtsh_ss(x[i].d) * _cvtsh_ss(y[i].d));
        const __m128i tmp = _mm_loadu_si128((const __m128i *)x[i].qs);
        __m256i qx = _mm256_set_m128i(_mm_srli_epi16(tmp, 4), tmp);
        qx = _mm256_and_si256(_mm256_set1_epi8(0xF), qx);
        qx = _mm256_sub_epi8(qx, _mm256_set1_epi8(8));
        const __m256i qy = _mm256_loadu_si256((const __m256i *)y[i].qs);
        acc = _mm256_fmadd_ps(d, mul_sum_i8_pairs_float(qx, qy), acc);
    }
    *s = hsum_float_8(acc);
}

extern "C" void orc_vec_dot_q8_0_q8_0_avx2(int n, float *s, const void *vx, const void *vy) {
    const block_q8_0 *x = (const block_q8_0 *)vx;
    const block_q8_0 *y = (const block_q8_0 *)vy;
    const int nb = n / 32;
    __m256 acc = _mm256_setzero_ps();
    for (int i = 0; i < nb; ++i) {
        const __m256 d = _mm256_set1_ps(_cvtsh_ss(x[i].d) * _cvtsh_ss(y[i].d));
        const __m256i qx = _mm256_loadu_si256((const __m256i *)x[i].qs);
        const __m256i qy = _mm256_loadu_si256((const __m256i *)y[i].qs);
        acc = _mm256_fmadd_ps(d, mul_sum_i8_pairs_float(qx, qy), acc);
    }
    *s = hsum_float_8(acc);
}

extern "C" void orc_vec_dot_f16_avx2(int n, float *s, const uint16_t *x, const uint16_t *y) {
    const int np = n & ~31;
    __m256 sum[4] = {_mm256_setzero_ps(), _mm256_setzero_ps(), _mm256_setzero_ps(), _mm256_setzero_ps()};
    for (int i = 0; i < np; i += 32)
        for (int j = 0; j < 4; ++j) {
            const __m256 ax = _mm256_cvtph_ps(_mm_loadu_si128((const __m128i *)(x + i + j * 8)));
            const __m256 ay = _mm256_cvtph_ps(_mm_loadu_si128((const __m128i *)(y + i + j * 8)));
            sum[j] = _mm256_fmadd_ps(ax, ay, sum[j]);
        }
    sum[0] = _mm256_add_ps(sum[0], sum[2]);
    sum[1] = _mm256_add_ps(sum[1], sum[3]);
    sum[0] = _mm256_add_ps(sum[0], sum[1]);
    const __m128 t0 = _mm_add_ps(_mm256_castps256_ps128(sum[0]), _mm256_extractf128_ps(sum[0], 1));
    const __m128 t1 = _mm_hadd_ps(t0, t0);
    double sumf = _mm_cvtss_f32(_mm_hadd_ps(t1, t1));
    for (int i = np; i < n; ++i) sumf += (double)(_cvtsh_ss(x[i]) * _cvtsh_ss(y[i]));
    *s = (float)sumf;
}

// ---------------------------------------------------------------- float ops
// SURVEY A.5 rms_norm (src/gemma_model.cpp:438-442): sum(double) += (double)(x*x in fp32);
// mean = (float)(sum/n); scale = 1.0f/sqrtf(mean + eps); y = x*scale.
extern "C" void orc_rms_norm(const float *x, float *y, int n, float eps) {
    double sum = 0.0;
    for (int i = 0; i < n; i++) sum += (double)(x[i] * x[i]);
    const float mean = (float)(sum / n);
    const float scale = 1.0f / sqrtf(mean + eps);
    for (int i = 0; i < n; i++) y[i] = x[i] * scale;
}

// SURVEY A.6 soft_max_ext (src/gemma_model.cpp:476): w = x*scale + mask; max; e = table_exp
// [f16(w-max)] (w == -inf -> 0); sum in double; y = e * (float)(1.0/sum).
extern "C" void orc_soft_max_row(const float *x, const float *mask, float *y, int n, float scale) {
    orc_init_tables(g_gelu_clamp);
    float max = -INFINITY;
    for (int i = 0; i < n; i++) {
        y[i] = x[i] * scale;
        if (mask) y[i] += mask[i];
        max = std::max(max, y[i]);
    }
    double sum = 0.0;
    for (int i = 0; i < n; i++) {
        if (y[i] == -INFINITY) {
            y[i] = 0.0f;
        } else {
            const float val = orc_fp16_to_fp32(g_exp_f16[orc_fp32_to_fp16(y[i] - max)]);
            sum += (double)val;
            y[i] = val;
        }
    }
    sum = 1.0 / sum;
    const float v = (float)sum;
    for (int i = 0; i < n; i++) y[i] *= v;
}

// SURVEY A.8 rope NEOX (src/gemma_model.cpp:698-716, src/macro.h:12-18): theta_scale =
// powf(base, -2/n_dims); theta = (float)pos, then theta *= theta_scale after each pair;
// cos = cosf(theta), sin = sinf(theta) (ext_factor 0, freq_scale 1, attn_factor 1).
extern "C" void orc_rope_cos_sin(int pos, int n_dims, float freq_base, float *c, float *s) {
    const float theta_scale = powf(freq_base, -2.0f / n_dims);
    float theta = (float)pos;
    for (int i = 0; i < n_dims / 2; ++i) {
        c[i] = cosf(theta) * 1.0f;
        s[i] = sinf(theta) * 1.0f;
        theta *= theta_scale;
    }
}

// x: n_heads rows of n_dims floats for one position; pairs (i, i + n_dims/2).
extern "C" void orc_rope_neox(float *x, int n_dims, int n_heads, int pos, float freq_base) {
    float c[512], s[512];
    orc_rope_cos_sin(pos, n_dims, freq_base, c, s);
    for (int h = 0; h < n_heads; ++h) {
        float *r = x + (size_t)h * n_dims;
        for (int i = 0; i < n_dims / 2; ++i) {
            const float x0 = r[i], x1 = r[i + n_dims / 2];
            const float a = x0 * c[i], b = x1 * s[i];
            const float e = x0 * s[i], f = x1 * c[i];
            r[i] = a - b;
            r[i + n_dims / 2] = e + f;
        }
    }
}

// SURVEY A.7 gelu (src/gemma_model.cpp:448): y = f32(table_gelu_f16[f16(x)]); with the optional
// later-ggml clamp (x <= -10 -> 0, x >= 10 -> x) behind orc_init_tables(gelu_clamp=1).
extern "C" void orc_gelu(const float *x, float *y, int n) {
    orc_init_tables(g_gelu_clamp);
    for (int i = 0; i < n; ++i) {
        if (g_gelu_clamp && x[i] <= -10.0f) y[i] = 0.0f;
        else if (g_gelu_clamp && x[i] >= 10.0f) y[i] = x[i];
        else y[i] = orc_fp16_to_fp32(g_gelu_f16[orc_fp32_to_fp16(x[i])]);
    }
}
