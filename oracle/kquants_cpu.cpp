// kquants_cpu.cpp — ORACLE (test infrastructure only; see oracle.h): the K-quant formats on the
// reference's hot path: Q4_K and Q6_K weights against Q8_K
// activations.
//
// Restated, clean-room:
//   * block layouts: src/kernals.cl:13-34 (block_q4_K 144 B, block_q6_K 210 B, block_q8_K 292 B);
//   * the generic (scalar) dots: src/kernals.cl:48-111 (vec_dot_q4_K_q8_K) as the reference's
//     OpenCL shadow computes it — 8 int32 accumulators aux32[l] over element index l = e % 8,
//     float sums[l] += d * aux32[l] — and ggml's QK_K = 256 generic q6_K (see below);
//   * the [ext] ggml Feb–Mar 2024 CPU semantics the reference's CPU path runs on an AVX2 host
//     (called through the vec_dot pointer at src/hpc.cpp:35-36; ggml is not in /root/reference,
//     so this part is "parity unpinned"):
//       - quantize_row_q8_K (ggml INIT for K-quant src0): per 256 values amax/max, iscale =
//         -127/max, q = min(127, nearest_int(iscale*x)), bsums = 16-element sums, d = 1/iscale;
//       - AVX2 vec_dot_q4_K_q8_K: per super-block, 8 fp32 lanes, lane l = exact int32
//         Σ_j sc[2j]·dot4(lo nibbles, q8) + sc[2j+1]·dot4(hi nibbles, q8) over bytes 4l..4l+3 of
//         each 32-byte chunk j; acc_l = fmaf(y.d*f16(x.d), (float)lane_l, acc_l); the mins go to
//         4 lanes acc_m_k = fmaf(-y.d*f16(x.dmin), (float)(m[2k]·S(2k) + m[2k+1]·S(2k+1)),
//         acc_m_k) with S(s) the 32-element sums; result hsum_float_8(acc) + ((m0+m2)+(m1+m3));
//       - AVX2 vec_dot_q6_K_q8_K: lane l = Σ over 32-element chunks of sc(16-group) ·
//         Σ_{bytes 4l..4l+3} (q6 − 32)·q8; acc_l = fmaf(y.d*f16(x.d), (float)lane_l, acc_l);
//         hsum_float_8(acc).
//     Each is given twice: a portable emulation (the oracle) and an AVX2-intrinsics form that must
//     agree with it bit for bit (tests/test_oracle_kquants.py).
#include <immintrin.h>
#include <math.h>
#include <stdint.h>
#include <string.h>

#include "oracle.h"

namespace {

constexpr int QK_K = 256;

#pragma pack(push, 1)
struct block_q4_K { uint16_t d, dmin; uint8_t scales[12]; uint8_t qs[128]; };
struct block_q6_K { uint8_t ql[128]; uint8_t qh[64]; int8_t scales[16]; uint16_t d; };
struct block_q8_K { float d; int8_t qs[QK_K]; int16_t bsums[QK_K / 16]; };
#pragma pack(pop)
static_assert(sizeof(block_q4_K) == 144, "q4_K");
static_assert(sizeof(block_q6_K) == 210, "q6_K");
static_assert(sizeof(block_q8_K) == 292, "q8_K");

constexpr uint32_t kmask1 = 0x3f3f3f3f, kmask2 = 0x0f0f0f0f, kmask3 = 0x03030303;

// 12 packed bytes -> 8 six-bit scales (bytes 0..7 of utmp) and 8 six-bit mins (bytes 8..15)
// (src/kernals.cl:79-84)
void unpack_q4_K_scales(const uint8_t *packed, uint8_t sc[8], uint8_t mn[8]) {
    uint32_t utmp[4];
    memcpy(utmp, packed, 12);
    utmp[3] = ((utmp[2] >> 4) & kmask2) | (((utmp[1] >> 6) & kmask3) << 4);
    const uint32_t uaux = utmp[1] & kmask1;
    utmp[1] = (utmp[2] & kmask2) | (((utmp[0] >> 6) & kmask3) << 4);
    utmp[2] = uaux;
    utmp[0] &= kmask1;
    memcpy(sc, &utmp[0], 8);
    memcpy(mn, &utmp[2], 8);
}

inline int nearest_int(float fval) {  // ggml: round half to even through the 1.5*2^23 magic
    float val = fval + 12582912.f;
    int i;
    memcpy(&i, &val, sizeof(int));
    return (i & 0x007fffff) - 0x00400000;
}

inline float hsum8(const float a[8]) {
    const float r0 = a[0] + a[4], r1 = a[1] + a[5], r2 = a[2] + a[6], r3 = a[3] + a[7];
    return (r0 + r2) + (r1 + r3);
}

// exact int32 lane sums of one super-block (lane l = bytes 4l..4l+3 of every 32-byte chunk)
void q4_K_lanes(const block_q4_K *x, const block_q8_K *y, int32_t lanes[8], int32_t mins4[4]) {
    uint8_t sc[8], mn[8];
    unpack_q4_K_scales(x->scales, sc, mn);
    for (int l = 0; l < 8; ++l) {
        int32_t s = 0;
        for (int j = 0; j < 4; ++j) {
            int32_t lo = 0, hi = 0;
            for (int k = 0; k < 4; ++k) {
                const uint8_t b = x->qs[32 * j + 4 * l + k];
                lo += (int32_t)(b & 0xF) * y->qs[64 * j + 4 * l + k];
                hi += (int32_t)(b >> 4) * y->qs[64 * j + 32 + 4 * l + k];
            }
            s += (int32_t)sc[2 * j] * lo + (int32_t)sc[2 * j + 1] * hi;
        }
        lanes[l] = s;
    }
    for (int k = 0; k < 4; ++k) {
        const int32_t s0 = y->bsums[4 * k] + y->bsums[4 * k + 1];
        const int32_t s1 = y->bsums[4 * k + 2] + y->bsums[4 * k + 3];
        mins4[k] = (int32_t)mn[2 * k] * s0 + (int32_t)mn[2 * k + 1] * s1;
    }
}

inline int q6_value(const block_q6_K *x, int e) {  // element e (0..255) of a super-block, 0..63
    const int h = e / 128, r = e % 128, i = r / 32, t = r % 32;
    const uint8_t lq = x->ql[64 * h + 32 * (i & 1) + t];
    const int lo = (i < 2) ? (lq & 0xF) : (lq >> 4);
    const int hb = (x->qh[32 * h + t] >> (2 * i)) & 3;
    return lo | (hb << 4);
}

void q6_K_lanes(const block_q6_K *x, const block_q8_K *y, int32_t lanes[8]) {
    for (int l = 0; l < 8; ++l) {
        int32_t s = 0;
        for (int c = 0; c < 8; ++c) {  // 32-element chunks
            int32_t p = 0;
            for (int k = 0; k < 4; ++k) {
                const int e = 32 * c + 4 * l + k;
                p += (q6_value(x, e) - 32) * (int32_t)y->qs[e];
            }
            s += (int32_t)x->scales[2 * c + (l >> 2)] * p;
        }
        lanes[l] = s;
    }
}

// ---- AVX2 forms (must equal the emulation bit for bit) -------------------------------------
inline float hsum_float_8(__m256 x) {
    __m128 res = _mm256_extractf128_ps(x, 1);
    res = _mm_add_ps(res, _mm256_castps256_ps128(x));
    res = _mm_add_ps(res, _mm_movehl_ps(res, res));
    res = _mm_add_ss(res, _mm_movehdup_ps(res));
    return _mm_cvtss_f32(res);
}

}  // namespace

extern "C" void orc_quantize_row_q8_K(const float *x, void *vy, int k) {
    block_q8_K *y = (block_q8_K *)vy;
    const int nb = k / QK_K;
    for (int i = 0; i < nb; ++i, x += QK_K) {
        float max = 0, amax = 0;
        for (int j = 0; j < QK_K; ++j) {
            const float ax = fabsf(x[j]);
            if (ax > amax) {
                amax = ax;
                max = x[j];
            }
        }
        if (!amax) {
            y[i].d = 0;
            memset(y[i].qs, 0, QK_K);
            memset(y[i].bsums, 0, sizeof(y[i].bsums));
            continue;
        }
        const float iscale = -127.f / max;
        for (int j = 0; j < QK_K; ++j) {
            const int v = nearest_int(iscale * x[j]);
            y[i].qs[j] = (int8_t)(v < 127 ? v : 127);
        }
        for (int j = 0; j < QK_K / 16; ++j) {
            int sum = 0;
            for (int ii = 0; ii < 16; ++ii) sum += y[i].qs[j * 16 + ii];
            y[i].bsums[j] = (int16_t)sum;
        }
        y[i].d = 1 / iscale;
    }
}

extern "C" void orc_vec_dot_q4_K_q8_K(int n, float *s, const void *vx, const void *vy) {
    const block_q4_K *x = (const block_q4_K *)vx;
    const block_q8_K *y = (const block_q8_K *)vy;
    float acc[8] = {0, 0, 0, 0, 0, 0, 0, 0}, accm[4] = {0, 0, 0, 0};
    for (int i = 0; i < n / QK_K; ++i) {
        const float d = y[i].d * orc_fp16_to_fp32(x[i].d);
        const float dmin = -y[i].d * orc_fp16_to_fp32(x[i].dmin);
        int32_t lanes[8], mins4[4];
        q4_K_lanes(&x[i], &y[i], lanes, mins4);
        for (int k = 0; k < 4; ++k) accm[k] = fmaf(dmin, (float)mins4[k], accm[k]);
        for (int l = 0; l < 8; ++l) acc[l] = fmaf(d, (float)lanes[l], acc[l]);
    }
    *s = hsum8(acc) + ((accm[0] + accm[2]) + (accm[1] + accm[3]));
}

extern "C" void orc_vec_dot_q6_K_q8_K(int n, float *s, const void *vx, const void *vy) {
    const block_q6_K *x = (const block_q6_K *)vx;
    const block_q8_K *y = (const block_q8_K *)vy;
    float acc[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    for (int i = 0; i < n / QK_K; ++i) {
        const float d = y[i].d * orc_fp16_to_fp32(x[i].d);
        int32_t lanes[8];
        q6_K_lanes(&x[i], &y[i], lanes);
        for (int l = 0; l < 8; ++l) acc[l] = fmaf(d, (float)lanes[l], acc[l]);
    }
    *s = hsum8(acc);
}

extern "C" void orc_vec_dot_q4_K_q8_K_avx2(int n, float *s, const void *vx, const void *vy) {
    const block_q4_K *x = (const block_q4_K *)vx;
    const block_q8_K *y = (const block_q8_K *)vy;
    const __m256i m4 = _mm256_set1_epi8(0xF);
    __m256 acc = _mm256_setzero_ps();
    __m128 acc_m = _mm_setzero_ps();
    for (int i = 0; i < n / QK_K; ++i) {
        const float d = y[i].d * orc_fp16_to_fp32(x[i].d);
        const float dmin = -y[i].d * orc_fp16_to_fp32(x[i].dmin);
        uint8_t sc[8], mn[8];
        unpack_q4_K_scales(x[i].scales, sc, mn);
        // mins: 8 int16 mins x 8 int16 32-element sums, pairwise (madd) -> 4 int32 lanes
        const __m128i mins16 = _mm_cvtepu8_epi16(_mm_loadl_epi64((const __m128i *)mn));
        const __m256i q8sums = _mm256_loadu_si256((const __m256i *)y[i].bsums);
        const __m128i q8s = _mm_hadd_epi16(_mm256_extracti128_si256(q8sums, 0), _mm256_extracti128_si256(q8sums, 1));
        const __m128i prod = _mm_madd_epi16(mins16, q8s);
        acc_m = _mm_fmadd_ps(_mm_set1_ps(dmin), _mm_cvtepi32_ps(prod), acc_m);
        const uint8_t *q4 = x[i].qs;
        const int8_t *q8 = y[i].qs;
        __m256i sumi = _mm256_setzero_si256();
        for (int j = 0; j < QK_K / 64; ++j) {
            const __m256i scale_l = _mm256_set1_epi16(sc[2 * j]);
            const __m256i scale_h = _mm256_set1_epi16(sc[2 * j + 1]);
            const __m256i q4bits = _mm256_loadu_si256((const __m256i *)q4);
            q4 += 32;
            const __m256i q4l = _mm256_and_si256(q4bits, m4);
            const __m256i q4h = _mm256_and_si256(_mm256_srli_epi16(q4bits, 4), m4);
            const __m256i q8l = _mm256_loadu_si256((const __m256i *)q8);
            q8 += 32;
            __m256i p16l = _mm256_maddubs_epi16(q4l, q8l);
            p16l = _mm256_madd_epi16(scale_l, p16l);
            const __m256i q8h = _mm256_loadu_si256((const __m256i *)q8);
            q8 += 32;
            __m256i p16h = _mm256_maddubs_epi16(q4h, q8h);
            p16h = _mm256_madd_epi16(scale_h, p16h);
            sumi = _mm256_add_epi32(sumi, _mm256_add_epi32(p16l, p16h));
        }
        acc = _mm256_fmadd_ps(_mm256_set1_ps(d), _mm256_cvtepi32_ps(sumi), acc);
    }
    acc_m = _mm_add_ps(acc_m, _mm_movehl_ps(acc_m, acc_m));
    acc_m = _mm_add_ss(acc_m, _mm_movehdup_ps(acc_m));
    *s = hsum_float_8(acc) + _mm_cvtss_f32(acc_m);
}

extern "C" void orc_vec_dot_q6_K_q8_K_avx2(int n, float *s, const void *vx, const void *vy) {
    const block_q6_K *x = (const block_q6_K *)vx;
    const block_q8_K *y = (const block_q8_K *)vy;
    const __m256i m4 = _mm256_set1_epi8(0xF), m2 = _mm256_set1_epi8(3), m32s = _mm256_set1_epi8(32);
    __m256 acc = _mm256_setzero_ps();
    for (int i = 0; i < n / QK_K; ++i) {
        const float d = y[i].d * orc_fp16_to_fp32(x[i].d);
        const uint8_t *q4 = x[i].ql;
        const uint8_t *qh = x[i].qh;
        const int8_t *q8 = y[i].qs;
        __m256i sumi = _mm256_setzero_si256();
        for (int j = 0; j < QK_K / 128; ++j) {
            // 32-element chunk c uses scales 2c (bytes 0..15) and 2c+1 (bytes 16..31)
            // 32-element chunk c: int16 lanes 0..7 (bytes 0..15) use scale 2c, lanes 8..15 scale 2c+1
            auto sc16 = [&](int c) {
                const int16_t s0 = x[i].scales[2 * c], s1 = x[i].scales[2 * c + 1];
                return _mm256_set_epi16(s1, s1, s1, s1, s1, s1, s1, s1, s0, s0, s0, s0, s0, s0, s0, s0);
            };
            const int c0 = 4 * j;
            const __m256i q4bits1 = _mm256_loadu_si256((const __m256i *)q4);
            q4 += 32;
            const __m256i q4bits2 = _mm256_loadu_si256((const __m256i *)q4);
            q4 += 32;
            const __m256i q4bitsH = _mm256_loadu_si256((const __m256i *)qh);
            qh += 32;
            const __m256i q4h_0 = _mm256_slli_epi16(_mm256_and_si256(q4bitsH, m2), 4);
            const __m256i q4h_1 = _mm256_slli_epi16(_mm256_and_si256(_mm256_srli_epi16(q4bitsH, 2), m2), 4);
            const __m256i q4h_2 = _mm256_slli_epi16(_mm256_and_si256(_mm256_srli_epi16(q4bitsH, 4), m2), 4);
            const __m256i q4h_3 = _mm256_slli_epi16(_mm256_and_si256(_mm256_srli_epi16(q4bitsH, 6), m2), 4);
            const __m256i q4_0 = _mm256_or_si256(_mm256_and_si256(q4bits1, m4), q4h_0);
            const __m256i q4_1 = _mm256_or_si256(_mm256_and_si256(q4bits2, m4), q4h_1);
            const __m256i q4_2 = _mm256_or_si256(_mm256_and_si256(_mm256_srli_epi16(q4bits1, 4), m4), q4h_2);
            const __m256i q4_3 = _mm256_or_si256(_mm256_and_si256(_mm256_srli_epi16(q4bits2, 4), m4), q4h_3);
            const __m256i q8_0 = _mm256_loadu_si256((const __m256i *)q8);
            q8 += 32;
            const __m256i q8_1 = _mm256_loadu_si256((const __m256i *)q8);
            q8 += 32;
            const __m256i q8_2 = _mm256_loadu_si256((const __m256i *)q8);
            q8 += 32;
            const __m256i q8_3 = _mm256_loadu_si256((const __m256i *)q8);
            q8 += 32;
            __m256i p16_0 = _mm256_sub_epi16(_mm256_maddubs_epi16(q4_0, q8_0), _mm256_maddubs_epi16(m32s, q8_0));
            __m256i p16_1 = _mm256_sub_epi16(_mm256_maddubs_epi16(q4_1, q8_1), _mm256_maddubs_epi16(m32s, q8_1));
            __m256i p16_2 = _mm256_sub_epi16(_mm256_maddubs_epi16(q4_2, q8_2), _mm256_maddubs_epi16(m32s, q8_2));
            __m256i p16_3 = _mm256_sub_epi16(_mm256_maddubs_epi16(q4_3, q8_3), _mm256_maddubs_epi16(m32s, q8_3));
            p16_0 = _mm256_madd_epi16(sc16(c0 + 0), p16_0);
            p16_1 = _mm256_madd_epi16(sc16(c0 + 1), p16_1);
            p16_2 = _mm256_madd_epi16(sc16(c0 + 2), p16_2);
            p16_3 = _mm256_madd_epi16(sc16(c0 + 3), p16_3);
            sumi = _mm256_add_epi32(sumi, _mm256_add_epi32(p16_0, p16_1));
            sumi = _mm256_add_epi32(sumi, _mm256_add_epi32(p16_2, p16_3));
        }
        acc = _mm256_fmadd_ps(_mm256_broadcast_ss(&d), _mm256_cvtepi32_ps(sumi), acc);
    }
    *s = hsum_float_8(acc);
}

// ---- the generic (scalar) forms, restated ----------------------------------------------------
// q4_K: src/kernals.cl:48-111.  q6_K: ggml's generic QK_K = 256 loop; src/kernals.cl:127-134
// fills only the first 64 values of each super-block (the QK_K = 64 variant), the bug SURVEY §0.6
// records (−22.625 for a known answer of 32), so it is not restated as such.
extern "C" void orc_vec_dot_q4_K_q8_K_generic(int n, float *s, const void *vx, const void *vy) {
    const block_q4_K *x = (const block_q4_K *)vx;
    const block_q8_K *y = (const block_q8_K *)vy;
    float sums[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    float sumf = 0;
    for (int i = 0; i < n / QK_K; ++i) {
        int8_t aux8[QK_K];
        int8_t *a = aux8;
        const uint8_t *q4 = x[i].qs;
        for (int j = 0; j < QK_K / 64; ++j) {
            for (int l = 0; l < 32; ++l) a[l] = (int8_t)(q4[l] & 0xF);
            a += 32;
            for (int l = 0; l < 32; ++l) a[l] = (int8_t)(q4[l] >> 4);
            a += 32;
            q4 += 32;
        }
        uint8_t sc[8], mn[8];
        unpack_q4_K_scales(x[i].scales, sc, mn);
        int sumi = 0;
        for (int j = 0; j < QK_K / 16; ++j) sumi += y[i].bsums[j] * mn[j / 2];
        int32_t aux32[8] = {0, 0, 0, 0, 0, 0, 0, 0};
        const int8_t *q8 = y[i].qs;
        a = aux8;
        for (int j = 0; j < QK_K / 32; ++j) {
            const int32_t scale = sc[j];
            for (int q = 0; q < 4; ++q) {
                for (int l = 0; l < 8; ++l) aux32[l] += scale * (int16_t)(q8[l] * a[l]);
                q8 += 8;
                a += 8;
            }
        }
        const float d = orc_fp16_to_fp32(x[i].d) * y[i].d;
        for (int l = 0; l < 8; ++l) sums[l] += d * aux32[l];
        const float dmin = orc_fp16_to_fp32(x[i].dmin) * y[i].d;
        sumf -= dmin * sumi;
    }
    for (int l = 0; l < 8; ++l) sumf += sums[l];
    *s = sumf;
}

extern "C" void orc_vec_dot_q6_K_q8_K_generic(int n, float *s, const void *vx, const void *vy) {
    const block_q6_K *x = (const block_q6_K *)vx;
    const block_q8_K *y = (const block_q8_K *)vy;
    float sums[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    float sumf = 0;
    for (int i = 0; i < n / QK_K; ++i) {
        int8_t aux8[QK_K];
        int8_t *a = aux8;
        const uint8_t *q4 = x[i].ql;
        const uint8_t *qh = x[i].qh;
        for (int j = 0; j < QK_K; j += 128) {
            for (int l = 0; l < 32; ++l) {
                a[l + 0] = (int8_t)((q4[l + 0] & 0xF) | (((qh[l] >> 0) & 3) << 4)) - 32;
                a[l + 32] = (int8_t)((q4[l + 32] & 0xF) | (((qh[l] >> 2) & 3) << 4)) - 32;
                a[l + 64] = (int8_t)((q4[l + 0] >> 4) | (((qh[l] >> 4) & 3) << 4)) - 32;
                a[l + 96] = (int8_t)((q4[l + 32] >> 4) | (((qh[l] >> 6) & 3) << 4)) - 32;
            }
            a += 128;
            q4 += 64;
            qh += 32;
        }
        int32_t aux32[8] = {0, 0, 0, 0, 0, 0, 0, 0};
        const int8_t *q8 = y[i].qs;
        a = aux8;
        for (int j = 0; j < QK_K / 16; ++j) {
            const int scale = x[i].scales[j];
            for (int q = 0; q < 2; ++q) {
                for (int l = 0; l < 8; ++l) aux32[l] += scale * (int16_t)(q8[l] * a[l]);
                q8 += 8;
                a += 8;
            }
        }
        const float d = orc_fp16_to_fp32(x[i].d) * y[i].d;
        for (int l = 0; l < 8; ++l) sums[l] += d * aux32[l];
    }
    for (int l = 0; l < 8; ++l) sumf += sums[l];
    *s = sumf;
}

// ---- synthetic K-quant weights: random valid blocks (seeded; the quantizer is not on the path) ----
static uint64_t sm64(uint64_t &st) {
    uint64_t z = (st += 0x9E3779B97F4A7C15ull);
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}

extern "C" void orc_synth_kquant(int type, uint64_t seed, int64_t rows, int64_t k, void *out) {
    uint64_t st = seed * 0x2545F4914F6CDD1Dull + (uint64_t)type;
    const int64_t nb = k / QK_K;
    for (int64_t b = 0; b < rows * nb; ++b) {
        if (type == ORC_Q4_K) {
            block_q4_K *x = (block_q4_K *)out + b;
            // d in [1e-3, 4e-3), dmin in [0, 2e-3): positive fp16 normals
            x->d = orc_fp32_to_fp16(1e-3f + 3e-3f * (float)(sm64(st) % 1000) / 1000.f);
            x->dmin = orc_fp32_to_fp16(2e-3f * (float)(sm64(st) % 1000) / 1000.f);
            for (int i = 0; i < 12; ++i) x->scales[i] = (uint8_t)sm64(st);
            for (int i = 0; i < 128; ++i) x->qs[i] = (uint8_t)sm64(st);
        } else {
            block_q6_K *x = (block_q6_K *)out + b;
            for (int i = 0; i < 128; ++i) x->ql[i] = (uint8_t)sm64(st);
            for (int i = 0; i < 64; ++i) x->qh[i] = (uint8_t)sm64(st);
            for (int i = 0; i < 16; ++i) x->scales[i] = (int8_t)(sm64(st) % 255) - 127 + 0;
            x->d = orc_fp32_to_fp16(2e-4f + 6e-4f * (float)(sm64(st) % 1000) / 1000.f);
        }
    }
}

// ggml dequantize_row_q4_K / dequantize_row_q6_K [ext] (get_rows on a K-quant token_embd, as a
// llama.cpp Q4_K_M / Q4_0 Gemma file stores it).  Q4_K, per 64 values j: d1 = d*sc[2j],
// m1 = dmin*m[2j] -> y = d1*(low nibble) - m1, then d2, m2 for the high nibbles.  Q6_K, per 128
// values: y = d*sc[is]*(q6 - 32), left to right.  ⚠ Q4_K's `d1*q - m1` is restated WITHOUT FMA
// contraction (ISO C evaluation, this oracle's -ffp-contract=off policy); a ggml build that
// contracts it would differ in the last bit of some embedding values (parity unpinned, §7).
extern "C" void orc_dequantize_row_q4_K(const void *vx, float *y, int k) {
    const block_q4_K *x = (const block_q4_K *)vx;
    for (int i = 0; i < k / QK_K; ++i) {
        const float d = orc_fp16_to_fp32(x[i].d), mn = orc_fp16_to_fp32(x[i].dmin);
        uint8_t sc[8], m[8];
        unpack_q4_K_scales(x[i].scales, sc, m);
        const uint8_t *q = x[i].qs;
        for (int j = 0; j < 4; ++j) {
            const float d1 = d * (float)sc[2 * j], m1 = mn * (float)m[2 * j];
            const float d2 = d * (float)sc[2 * j + 1], m2 = mn * (float)m[2 * j + 1];
            for (int l = 0; l < 32; ++l) *y++ = d1 * (float)(q[l] & 0xF) - m1;
            for (int l = 0; l < 32; ++l) *y++ = d2 * (float)(q[l] >> 4) - m2;
            q += 32;
        }
    }
}

extern "C" void orc_dequantize_row_q6_K(const void *vx, float *y, int k) {
    const block_q6_K *x = (const block_q6_K *)vx;
    for (int i = 0; i < k / QK_K; ++i) {
        const float d = orc_fp16_to_fp32(x[i].d);
        const uint8_t *ql = x[i].ql, *qh = x[i].qh;
        const int8_t *sc = x[i].scales;
        for (int n = 0; n < QK_K; n += 128) {
            for (int l = 0; l < 32; ++l) {
                const int is = l / 16;
                const int q1 = (int)((ql[l] & 0xF) | (((qh[l] >> 0) & 3) << 4)) - 32;
                const int q2 = (int)((ql[l + 32] & 0xF) | (((qh[l] >> 2) & 3) << 4)) - 32;
                const int q3 = (int)((ql[l] >> 4) | (((qh[l] >> 4) & 3) << 4)) - 32;
                const int q4 = (int)((ql[l + 32] >> 4) | (((qh[l] >> 6) & 3) << 4)) - 32;
                y[l + 0] = d * (float)sc[is + 0] * (float)q1;
                y[l + 32] = d * (float)sc[is + 2] * (float)q2;
                y[l + 64] = d * (float)sc[is + 4] * (float)q3;
                y[l + 96] = d * (float)sc[is + 6] * (float)q4;
            }
            y += 128;
            ql += 64;
            qh += 32;
            sc += 8;
        }
    }
}
