// attn_mx.hip — the exact causal prefill attention on the f32 matrix cores.
//
// What it computes: rows i < T of the reference's prefill KQ -> soft_max_ext -> KQV
// (src/gemma_model.cpp:454-497 with T tokens; mask -inf for j > i, scale 1.0), every dot product in
// ggml's AVX/F16C vec_dot_f16 order: 32 fmaf chains per output — chain c = 8j + l
// runs over elements 32s + c, s = 0, 1, ... — folded as ((c0+c16)+(c8+c24)) per l, then halves and
// hadds.  The same arithmetic k_attn_rows runs with v_fma_mix, bit for bit.
//
// Why the matrix cores can carry it: v_mfma_f32_16x16x4_f32 computes every output as an fmaf chain
// over its 4 K terms in K order, starting from the accumulator input (measured bit for bit on
// gfx950, tests/micro/mfma_f32_layout.hip: every register of 256 random blocks equals the fmaf chain
// of its (m, n)).  f16 q / k / P / v values widen to f32 exactly.  So K = 4 consecutive STEPS of one
// chain is one MFMA: A[m][k] = q[m][32(4t + k) + c], B[k][n] = K[n][32(4t + k) + c]; the 32 chains
// are 32 accumulator tiles, folded in registers at the end (each lane holds the same (m, n) of all
// 32 tiles).  f32 MFMA runs at the f32 vector peak, 3x what v_fma_mix issues.
//
// Tile: one 512-thread workgroup per (P = 16/G query positions x the G heads of a kv head): M = 16
// rows (position, head).  KQ: wave w takes 16-position key tiles w, w+8, ...; scores of unmasked
// positions go to LDS S[16][L], L = the block's largest padded n_kv; the keys past the block's last
// row are never computed (masked: the softmax reads -inf for j > i).  Softmax per row exactly as
// k_attn_rows (fp16 exp, integer-exact sum, (float)(1/sum)), P16 written over S in place, zeros for
// [n_kv(i), L).  KQV: wave w takes 16-dim tiles; chain c's steps 4u..4u+3 are one MFMA with
// A = P16 (LDS) and B = V (the [d][ctx] cache rows); steps past a row's n_kv multiply P = 0 (exact
// no-ops: fmaf(0, v, acc) = acc), steps past L are zero operands.  hd = 256 (Gemma); other shapes
// take k_attn_rows.
#include "device_util.h"
#include "kernels.h"

namespace ghip {
namespace {

typedef float mx4 __attribute__((ext_vector_type(4)));
#ifndef GHIP_MX_ABL
#define GHIP_MX_ABL 0  // timing ablations only (wrong results): 1 K rows all row 0, 2 V rows all row 0, 4 no softmax passes,
                       // 8 no KQV, 16 no KQ
#endif
#ifndef GHIP_MX_THREADS
#define GHIP_MX_THREADS 512  // 256: 4-wave workgroups, two per CU where the scores fit 80 KB
#endif
constexpr int MX_THREADS = GHIP_MX_THREADS, MX_WAVES = MX_THREADS / 64, MX_HD = 256;

// ggml_vec_dot_f16's fold of the 32 chain values of one output (reduce_f16_acc, attn_impl.h)
__device__ __forceinline__ float fold32(const mx4 acc[32], int r) {
    float x0[8];
#pragma unroll
    for (int l = 0; l < 8; ++l) {
        const float a = acc[l][r] + acc[16 + l][r];
        const float b = acc[8 + l][r] + acc[24 + l][r];
        x0[l] = a + b;
    }
    float t0[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) t0[i] = x0[i] + x0[i + 4];
    const float h0 = t0[0] + t0[1], h1 = t0[2] + t0[3];
    return h0 + h1;
}

// 32 consecutive f16 (64 B) -> 32 f32 operands (exact widening)
__device__ __forceinline__ void widen32(const uint4 v[4], float out[32]) {
#pragma unroll
    for (int q = 0; q < 4; ++q) {
        const uint32_t w[4] = {v[q].x, v[q].y, v[q].z, v[q].w};
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            out[8 * q + 2 * k] = h2f(w[k]);
            out[8 * q + 2 * k + 1] = h2f(w[k] >> 16);
        }
    }
}

__global__ void __launch_bounds__(MX_THREADS) k_attn_mx(attnp_args a) {
    extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int G = a.H / a.Hkv, P = 16 / G, kvh = blockIdx.x % a.Hkv;
    const int nblk = (a.T + P - 1) / P;
    const int pb = nblk - 1 - (int)(blockIdx.x / a.Hkv);  // longest blocks first
    const int i0 = pb * P;
    const int kvw = a.Hkv * MX_HD;
    // this block's rows: m = p * G + g -> position i0 + p, head kvh * G + g
    const int i_last = min(i0 + P - 1, a.T - 1);
    int L = 32 * ((i_last + 1) / 32 + 1);
    if (L > a.n_kv) L = a.n_kv;
    // S [16][LS], LS = L + 4: the 16 rows of an MFMA operand read sit 16 B apart in the banks
    const int LS = L + 4;
    float *S = (float *)smem;  // P16 row m over S row m (in place)
    const int m_l = lane & 15, kk = lane >> 4;  // MFMA A row / B column, K index of this lane

    // ---- q operands: row m_l = (position, head), elements 32(4t + kk) + c, t = 0, 1 ----------
    float qf[2][32];
    {
        const int ip = i0 + m_l / G, h = kvh * G + m_l % G;
        const bool ok = ip < a.T;
        const uint16_t *qr = a.q16 + ((int64_t)(ok ? ip : 0) * a.H + h) * MX_HD;
#pragma unroll
        for (int t = 0; t < 2; ++t) {
            uint4 v[4];
#pragma unroll
            for (int q = 0; q < 4; ++q) v[q] = *(const uint4 *)(qr + 32 * (4 * t + kk) + 8 * q);
            widen32(v, qf[t]);
        }
    }
    // ---- KQ: 16-position key tiles; wave w takes tiles w, w + 8, ... ----------------------------
    const int n_keys = i_last + 1;  // positions past the block's last row are all masked
    const int n_kt = (n_keys + 15) / 16;
    // this lane's 128 B of key row kt*16 + (lane & 15); the next tile's loads are issued before
    // the current tile's MFMAs
    auto kload = [&](int kt, uint4 kv[2][4]) {
        const int j = kt * 16 + m_l;
        const uint16_t *kr = a.kc + (int64_t)((GHIP_MX_ABL & 1) ? 0 : j < n_keys ? j : 0) * kvw + (int64_t)kvh * MX_HD;
#pragma unroll
        for (int t = 0; t < 2; ++t)
#pragma unroll
            for (int q = 0; q < 4; ++q) kv[t][q] = *(const uint4 *)(kr + 32 * (4 * t + kk) + 8 * q);
    };
    uint4 kn[2][4];
    if (wave < n_kt) kload(wave, kn);
    for (int kt = wave; kt < ((GHIP_MX_ABL & 16) ? 0 : n_kt); kt += MX_WAVES) {
        uint4 kv[2][4];
#pragma unroll
        for (int t = 0; t < 2; ++t)
#pragma unroll
            for (int q = 0; q < 4; ++q) kv[t][q] = kn[t][q];
        if (kt + MX_WAVES < n_kt) kload(kt + MX_WAVES, kn);
        mx4 acc[32];
        const mx4 z = {0.0f, 0.0f, 0.0f, 0.0f};
        {
            float kf[32];
            widen32(kv[0], kf);
#pragma unroll
            for (int c = 0; c < 32; ++c) acc[c] = __builtin_amdgcn_mfma_f32_16x16x4f32(qf[0][c], kf[c], z, 0, 0, 0);
            widen32(kv[1], kf);
#pragma unroll
            for (int c = 0; c < 32; ++c) acc[c] = __builtin_amdgcn_mfma_f32_16x16x4f32(qf[1][c], kf[c], acc[c], 0, 0, 0);
        }
        // register r of this lane: row m = 4 kk + r, key position kt*16 + (lane & 15)
        const int jn = kt * 16 + m_l;
#pragma unroll
        for (int r = 0; r < 4; ++r) {
            const float kq = fold32(acc, r);
            const int m = 4 * kk + r;
            if (jn < L) S[m * LS + jn] = kq * 1.0f + 0.0f;  // ggml: kq * scale + mask (0 where unmasked)
        }
    }
    __syncthreads();
    // ---- soft_max_ext per row (k_attn_rows' arithmetic): wave w takes rows 2w, 2w + 1 ---------
    for (int m = wave; m < ((GHIP_MX_ABL & 4) ? 0 : 16); m += MX_WAVES) {
        const int ip = i0 + m / G;
        float *Sr = S + m * LS;
        uint16_t *Pr = (uint16_t *)Sr;
        if (ip >= a.T) {  // padding row of the last block: zeros (its outputs are not stored)
            for (int j = lane; j < L; j += 64) Pr[j] = 0;
            continue;
        }
        int n_kv = 32 * ((ip + 1) / 32 + 1);
        if (n_kv > a.n_kv) n_kv = a.n_kv;
        float mx = -INFINITY;
        for (int j = lane; j < n_kv; j += 64) mx = fmaxf(mx, j > ip ? -INFINITY : Sr[j]);
        mx = wave_max(mx);
        unsigned long long isum = 0;
        for (int j = lane; j < n_kv; j += 64) {
            const float w = j > ip ? -INFINITY : Sr[j];
            const float e = w != -INFINITY ? h2f(exp_f16_of(f2h(w - mx))) : 0.0f;
            isum += (unsigned long long)(uint32_t)(e * 16777216.0f);  // e * 2^24 <= 2^24: exact
        }
        const unsigned long long tot = wave_sum_u64(isum);
        const double sum = (double)tot * (1.0 / 16777216.0);
        const float inv = (float)(1.0 / sum);
        // in place: iteration u reads S[64u + lane] and writes P16[64u + lane], bytes of S[32u ..]
        // that earlier iterations (or this one, before its write) already read.  The float reads and
        // the u16 writes alias by design: the empty asm with a memory clobber keeps every write behind
        // its iteration's read whatever type-based alias analysis concludes
        for (int j = lane; j < L; j += 64) {
            float w = -INFINITY;
            if (j <= ip && j < n_kv) w = Sr[j];
            asm volatile("" ::: "memory");
            const float e = w != -INFINITY ? h2f(exp_f16_of(f2h(w - mx))) : 0.0f;
            Pr[j] = (uint16_t)f2h(e * inv);
        }
    }
    __syncthreads();
    // ---- KQV: out[m][d] = vec_dot_f16 over the row's n_kv of P16[m] and V[d]; wave w takes the
    // 16-dim tiles w, w + 8; steps 4u .. 4u + 3 of chain c are one MFMA
    const int n_sg = (L / 32 + 3) / 4;  // step groups (steps past L: zero operands)
    for (int dt = wave; dt < ((GHIP_MX_ABL & 8) ? 0 : MX_HD / 16); dt += MX_WAVES) {
        const int d = dt * 16 + m_l;  // this lane's V row (B column)
        const uint16_t *vr = a.vc + ((int64_t)kvh * MX_HD + ((GHIP_MX_ABL & 2) ? 0 : d)) * a.ctx;
        const uint16_t *pr = (const uint16_t *)(S + m_l * LS);  // A row m_l of P16
        mx4 acc[32];
#pragma unroll
        for (int c = 0; c < 32; ++c) acc[c] = (mx4){0.0f, 0.0f, 0.0f, 0.0f};
        // this lane's V step of group u (positions 32(4u + kk) ..), one group ahead of its MFMAs
        auto vload = [&](int u, uint4 vv[4]) {
            const int e0 = 32 * (4 * u + kk);
#pragma unroll
            for (int q = 0; q < 4; ++q) vv[q] = e0 < L ? *(const uint4 *)(vr + e0 + 8 * q) : make_uint4(0u, 0u, 0u, 0u);
        };
        uint4 vn[4];
        vload(0, vn);
        for (int u = 0; u < n_sg; ++u) {
            const int e0 = 32 * (4 * u + kk);  // this lane's step: positions e0 .. e0 + 31
            uint4 pv[4], vv[4];
#pragma unroll
            for (int q = 0; q < 4; ++q) vv[q] = vn[q];
            if (u + 1 < n_sg) vload(u + 1, vn);
#pragma unroll
            for (int q = 0; q < 4; ++q) pv[q] = e0 < L ? *(const uint4 *)(pr + e0 + 8 * q) : make_uint4(0u, 0u, 0u, 0u);
            float pf[32], vf[32];
            widen32(pv, pf);
            widen32(vv, vf);
#pragma unroll
            for (int c = 0; c < 32; ++c) acc[c] = __builtin_amdgcn_mfma_f32_16x16x4f32(pf[c], vf[c], acc[c], 0, 0, 0);
        }
#pragma unroll
        for (int r = 0; r < 4; ++r) {
            const int m = 4 * kk + r, ip = i0 + m / G, h = kvh * G + m % G;
            const float o = fold32(acc, r);
            if (ip < a.T) a.out[(int64_t)ip * a.ldo + (int64_t)h * MX_HD + dt * 16 + m_l] = o;
        }
    }
}

}  // namespace

// nullptr when the matrix-core form runs these shapes, else why not (the engine then runs k_attn_rows)
const char *attn_mx_unsupported(const attnp_args &a) {
    if (a.hd != MX_HD) return "head_dim != 256";
    if (a.Hkv <= 0 || a.H % a.Hkv) return "heads";
    const int G = a.H / a.Hkv;
    if (G > 16 || 16 % G) return "query heads per kv head must divide 16";
    if (a.ctx % 32 || a.n_kv % 32 || a.n_kv > a.ctx || a.T <= 0 || a.T > a.n_kv) return "context";
    int L = 32 * (a.T / 32 + 1);  // the last row's padded n_kv
    if (L > a.n_kv) L = a.n_kv;
    if ((size_t)16 * (L + 4) * 4 > 160 * 1024) return "scores of 16 rows exceed the LDS (n_kv > 2556)";
    return nullptr;
}

int launch_attn_mx(const attnp_args &a, hipStream_t s) {
    if (const char *why = attn_mx_unsupported(a)) {
        set_error(std::string("attn_mx: ") + why);
        return -1;
    }
    const int G = a.H / a.Hkv, P = 16 / G;
    int L = 32 * (a.T / 32 + 1);
    if (L > a.n_kv) L = a.n_kv;
    const size_t lds = (size_t)16 * (L + 4) * 4;
    if (allow_full_lds((const void *)k_attn_mx, LDS_SLOT_ATTN_MX)) return -1;
    const int nblk = (a.T + P - 1) / P;
    hipLaunchKernelGGL(k_attn_mx, dim3((unsigned)(nblk * a.Hkv)), dim3(MX_THREADS), lds, s, a);
    GHIP_CHECK(hipGetLastError());
    return 0;
}

}  // namespace ghip
