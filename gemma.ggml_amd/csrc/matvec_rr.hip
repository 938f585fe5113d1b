// matvec_rr.hip — the round-pipelined K-split matvec ("rr" form, launch_matvec ks = KS_RR).
//
// Same arithmetic as k_matvec (matvec_impl.h): ggml's AVX2 lane order, one thread per AVX2 lane,
// lane l of row r runs fmaf(d_w*d_a, isum_l, acc) block after block — so results are bit-identical
// to the CPU path (src/hpc.cpp:15-41 calling ggml_vec_dot_q4_0_q8_0 / q8_0_q8_0).
//
// Why another form: at batch 1 a workgroup owns ONE 8-row tile (2048-row matrices have 256 tiles
// for 256 CUs), so its whole K range must be in flight at once and its 64 lane chains are serial
// over K.  The KS = 8 form (k_matvec) gives wave w the contiguous segment w of K and lets wave 0
// carry the chains through segments 1..7 only after ALL loads have landed: the ~450-step carry
// (~1.5 us) sits behind the stream.  Here:
//   * 8 loader waves take block tiles w, w+8, w+16, ... (K interleaved by rounds), so round r's
//     tiles 8r..8r+7 are issued together, early rounds first;
//   * loaders turn round r into exact (d, isum) terms in an LDS slot (two slots, ping-pong);
//   * a 9th wave, the carrier, runs the 64 chains through round r-1 while the loaders convert
//     round r — the chain is consumed as the data lands and ends one round after the last load.
// One s_barrier per round; no vmcnt(0) drain (loads stay in flight across the barriers).
#include "matvec_rr.h"

namespace ghip {
namespace {

template <int WT, int PRO, int EPI, int NR, int R, int DD>
__global__ void __launch_bounds__(RR_NTH) k_matvec_rr(mv_args a) {
    extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
    using G = rr_geom<WT>;
    constexpr int BT = G::BT, SB = wfmt<WT>::SCALE_BYTES;
    constexpr bool NSA = true;
    const int tid = threadIdx.x, lane = tid & 63, wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int rr = lane >> 3, l = lane & 7;
    const int col = blockIdx.y;
    const int64_t rt = blockIdx.x;
    const lds_map m = make_lds_map<WT, NSA>(1, a.n_bt, a.n_bt, 0);
    const size_t slot0 = (m.total + 15) & ~(size_t)15;
    const bool loader = wave < RR_NL;
    unsigned long long *stp = GHIP_STAMPS && a.dbg_t ? a.dbg_t + ((int64_t)blockIdx.y * gridDim.x + blockIdx.x) * 16 : nullptr;
    if (GHIP_STAMPS && stp && tid == 0) stp[0] = __builtin_amdgcn_s_memrealtime();

    // 0) the Q8_0 activation image in LDS FIRST, weights after: issued together, the activation
    //    loads queue behind the whole weight stream in the fabric (stamps: image ready at ~4 us of
    //    a 9.5 us down), and the chain cannot start before it.  Alone they return in ~1 us.
    constexpr int D = DD < NR ? DD : NR;
    uint4 qb[D], sb[D];
    const uint32_t q_off = (uint32_t)lane * 16u, s_off = (uint32_t)rr * SB;
    auto issue = [&](int r) {
        const int64_t tile = rt * a.n_bt + (loader ? wave : 0) + RR_NL * r;
        qb[r % D] = ld_nt16(a.qs + tile * 1024 + q_off);
        if (WT == T_Q4_0) {
            sb[r % D] = ld_sc16(a.sc + tile * 8 * SB + s_off);
        } else {
            const uint2 v = ld_sc8(a.sc + tile * 8 * SB + s_off);
            sb[r % D] = make_uint4(v.x, v.y, 0, 0);
        }
    };
    // (weight rounds issued before the activation, or right behind its loads, measured slower: DESIGN.md §10)
    act_regs<R> ar;
    prefetch_activation<WT, PRO, R, RR_NTH>(a, col, ar);
    norm_state ns;
    if (!(a.ablate & 1)) ns = build_activation<WT, PRO, R, NSA, RR_NTH>(a, col, smem, m, ar);  // timing ablations only
    if (GHIP_STAMPS && stp && tid == 0) stp[10] = __builtin_amdgcn_s_memrealtime();
    // 1) the rest of the ring (loader w, round r -> block tile w + 8r; D rounds in flight per wave),
    //    issued after the image is used, so these loads may sit in a loader-only branch
    if (loader) {
#pragma unroll
        for (int r = 0; r < D; ++r) issue(r);
    }
    // the norm's check (PRO_NORM / PRO_EMBED) with the weights already in flight: off the path to
    // the first weight load (measured: +0.35-0.45 us on qkv with the check in front of the issue);
    // the fallback reloads x and w, so only the ring's D rounds stay live beside it
    if (!(a.ablate & 1)) finish_activation<WT, PRO, R, NSA, RR_NTH>(a, col, smem, m, ar, ns);
    if (GHIP_STAMPS && stp && tid == 0) stp[11] = __builtin_amdgcn_s_memrealtime();
    lds_barrier();
    if (GHIP_STAMPS && stp && tid == 0) stp[1] = __builtin_amdgcn_s_memrealtime();
    // the carrier's dependent fmaf chain is the critical path: first pick of the SIMD's issue slots
    if (!loader) __builtin_amdgcn_s_setprio(3);

    // 3) rounds: loaders stash round r while the carrier chains round r-1
    float acc = 0.0f;
    auto slot_s = [&](int r) { return (float *)(smem + slot0 + (size_t)(r & 1) * G::SLOT); };
    auto slot_d = [&](int r) { return (float *)(smem + slot0 + (size_t)(r & 1) * G::SLOT + G::S_BYTES); };
    const int crow = rr;  // the carrier's lane = (row, AVX2 lane) of the loaders' numbering
    auto chain = [&](int r) {
        const float4 *pd = (const float4 *)(slot_d(r) + (size_t)crow * G::SBPD);
        const uint4 *ps = (const uint4 *)(slot_s(r) + (size_t)(crow * 8 + l) * G::SBP);
        acc = carry_ring<false>(ps, pd, G::RUN / 4, acc);  // chunks of 4 blocks: (s, d) f32 pairs
    };
#pragma unroll
    for (int r = 0; r < NR; ++r) {
        if (loader) {
            float *st = slot_s(r) + (size_t)lane * G::SBP;
            float *sd = slot_d(r) + (size_t)rr * G::SBPD;
            const uint4 q = qb[r % D], sc = sb[r % D];
            if (a.ablate & 8)  // timing only: consume the loads without the dot products
                acc += __builtin_bit_cast(float, q.x ^ sc.y);
            else
                tile_terms<WT>(q, sc, smem, m, wave + RR_NL * r, l, st, sd, wave * BT);
            if (r + D < NR) issue(r + D);
            if (GHIP_STAMPS && stp && lane == 0 && wave == 0 && r < 8) stp[2 + r] = __builtin_amdgcn_s_memrealtime();
            if (GHIP_STAMPS && stp && lane == 0 && wave == RR_NL - 1 && r == NR - 1) stp[15] = __builtin_amdgcn_s_memrealtime();
        } else if (r > 0 && !(a.ablate & 4)) {
            chain(r - 1);
            if (GHIP_STAMPS && stp && lane == 0 && wave == RR_NL && r == 6) stp[12] = __builtin_amdgcn_s_memrealtime();
        }
        lds_barrier();
    }
    if (loader && (a.ablate & 8) && acc == 1.2345f) a.y[0] = acc;  // keeps the ablated loads live
    if (!loader) {
        if (!(a.ablate & 4)) chain(NR - 1);
        if (GHIP_STAMPS && stp && lane == 0 && wave == RR_NL) stp[13] = __builtin_amdgcn_s_memrealtime();
        const float v = fold8(acc);
        unsigned long long best = 0;
        if (l == 0) epilogue<EPI>(a, col, rt * 8 + crow, v, 0.0f, best);
        if (GHIP_STAMPS && stp && lane == 0 && wave == RR_NL) stp[14] = __builtin_amdgcn_s_memrealtime();
    }
}


template <int WT, int PRO, int EPI, int NR>
int launch_rr_t(const mv_args &a, hipStream_t s) {
    constexpr int R = (PRO == PRO_F32 || PRO == PRO_NORM) && NR * wfmt<WT>::BT * 8 > 144 ? 4 : 1;
    const lds_map m = make_lds_map<WT, true>(1, a.n_bt, a.n_bt, 0);
    const size_t lds = ((m.total + 15) & ~(size_t)15) + 2 * rr_geom<WT>::SLOT;
    if (lds > 160 * 1024) {
        set_error("matvec(rr): LDS image too large");
        return -1;
    }
    if (PRO == PRO_IMG && a.nb % 4) {
        set_error("matvec(rr): PRO_IMG needs K % 128 == 0");
        return -1;
    }
    // ring depth (rounds in flight per loader wave), measured on the down shape (NR 8), rounds issued
    // after the image: all 8 at once 8.2 us, 6 8.1, 4 7.9, 2 8.2 — four keep the CU's memory queue
    // full without stalling the first round's issue.  (Rounds issued before the image: 8.4 / 8.5 vs
    // 7.95 us; the ring right behind the activation loads: decode 1,449-1,456 vs 1,513-1,517 tok/s —
    // both removed.)
    constexpr bool deep = (PRO == PRO_IMG || PRO == PRO_F32) && EPI == EPI_ADD && NR >= 8;
    // NR 16 (the Q8_0 down: 16 rounds of 8 tiles) keeps 8 rounds in flight: Q8_0 decode 1,158-1,177 vs
    // 1,209 tok/s at 8 (1,191-1,193 at 6), while the Q4_0 down (NR 8) is best at 4 (1,540-1,544 vs
    // 1,535 at 6, 1,523 at 8) — same box, interleaved; NR 12 (the Gemma-7B down) at 6: the 7B leg
    // 556.7 vs 548.8 tok/s (554 at 8)
    constexpr int DD = NR >= 16 ? 8 : NR >= 12 ? 6 : 4;
    const void *fn = deep ? (const void *)k_matvec_rr<WT, PRO, EPI, NR, R, DD> : (const void *)k_matvec_rr<WT, PRO, EPI, NR, R, 64>;
    if (lds > 64 * 1024) GHIP_CHECK(hipFuncSetAttribute(fn, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
    mv_args la = a;
    void *args[] = {(void *)&la};
    GHIP_CHECK(hipLaunchKernel(fn, dim3((unsigned)a.n_rt, a.ncols), dim3(RR_NTH), args, lds, s));
    GHIP_CHECK(hipGetLastError());
    return 0;
}

template <int WT, int NR>
int rr_pro(int pro, int epi, const mv_args &a, hipStream_t s) {
    if (pro == PRO_Q8 && epi == EPI_STORE) return launch_rr_t<WT, PRO_Q8, EPI_STORE, NR>(a, s);
    if (pro == PRO_NORM && epi == EPI_STORE) return launch_rr_t<WT, PRO_NORM, EPI_STORE, NR>(a, s);
    if (pro == PRO_EMBED && epi == EPI_STORE) return launch_rr_t<WT, PRO_EMBED, EPI_STORE, NR>(a, s);
    if (pro == PRO_F32 && epi == EPI_ADD) return launch_rr_t<WT, PRO_F32, EPI_ADD, NR>(a, s);
    if (pro == PRO_IMG && epi == EPI_ADD) return launch_rr_t<WT, PRO_IMG, EPI_ADD, NR>(a, s);
    if (pro == PRO_F32 && epi == EPI_STORE) return launch_rr_t<WT, PRO_F32, EPI_STORE, NR>(a, s);
    set_error("matvec(rr): (prologue, epilogue) combination not instantiated");
    return -1;
}

}  // namespace

// n_bt block tiles per row = 8 loaders x NR rounds; NR in {1, 2, 3, 8, 12, 16}
bool matvec_rr_supported(int wtype, int64_t n_bt) {
    if (wtype != T_Q4_0 && wtype != T_Q8_0) return false;
    if (n_bt % RR_NL) return false;
    const int64_t nr = n_bt / RR_NL;
    return nr == 1 || nr == 2 || nr == 3 || nr == 8 || nr == 12 || nr == 16;
}

int matvec_dispatch_rr(int wtype, int pro, int epi, const mv_args &a, hipStream_t s) {
    if (!matvec_rr_supported(wtype, a.n_bt)) {
        set_error("matvec(rr): block tiles per row must be 8 x {1,2,3,8,12,16}");
        return -1;
    }
    const int nr = (int)(a.n_bt / RR_NL);
#define RR_CASE(N)                                                         \
    case N:                                                                \
        return wtype == T_Q4_0 ? rr_pro<T_Q4_0, N>(pro, epi, a, s) : rr_pro<T_Q8_0, N>(pro, epi, a, s);
    switch (nr) {
        RR_CASE(1)
        RR_CASE(2)
        RR_CASE(3)
        RR_CASE(8)
        RR_CASE(12)
        RR_CASE(16)
    }
#undef RR_CASE
    return -1;
}

}  // namespace ghip
