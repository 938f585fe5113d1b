// matvec_rr.h — pieces of the round-pipelined matvec (matvec_rr.hip) shared with the fused
// layer-front kernel (layer_front.hip): geometry, the exact-term stash, the LDS barrier.
#pragma once

#include "matvec_impl.h"

namespace ghip {
namespace {

constexpr int RR_NL = 8;                  // loader waves
constexpr int RR_NTH = 64 * (RR_NL + 1);  // + the carrier wave

// LDS barrier that does not drain the wave's outstanding global loads: LDS stores complete
// (lgkmcnt), then s_barrier.  (__syncthreads() would also wait for every in-flight load.)
__device__ __forceinline__ void lds_barrier() { asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory"); }

// stash slot geometry: per lane a run of the round's 8*BT terms (s), per row 8*BT d values.
// Lane stride 144 B (36 dwords): the 16-B stores of 8 lanes and the b128 reads of 16 lanes hit
// distinct banks; row stride of d 8*BT+4 floats.  A slot ends with slack for the carry ring's
// over-reads (up to 4 chunks past a run).
template <int WT> struct rr_geom {
    static constexpr int BT = wfmt<WT>::BT;
    static constexpr int RUN = 8 * BT;                      // blocks per round
    static constexpr int SBP = RUN + 4;                     // s stride (f32): 272 B (Q4_0) / 144 B (Q8_0), = 4 dwords mod 32
    static constexpr int SBPD = RUN + 4;                    // d stride (f32)
    static constexpr size_t S_BYTES = 64 * SBP * 4 + 256;
    static constexpr size_t D_BYTES = 8 * SBPD * 4 + 256;
    static constexpr size_t SLOT = S_BYTES + D_BYTES;
};

// exact (d, (float)isum) terms of one tile for this thread's (row, lane): the operands of the BT
// fmaf steps tile_dot<WT, false> would apply, stored for the carrier (s as f32: the carrier's
// chain is then LDS reads + fmaf only)
template <int WT>
__device__ __forceinline__ void tile_terms(uint4 q, uint4 scv, const uint8_t *smem, const lds_map &m, int64_t bt, int l,
                                           float *st_s, float *st_d, int j0) {
    const act_tile<WT> t = load_act<WT, true>(smem, m, bt, l);
    const uint32_t qv[4] = {q.x, q.y, q.z, q.w};
    if constexpr (WT == T_Q4_0) {
        const uint32_t sv[4] = {scv.x, scv.y, scv.z, scv.w};
        float dd[8], ss[8];
#pragma unroll
        for (int p = 0; p < 4; ++p) {
            const uint32_t lo = qv[p] & 0x0F0F0F0Fu, hi = (qv[p] >> 4) & 0x0F0F0F0Fu;
            ss[2 * p] = (float)sdot4(lo, t.av[2 * p], (int)t.nv[2 * p]);
            ss[2 * p + 1] = (float)sdot4(hi, t.av[2 * p + 1], (int)t.nv[2 * p + 1]);
            dd[2 * p] = mix_lo(sv[p], t.dav[2 * p]);
            dd[2 * p + 1] = mix_hi(sv[p], t.dav[2 * p + 1]);
        }
        *(float4 *)(st_s + j0) = make_float4(ss[0], ss[1], ss[2], ss[3]);
        *(float4 *)(st_s + j0 + 4) = make_float4(ss[4], ss[5], ss[6], ss[7]);
        if (l == 0) {
            *(float4 *)(st_d + j0) = make_float4(dd[0], dd[1], dd[2], dd[3]);
            *(float4 *)(st_d + j0 + 4) = make_float4(dd[4], dd[5], dd[6], dd[7]);
        }
    } else {
        const uint32_t sv[2] = {scv.x, scv.y};
        float dd[4], ss[4];
#pragma unroll
        for (int p = 0; p < 4; ++p) {
            ss[p] = (float)sdot4(qv[p], t.av[p], 0);
            dd[p] = (p & 1) ? mix_hi(sv[p >> 1], t.dav[p]) : mix_lo(sv[p >> 1], t.dav[p]);
        }
        *(float4 *)(st_s + j0) = make_float4(ss[0], ss[1], ss[2], ss[3]);
        if (l == 0) *(float4 *)(st_d + j0) = make_float4(dd[0], dd[1], dd[2], dd[3]);
    }
}

}  // namespace
}  // namespace ghip
