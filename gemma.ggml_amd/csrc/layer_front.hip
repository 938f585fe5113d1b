// layer_front.hip — the front half of a decode layer in ONE launch: qkv matvec -> attention ->
// attn-out (+ residual).  Replaces three dependent launches of the reference's per-token graph
// (src/gemma_model.cpp:692-723: rms_norm*w -> Wq|Wk|Wv -> rope -> KQ -> soft_max_ext -> KQV ->
// Wo -> + inpL) with in-launch hand-offs, same arithmetic and bits as the separate kernels.
//
// Roles by workgroup index wg (one workgroup of 576 threads = 8 loader waves + 1 carrier, as the
// round-pipelined matvec, matvec_rr.hip):
//   * wg < qkv row tiles:           one 8-row tile of q|k|v (rr form, PRO_NORM), rows stored sc1;
//                                   then one lane adds to counter shard wg % 8;
//   * wg < H (also a qkv tile):     after all qkv shards are complete, the attention of query head
//                                   wg (attn_impl.h, sc1 loads of q|k|v), its output's Q8_0 image
//                                   stored sc1; one lane adds to the attention counter;
//   * H <= wg < H + attn-out tiles: the attn-out tile wg - H: its Wo weights are issued BEFORE
//                                   waiting for the attention counter (the HBM stream overlaps the
//                                   wait), then the image (sc1 loads), rr rounds, + residual.
// Hand-off protocol (MI355X_MICROARCH §inter-workgroup visibility, sc1 table row 1): every handed-off
// byte is stored and loaded with sc1 accesses; each storing wave drains vmcnt before the workgroup
// barrier; one lane then adds to the (sharded) counter; the consumer polls with sc1 loads and joins
// a workgroup barrier before any of its sc1 loads.  Counters are zeroed by a memset node before
// the token's first layer.  Every poll is bounded: on timeout the sticky error word is set and the
// kernel finishes (wrong numbers, never a hung GPU).  Waiters only wait on lower phases, and the
// grid (<= 3 workgroups per CU) is resident at once.
#include <algorithm>

#include "attn_impl.h"
#include "matvec_rr.h"

namespace ghip {
namespace {

constexpr int LF_NTH = 1024;  // 16 waves: 8 loaders + 1 carrier in the matvec phases, all 16 in attention
constexpr int LF_CS = 32;     // counter stride (u32): every counter on its own 128-B line
constexpr int LF_NREP = 8;    // replicas of the attention counter (one per poller group)
constexpr int LF_POLL = 1 << 22;  // ~0.2 s of s_sleep(2) polls

typedef __attribute__((address_space(1))) unsigned gu32_t;
__device__ __forceinline__ unsigned ld_sc1_cnt(const unsigned *p) {
    return __hip_atomic_load((const gu32_t *)p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ void add_cnt(unsigned *p) {
    __hip_atomic_fetch_add((gu32_t *)p, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
// one lane: wait until cnt[s] >= tgt(s) for the n shards.  err[0] sticky timeout flag, err[1] the
// poll site, err[2] / err[3] the counter value / target at the timeout, err[4] max polls seen
template <typename Tgt>
__device__ void poll_counters(const unsigned *cnt, int n, Tgt tgt, int *err, int site) {
    unsigned most = 0;
    for (int s = 0; s < n; ++s) {
        unsigned it = 0, v;
        while ((v = ld_sc1_cnt(cnt + s)) < tgt(s)) {
            __builtin_amdgcn_s_sleep(4);
            if (++it > (unsigned)LF_POLL) {
                __hip_atomic_store((gu32_t *)err + 1, (unsigned)site, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                __hip_atomic_store((gu32_t *)err + 2, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                __hip_atomic_store((gu32_t *)err + 3, (unsigned)tgt(s), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                __hip_atomic_store((gu32_t *)err, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                return;
            }
        }
        most = it > most ? it : most;
    }
    __hip_atomic_fetch_max((gu32_t *)err + 4, most, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
// every wave's stores drained, then one lane signals for the workgroup
__device__ __forceinline__ void signal_after_stores(unsigned *cnt) {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (threadIdx.x == 0) add_cnt(cnt);
}

// One or two row tiles (rt1 < 0: one) of the round-pipelined matvec (k_matvec_rr, K = 8 block
// tiles: one round per row tile) inside the fused launch.  The activation image is built once;
// round r covers row tile r and the carrier stores each tile's rows after chaining its round.
//   WAIT = false: image first (prologue from f32 x), then the weights; rows stored sc1 (EPI_STORE).
//   WAIT = true:  weights first, then wait for `wcnt` >= wtarget, then the image from the handed-off
//                 Q8_0 image (sc1 loads), EPI_ADD with plain stores (consumed after the launch).
// Both tiles' weights are always issued (a missing second tile re-reads the first: L2 hits) so the
// compiler's counted waits stay exact.
struct no_hook {
    __device__ void operator()() const {}
};
// one 16-B load through to the handed-off bytes (sc1: past this CU's L1), waited for here
__device__ __forceinline__ uint4 ld_sc1_16(const void *p) {
    uint4 v;
    asm volatile("global_load_dwordx4 %0, %1, off sc1\n\ts_waitcnt vmcnt(0)" : "=v"(v) : "v"(p) : "memory");
    return v;
}
// on_poll: run by thread 0 right after its poll matched (before the workgroup's barrier)
template <int WT, int PRO, int EPI, bool WAIT, typename Hook = no_hook>
__device__ void rr_tiles(const mv_args &a, int64_t rt0, int64_t rt1, uint8_t *smem, const unsigned *wcnt,
                         unsigned wtarget, int *err, unsigned long long *stp = nullptr, Hook on_poll = Hook()) {
#define RT_STAMP(i) \
    if (GHIP_STAMPS && stp && threadIdx.x == 0) stp[i] = __builtin_amdgcn_s_memrealtime()
    using G = rr_geom<WT>;
    constexpr int BT = G::BT, SB = wfmt<WT>::SCALE_BYTES, R = 1;
    constexpr bool NSA = true;
    const int tid = threadIdx.x, lane = tid & 63, wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int rr = lane >> 3, l = lane & 7;
    const lds_map m = make_lds_map<WT, NSA>(1, a.n_bt, a.n_bt, 0);
    const size_t slot0 = (m.total + 15) & ~(size_t)15;
    const bool loader = wave < RR_NL;
    const int nt = rt1 >= 0 ? 2 : 1;
    act_regs<R> ar;
    norm_state ns;
    if (!WAIT) {
        prefetch_activation<WT, PRO, R, LF_NTH>(a, 0, ar);
        ns = build_activation<WT, PRO, R, NSA, LF_NTH>(a, 0, smem, m, ar);
        finish_activation<WT, PRO, R, NSA, LF_NTH>(a, 0, smem, m, ar, ns);  // the norm's check
    }
    uint4 qb[2], sb[2];
    const uint32_t q_off = (uint32_t)lane * 16u, s_off = (uint32_t)rr * SB;
    if (loader) {
#pragma unroll
        for (int r = 0; r < 2; ++r) {
            const int64_t tile = (r == 0 || rt1 < 0 ? rt0 : rt1) * a.n_bt + wave;
            qb[r] = ld_nt16(a.qs + tile * 1024 + q_off);
            if (WT == T_Q4_0) {
                sb[r] = ld_sc16(a.sc + tile * 8 * SB + s_off);
            } else {
                const uint2 v = ld_sc8(a.sc + tile * 8 * SB + s_off);
                sb[r] = make_uint4(v.x, v.y, 0, 0);
            }
        }
    }
    if (WAIT) {
        static_assert(!WAIT || PRO == PRO_IMG, "the handed-off activation is a Q8_0 image");
        RT_STAMP(1);
        if (tid == 0) {
            poll_counters(wcnt, 1, [&](int) { return wtarget; }, err, 2);
            on_poll();
        }
        __syncthreads();
        RT_STAMP(2);
        // the image: one 16-B sc1 load per item, only by the threads that own an item (build_activation
        // stores items < T only; clamped duplicates were 8x the loads on one line)
        const int64_t T = a.nb * 2 + a.nb / 4;  // image items (host: T <= 2 * LF_NTH)
#pragma unroll
        for (int i = 0; i < 2 * R; ++i) {
            const int64_t it = tid + (int64_t)i * LF_NTH;
            float *dst = (i & 1) ? &ar.w[i >> 1][0] : &ar.x[i >> 1][0];
            if (it < T) {
                const uint4 v = ld_sc1_16(img_item(a, it));
                dst[0] = __builtin_bit_cast(float, v.x); dst[1] = __builtin_bit_cast(float, v.y);
                dst[2] = __builtin_bit_cast(float, v.z); dst[3] = __builtin_bit_cast(float, v.w);
            }
        }
        build_activation<WT, PRO, R, NSA, LF_NTH>(a, 0, smem, m, ar);  // PRO_IMG: no norm
    }
    lds_barrier();
    RT_STAMP(3);
    if (wave == RR_NL) __builtin_amdgcn_s_setprio(3);
    auto slot_s = [&](int r) { return (float *)(smem + slot0 + (size_t)(r & 1) * G::SLOT); };
    auto slot_d = [&](int r) { return (float *)(smem + slot0 + (size_t)(r & 1) * G::SLOT + G::S_BYTES); };
    auto finish = [&](int r) {  // carrier: chain row tile r's round and store its rows
        const float4 *pd = (const float4 *)(slot_d(r) + (size_t)rr * G::SBPD);
        const uint4 *ps = (const uint4 *)(slot_s(r) + (size_t)lane * G::SBP);
        const float v = fold8(carry_ring<false>(ps, pd, G::RUN / 4, 0.0f));
        const int64_t row = (r == 0 ? rt0 : rt1) * 8 + rr;
        if (l == 0 && row < a.rows) {
            if (EPI == EPI_STORE) st_sc1(a.y + row, v);       // handed off inside this launch
            if (EPI == EPI_ADD) a.y[row] = v + a.resid[row];  // consumed after the launch
        }
    };
    if (loader) {
        tile_terms<WT>(qb[0], sb[0], smem, m, wave, l, slot_s(0) + (size_t)lane * G::SBP, slot_d(0) + (size_t)rr * G::SBPD,
                       wave * BT);
        if (nt == 2) {
            lds_barrier();
            tile_terms<WT>(qb[1], sb[1], smem, m, wave, l, slot_s(1) + (size_t)lane * G::SBP,
                           slot_d(1) + (size_t)rr * G::SBPD, wave * BT);
        }
        lds_barrier();
    } else {  // the carrier (wave RR_NL) chains; waves past it only keep the barrier count
        const bool carrier = wave == RR_NL;
        lds_barrier();
        if (carrier) finish(0);
        if (nt == 2) {
            lds_barrier();
            if (carrier) finish(1);
        }
        __builtin_amdgcn_s_setprio(0);
    }
    RT_STAMP(4);
#undef RT_STAMP
}

// Workgroup roles over a grid of G = one workgroup per CU (every workgroup resident: the waiters
// never hold a CU another producer needs): qkv row tile w, plus tile w + (nq - G) for the last
// nq - G workgroups; attention of head w for w < H; attn-out tile w - H for w >= H, plus tile
// w - H + (G - H) for the first no - (G - H) of them.
template <int WT>
__global__ void __launch_bounds__(LF_NTH) k_layer_front(front_args f) {
    extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
    const int w = blockIdx.x, G = gridDim.x;
    const int nq = (int)f.q.n_rt, no = (int)f.o.n_rt, H = f.t.H;
    const int xq = nq - G, xo = no - (G - H);
    unsigned long long *stp = GHIP_STAMPS && f.dbg_t ? f.dbg_t + (int64_t)w * 16 : nullptr;
#define LF_STAMP(i) \
    if (GHIP_STAMPS && stp && threadIdx.x == 0) stp[i] = __builtin_amdgcn_s_memrealtime()
    LF_STAMP(0);
    rr_tiles<WT, PRO_NORM, EPI_STORE, false>(f.q, w, w >= G - xq ? w + xq : -1, smem, nullptr, 0, f.err);
    LF_STAMP(1);
    signal_after_stores(f.cnt + (w & 7) * LF_CS);
    LF_STAMP(2);
    if (w < H) {
        // the first pass's K / V rows in flight while the other workgroups finish q|k|v
        attn_pre<8, 8> pre;
        attn_prefetch<LF_NTH, 8, 8>(f.t, w, pre);
        if (threadIdx.x < 64) {  // lane s polls shard s (G workgroups, w % 8 sharded)
            const int sh = threadIdx.x & 7;
            const unsigned tgt = (unsigned)((G - sh + 7) / 8);
            for (int it = 0;; ++it) {
                const bool ok = ld_sc1_cnt(f.cnt + sh * LF_CS) >= tgt;
                if (__builtin_amdgcn_read_exec() == __builtin_amdgcn_ballot_w64(ok)) break;
                if (it > LF_POLL) {
                    if (threadIdx.x == 0) __hip_atomic_store((gu32_t *)f.err, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                    break;
                }
                __builtin_amdgcn_s_sleep(1);
            }
        }
        __syncthreads();
        LF_STAMP(3);
        attn_head_dev<LF_NTH, true, 8, 8, true>(f.t, w, smem, &pre);
        LF_STAMP(4);
        // every replica of the attention counter, one lane each (one wave instruction)
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __syncthreads();
        if (threadIdx.x < LF_NREP) add_cnt(f.cnt + (8 + threadIdx.x) * LF_CS);
        LF_STAMP(5);
    } else {
        __syncthreads();  // the qkv phase's LDS is dead for every wave
        rr_tiles<WT, PRO_IMG, EPI_ADD, true>(f.o, w - H, w - H < xo ? w - H + (G - H) : -1, smem,
                                             f.cnt + (8 + (w & (LF_NREP - 1))) * LF_CS, (unsigned)H, f.err);
        LF_STAMP(6);
    }
#undef LF_STAMP
}

// ---- attention + attn-out in ONE launch (the decode step's K2 + K3; src/gemma_model.cpp:454-497,
// :723) ------------------------------------------------------------------------------------------
// The per-head attention launch has 8*H*S workgroups of which only one in eight works: the G*S
// workgroups of a kv head share one XCD (its L2 serves their K / V rows), the other seven of every
// octet return at once.  Here those seven run attn-out's row tiles (rr_tiles: weights issued first,
// then the wait, then the attention's Q8_0 image by sc1 loads, rr rounds, + residual), so attn-out's
// weight stream and launch ramp overlap the attention instead of following it, and one kernel
// boundary per layer disappears.  Same operands, same fmaf chains: bit-identical to the two launches.
// Hand-off (MI355X_MICROARCH sc1 table row 1): each attention workgroup stores its image blocks sc1,
// drains vmcnt, barriers, then adds 1 to each of the 8 counter replicas; consumer c polls replica
// c % 8 for H*S.  Reset without a memset node: every consumer adds 1 to `done` after its poll, and
// the one that completes it subtracts the targets (order-free: a replica increment still in flight
// nets to zero; nobody polls any more).  Dispatch: the attention workgroups of a kv head have the
// lowest block index of their XCD's share and never wait, so the waiters cannot starve them; the
// launcher caps the grid at one workgroup per CU.
constexpr int AO_DONE = LF_NREP;  // counter slot of the consumers' done count
template <int WT>
__global__ void __launch_bounds__(LF_NTH) k_attn_o(attn_o_args f) {
    extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
    const int b = blockIdx.x, S = f.t.dsplit, H = f.t.H, G = H / f.t.Hkv;
    const int hs = b >> 3, h = hs / S, sp = hs % S, att = (h / G) & 7, j = b & 7;
    unsigned long long *stp = GHIP_STAMPS && f.dbg_t ? f.dbg_t + (int64_t)b * 16 : nullptr;
    if (GHIP_STAMPS && stp && threadIdx.x == 0) stp[0] = __builtin_amdgcn_s_memrealtime();
    if (j == att) {  // the attention of (head h, dims split sp), exactly k_attn_head's body
        attn_head_dev<AH_THREADS, false, AH_KPF, AH_VPF, false, true>(f.t, h, smem, nullptr, sp);
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // this wave's image stores have landed
        __syncthreads();
        if (threadIdx.x < LF_NREP) add_cnt(f.cnt + threadIdx.x * LF_CS);
        if (GHIP_STAMPS && stp && threadIdx.x == 0) stp[5] = __builtin_amdgcn_s_memrealtime();
        return;
    }
    const int nc = (int)(gridDim.x >> 3) * 7;        // consumers (launcher: nc <= n_rt <= 2 nc)
    const int c = hs * 7 + (j < att ? j : j - 1);   // this consumer's index
    const int no = (int)f.o.n_rt, P = H * S;
    // the done count right behind the poll (its returned add and the resets overlap this
    // workgroup's image and rounds instead of trailing the launch)
    auto done = [&] {
        const unsigned old = __hip_atomic_fetch_add((gu32_t *)(f.cnt + AO_DONE * LF_CS), 1u, __ATOMIC_RELAXED,
                                                    __HIP_MEMORY_SCOPE_AGENT);
        if (old == (unsigned)nc - 1) {  // every consumer is past its poll: return the counters to zero
            for (int r = 0; r < LF_NREP; ++r)
                __hip_atomic_fetch_sub((gu32_t *)(f.cnt + r * LF_CS), (unsigned)P, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            __hip_atomic_fetch_sub((gu32_t *)(f.cnt + AO_DONE * LF_CS), (unsigned)nc, __ATOMIC_RELAXED,
                                   __HIP_MEMORY_SCOPE_AGENT);
        }
    };
    rr_tiles<WT, PRO_IMG, EPI_ADD, true>(f.o, c, c + nc < no ? c + nc : -1, smem, f.cnt + (c & (LF_NREP - 1)) * LF_CS,
                                         (unsigned)P, f.err, stp, done);
}

}  // namespace

static int cu_count() {
    static int n_cu = 0;
    if (!n_cu) {
        int dev = 0;
        hipDeviceProp_t prop;
        if (hipGetDevice(&dev) == hipSuccess && hipGetDeviceProperties(&prop, dev) == hipSuccess) n_cu = prop.multiProcessorCount;
    }
    return n_cu;
}

// the grid: one workgroup per CU, and the role arithmetic of k_layer_front must close
static bool front_grid_ok(int G, const mv_args &q, const attn_args &t, const mv_args &o) {
    const int64_t nq = q.n_rt, no = o.n_rt, H = t.H;
    return G >= 8 && nq >= G && nq - G <= G - H && no >= G - H && no - (G - H) <= G - H && H < G;
}

bool layer_front_supported(int wtype, const mv_args &q, const attn_args &t, const mv_args &o) {
    if (wtype != T_Q4_0 && wtype != T_Q8_0) return false;
    const int64_t nbt = wtype == T_Q4_0 ? 8 : 4;
    // one rr round per row tile (K = 8 block tiles), image items of attn-out within 2 per thread
    if (q.n_bt != 8 || o.n_bt != 8 || q.nb != 8 * nbt || o.nb != 8 * nbt) return false;
    if (o.nb % 4 || o.nb * 2 + o.nb / 4 > 2 * LF_NTH) return false;
    if (t.mode != ATTN_PER_HEAD || t.hd % 32 || t.hd > 256 || t.ctx % 32 || t.H % t.Hkv || !t.out_act || !t.rope_cur) return false;
    return front_grid_ok(cu_count(), q, t, o);
}

int launch_layer_front(int wtype, const front_args &f, hipStream_t s) {
    if (!layer_front_supported(wtype, f.q, f.t, f.o) || !f.cnt || !f.err) {
        set_error("layer_front: unsupported shape");
        return -1;
    }
    const size_t lds_mv = ((make_lds_map<T_Q4_0, true>(1, 8, 8, 0).total + 15) & ~(size_t)15) +
                          2 * (wtype == T_Q4_0 ? rr_geom<T_Q4_0>::SLOT : rr_geom<T_Q8_0>::SLOT);
    const size_t lds_mv8 = ((make_lds_map<T_Q8_0, true>(1, 8, 8, 0).total + 15) & ~(size_t)15) + 2 * rr_geom<T_Q8_0>::SLOT;
    const size_t lds_att = ((2 * (size_t)f.t.hd * 2 + 15) & ~(size_t)15) + (size_t)f.t.ctx * 6 + 16;
    size_t lds = wtype == T_Q4_0 ? lds_mv : lds_mv8;
    if (lds_att > lds) lds = lds_att;
    if (lds > 160 * 1024) {
        set_error("layer_front: LDS image too large");
        return -1;
    }
    const int grid = cu_count();
    const void *fn = wtype == T_Q4_0 ? (const void *)k_layer_front<T_Q4_0> : (const void *)k_layer_front<T_Q8_0>;
    if (lds > 64 * 1024) GHIP_CHECK(hipFuncSetAttribute(fn, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
    front_args la = f;
    void *args[] = {(void *)&la};
    GHIP_CHECK(hipLaunchKernel(fn, dim3(grid), dim3(LF_NTH), args, lds, s));
    return 0;
}

}  // namespace ghip

namespace ghip {

bool attn_o_supported(int wtype, const attn_args &t, const mv_args &o) {
    if (wtype != T_Q4_0 && wtype != T_Q8_0) return false;
    const int64_t nbt = wtype == T_Q4_0 ? 8 : 4;
    // rr_tiles: one round per row tile (K = 8 block tiles), the image within 2 items per thread
    if (o.n_bt != 8 || o.nb != 8 * nbt || o.nb % 4 || o.nb * 2 + o.nb / 4 > 2 * LF_NTH) return false;
    if (t.mode != ATTN_PER_HEAD || !t.out_act || !t.out_da || !t.rope_cur || t.out_q8k) return false;
    if (t.hd % 32 || t.hd > 256 || t.ctx % 32 || t.H % t.Hkv || t.dsplit < 1 || t.hd % (32 * t.dsplit) ||
        4 * (t.hd / t.dsplit) > AH_THREADS)
        return false;
    // one workgroup per CU for the whole grid (nobody waits for a CU), every consumer 1 or 2 tiles
    const int64_t grid = 8LL * t.H * t.dsplit, nc = grid / 8 * 7;
    return grid <= cu_count() && o.n_rt >= nc && o.n_rt <= 2 * nc;
}

int launch_attn_o(int wtype, const attn_o_args &f, hipStream_t s) {
    if (!attn_o_supported(wtype, f.t, f.o) || !f.cnt || !f.err) {
        set_error("attn_o: unsupported shape");
        return -1;
    }
    const size_t lds_mv = wtype == T_Q4_0
                              ? ((make_lds_map<T_Q4_0, true>(1, 8, 8, 0).total + 15) & ~(size_t)15) + 2 * rr_geom<T_Q4_0>::SLOT
                              : ((make_lds_map<T_Q8_0, true>(1, 8, 8, 0).total + 15) & ~(size_t)15) + 2 * rr_geom<T_Q8_0>::SLOT;
    const size_t lds_att = ((2 * (size_t)f.t.hd * 2 + 15) & ~(size_t)15) + (size_t)f.t.ctx * 6 + 16;
    const size_t lds = lds_mv > lds_att ? lds_mv : lds_att;
    if (lds > 160 * 1024) {
        set_error("attn_o: context too long for the LDS image");
        return -1;
    }
    const void *fn = wtype == T_Q4_0 ? (const void *)k_attn_o<T_Q4_0> : (const void *)k_attn_o<T_Q8_0>;
    if (lds > 64 * 1024) GHIP_CHECK(hipFuncSetAttribute(fn, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
    attn_o_args la = f;
    void *args[] = {(void *)&la};
    GHIP_CHECK(hipLaunchKernel(fn, dim3(8 * f.t.H * f.t.dsplit), dim3(LF_NTH), args, lds, s));
    return 0;
}

}  // namespace ghip
