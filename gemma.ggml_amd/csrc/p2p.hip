// Peer-to-peer all-gather of the row-split engine (GEMMA_TP_P2P): every rank PUSHES
// its shard straight into each peer's inbox (device memory of that peer, mapped into this process
// by hipIpcOpenMemHandle), signals the peer with one flag word, and copies the peers' shards out of
// its own inbox once their flags arrive — one kernel per gather, no RCCL.  The reference's counterpart
// is the row split of mul_mat over its workers (src/hpc.cpp:245-269); it has no multi-GPU path.
//
// Memory: each rank's arena (inboxes for every gathered vector + a flag word per source rank) is
// allocated UNCACHED (hipDeviceMallocUncached): a peer's stores land in this rank's HBM behind the
// back of its L2s, so nothing here may be served from a stale L2 line; the working buffers the
// matvecs read stay ordinary device memory (written by this kernel's copy-out, read by later
// kernels on the same device).  Order per gather, per peer p (one workgroup each):
//   push my shard -> p's inbox [rank*shard, +shard) ; every thread's system-scope release ;
//   barrier ; one flag store (system scope) p.flag[rank] = s ;
//   poll my flag[p] >= s (bounded; a timeout sets the sticky error word and goes on) ; acquire ;
//   copy my inbox [p*shard, +shard) -> work[p*shard, +shard).
// s = the engine's gather sequence + 1: every rank runs the same gathers in the same order, so the
// sequences agree; the last workgroup to finish advances it (all have read it before they count).
// A sender can be at most one gather ahead of a receiver (its next push waits for the receiver's
// push of that gather, which follows the receiver's copy-out of this one), and consecutive gathers
// use different inboxes, so a push never overwrites an inbox that is still being copied out.
#include "common.h"
#include "kernels.h"

namespace ghip {
namespace {

constexpr int P2P_NTH = 256;
constexpr long long P2P_SPIN = 1ll << 22;  // polls before the timeout (s_sleep between polls: ~0.5 s)

template <bool V16>
__device__ __forceinline__ void p2p_copy(uint8_t *dst, const uint8_t *src, int64_t bytes, int tid) {
    if (V16) {
        for (int64_t i = (int64_t)tid * 16; i < bytes; i += P2P_NTH * 16) *(uint4 *)(dst + i) = *(const uint4 *)(src + i);
    } else {
        for (int64_t i = (int64_t)tid * 4; i < bytes; i += P2P_NTH * 4) *(uint32_t *)(dst + i) = *(const uint32_t *)(src + i);
    }
}

__global__ void __launch_bounds__(P2P_NTH) k_p2p_gather(p2p_args a) {
    const int tid = threadIdx.x;
    const int p = (a.rank + 1 + (int)blockIdx.x) % a.n;  // this workgroup's peer
    const unsigned s = a.seq[0] + 1u;
    // 1) push every segment's shard into the peer's inbox
    for (int g = 0; g < a.nseg; ++g) {
        const p2p_seg &sg = a.seg[g];
        const uint8_t *src = sg.work + (int64_t)a.rank * sg.shard;
        uint8_t *dst = a.peer[p] + sg.inbox + (int64_t)a.rank * sg.shard;
        if (sg.shard % 16 == 0) p2p_copy<true>(dst, src, sg.shard, tid);
        else p2p_copy<false>(dst, src, sg.shard, tid);
    }
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "");  // system scope: the pushed bytes before the flag
    __syncthreads();
    if (tid == 0) {
        unsigned *flag = (unsigned *)(a.peer[p] + a.flags) + a.rank;
        __hip_atomic_store(flag, s, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        // 2) the peer's flag in my arena (after a timeout the engine's results are void: no more
        // waiting, so a dead peer costs one timeout, not one per gather)
        const unsigned *mine = (const unsigned *)(a.peer[a.rank] + a.flags) + p;
        long long spin = __hip_atomic_load(a.err, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) ? P2P_SPIN : 0;
        while (spin <= P2P_SPIN && (int)(__hip_atomic_load(mine, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) - s) < 0) {
            if (++spin > P2P_SPIN) {
                __hip_atomic_store(a.err, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                break;
            }
            __builtin_amdgcn_s_sleep(2);
        }
    }
    __syncthreads();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "");
    // 3) the peer's shards out of my inbox into the working vectors
    for (int g = 0; g < a.nseg; ++g) {
        const p2p_seg &sg = a.seg[g];
        const uint8_t *src = a.peer[a.rank] + sg.inbox + (int64_t)p * sg.shard;
        uint8_t *dst = sg.work + (int64_t)p * sg.shard;
        if (sg.shard % 16 == 0) p2p_copy<true>(dst, src, sg.shard, tid);
        else p2p_copy<false>(dst, src, sg.shard, tid);
    }
    // 4) the last workgroup advances the sequence (every workgroup read it before counting)
    __syncthreads();
    if (tid == 0) {
        const unsigned prev = __hip_atomic_fetch_add(&a.seq[1], 1u, __ATOMIC_ACQ_REL, __HIP_MEMORY_SCOPE_AGENT);
        if (prev == (unsigned)(a.n - 2)) {
            __hip_atomic_store(&a.seq[1], 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            __hip_atomic_store(&a.seq[0], s, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
    }
}

}  // namespace

int launch_p2p_gather(const p2p_args &a, hipStream_t s) {
    if (a.n < 2 || a.n > P2P_MAX_RANKS || a.rank < 0 || a.rank >= a.n || a.nseg < 1 || a.nseg > 2 || !a.seq || !a.err) {
        set_error("p2p_gather: bad arguments");
        return -1;
    }
    for (int g = 0; g < a.nseg; ++g)
        if (a.seg[g].shard <= 0 || a.seg[g].shard % 4 || a.seg[g].inbox % 16 || !a.seg[g].work) {
            set_error("p2p_gather: segments need 4-byte multiples and 16-byte aligned inboxes");
            return -1;
        }
    for (int r = 0; r < a.n; ++r)
        if (!a.peer[r]) {
            set_error("p2p_gather: peer arenas not opened (gemma_engine_p2p_open)");
            return -1;
        }
    hipLaunchKernelGGL(k_p2p_gather, dim3(a.n - 1), dim3(P2P_NTH), 0, s, a);
    GHIP_CHECK(hipGetLastError());
    return 0;
}

}  // namespace ghip
