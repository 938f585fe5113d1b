"""Multi-rank control flow of the row-split decode stream (BASELINE north star:
"partitioned across the 8 GPUs of one node by row-splitting the weight matrices with an RCCL
all-gather").  The reference splits every `mul_mat` by output rows across its workers
(src/hpc.cpp:245-269); here each rank (one process per GPU) owns a contiguous row shard of every
weight matrix and the engine all-gathers the shards over RCCL inside its hipGraph.

This module is the host-side coordination around those engines, over a gloo process group (CPU
tensors, so a test can drive it with world_size 2 on a machine without GPUs):

  new_rccl_id   rank 0 makes an RCCL unique id, every rank receives the same bytes (an id serves ONE
                communicator: its bootstrap root leaves once every rank has joined)
  share_plan    every rank runs the launch-plan tuner in lockstep — its trial schedule is fixed (the
                same decode steps, hence the same collectives, on every rank, whatever the timings),
                then rank 0's plan is broadcast and set everywhere, so all ranks run one plan
  check_parity  rank 0's UNSPLIT engine gives a sha1 per logits row; every rank compares the rows of
                its split engine; the mismatch count is summed over ranks and any mismatch raises
                ParityError (the leg's process exits 3)
  timed_steps   warmup, barrier + device sync, exactly K steps, device sync + barrier, max over ranks
  layouts       the engine's row-split layouts (0: every matrix split, 4 all-gathers per layer;
                TP_REP_ATTN: the attention block whole on every rank, 2 per layer) are each checked
                and timed in lockstep; the faster (by the max-over-ranks time every rank holds) is
                the stream's rate, the other is reported beside it

The engine is injected (`make_engine(tp)`), so tests/test_tp_control.py runs this exact code with a
stub engine on the CPU (gloo world 2, including a forced mismatch that must exit 3)."""
import hashlib
import time

import numpy as np

PLAN_CLASSES = ("qkv", "attn_out", "gate_up", "down", "logits")
EXIT_PARITY = 3
TP_REP_ATTN, TP_P2P = 1, 2  # include/gemma_hpc.h GEMMA_TP_REP_ATTN / GEMMA_TP_P2P
LAYOUT_NAMES = {0: "split", TP_REP_ATTN: "rep_attn", TP_P2P: "p2p", TP_P2P | TP_REP_ATTN: "p2p_rep_attn"}


def _mk(make_engine, tp, flags):
    """make_engine(tp) for the plain split (the stub engines' signature), (tp, flags) otherwise"""
    return make_engine(tp) if not flags else make_engine(tp, flags)


def make_split(comm, make_engine, make_id, flags, tp=None):
    """This rank's split engine of layout `flags`, made in lockstep on every rank.  RCCL layouts:
    a fresh id per communicator.  P2P layouts (an experimental transport): the engine is made, its
    inbox handle exchanged and the peers mapped only if that worked on EVERY rank; otherwise every
    rank returns None (the candidate is skipped, never fatal)."""
    if not flags & TP_P2P:
        return _mk(make_engine, tp or (comm.world, comm.rank, new_rccl_id(comm, make_id)), flags)
    e, ok = None, True
    try:
        e = _mk(make_engine, (comm.world, comm.rank, None), flags)
    except Exception:
        ok = False
    if comm.sum_int(0 if ok else 1):
        if e is not None:
            e.close()
        return None
    try:
        mine = e.p2p_handle()
    except Exception:
        mine, ok = b"", False
    handles = [comm.bcast_bytes(mine if r == comm.rank else b"", 64, src=r) for r in range(comm.world)]
    try:
        if ok and all(handles):
            e.p2p_open(handles)
        else:
            ok = False
    except Exception:
        ok = False
    if comm.sum_int(0 if ok else 1):
        comm.barrier()
        e.close()
        return None
    comm.barrier()  # every rank has mapped its peers before any rank pushes
    return e


class ParityError(RuntimeError):
    """the row-split logits differ from the unsplit engine's on some rank"""


class Comm:
    """The job's host-side group: torch.distributed (gloo) when world > 1, trivial otherwise."""

    def __init__(self, world=1, rank=0, dist=None):
        self.world, self.rank, self.dist = world, rank, dist
        if world > 1 and dist is None:
            raise ValueError("world > 1 needs an initialised torch.distributed module")

    @classmethod
    def from_env(cls, backend="gloo"):
        """RANK / WORLD_SIZE / MASTER_* from the environment (torch.distributed.run)."""
        import os
        world = int(os.environ.get("WORLD_SIZE", "1"))
        rank = int(os.environ.get("RANK", "0"))
        if world == 1:
            return cls()
        import torch.distributed as dist
        dist.init_process_group(backend=backend, init_method="env://")
        return cls(world, rank, dist)

    def close(self):
        if self.dist is not None:
            self.dist.barrier()
            self.dist.destroy_process_group()
            self.dist = None

    def barrier(self):
        if self.dist is not None:
            self.dist.barrier()

    def bcast_bytes(self, raw, n, src=0):
        """rank src's `raw` (at most n bytes) on every rank"""
        if self.dist is None:
            return bytes(raw)
        import torch
        t = torch.zeros(n + 4, dtype=torch.uint8)
        if self.rank == src:
            if len(raw) > n:
                raise ValueError(f"broadcast payload {len(raw)} > {n} bytes")
            t[:4] = torch.tensor(list(len(raw).to_bytes(4, "little")), dtype=torch.uint8)
            t[4:4 + len(raw)] = torch.tensor(list(raw), dtype=torch.uint8)
        self.dist.broadcast(t, src)
        b = bytes(t.numpy())
        return b[4:4 + int.from_bytes(b[:4], "little")]

    def bcast_ints(self, vals, n):
        """rank 0's list of n ints on every rank"""
        if self.dist is None:
            return [int(v) for v in vals]
        import torch
        t = torch.zeros(n, dtype=torch.int64)
        if self.rank == 0:
            t[:] = torch.tensor([int(v) for v in vals], dtype=torch.int64)
        self.dist.broadcast(t, 0)
        return [int(v) for v in t.tolist()]

    def sum_int(self, v):
        if self.dist is None:
            return int(v)
        import torch
        t = torch.tensor([int(v)], dtype=torch.int64)
        self.dist.all_reduce(t, op=self.dist.ReduceOp.SUM)
        return int(t.item())

    def max_float(self, v):
        if self.dist is None:
            return float(v)
        import torch
        t = torch.tensor([float(v)], dtype=torch.float64)
        self.dist.all_reduce(t, op=self.dist.ReduceOp.MAX)
        return float(t.item())


def new_rccl_id(comm, make_id):
    """A fresh RCCL unique id for one communicator: rank 0 calls make_id(), all ranks get its bytes."""
    return comm.bcast_bytes(make_id() if comm.rank == 0 else b"", 256)


def open_p2p(comm, engine):
    """GEMMA_TP_P2P engines: every rank's inbox arena handle to every rank (rank order), each rank
    maps its peers' arenas, then a barrier, so no rank pushes before every peer has mapped."""
    mine = engine.p2p_handle()
    handles = [comm.bcast_bytes(mine if r == comm.rank else b"", len(mine), src=r) for r in range(comm.world)]
    engine.p2p_open(handles)
    comm.barrier()


def plan_to_ints(plan):
    flat = []
    for k in PLAN_CLASSES:
        v = list(plan[k])
        flat += v + [0] * (3 - len(v))
    flat.append(int(plan.get("attention", 0)))
    return flat


def ints_to_plan(flat):
    p = {k: tuple(flat[3 * i:3 * i + 3]) for i, k in enumerate(PLAN_CLASSES)}
    p["attention"] = flat[15]
    return p


def share_plan(comm, engine, tune, iters):
    """Tune on every rank in lockstep (fixed trial schedule), then run rank 0's plan everywhere."""
    plan = engine.tune(iters) if tune else engine.plan()
    flat = comm.bcast_ints(plan_to_ints(plan) if comm.rank == 0 else [0] * 16, 16)
    plan0 = ints_to_plan(flat)
    engine.set_plan(plan0)
    return plan0


def row_hashes(lg):
    """8 bytes of sha1 per logits row (every bit of every logit)"""
    return np.frombuffer(b"".join(hashlib.sha1(np.ascontiguousarray(r).tobytes()).digest()[:8] for r in lg),
                         dtype=np.uint8).copy()


def mismatched_rows(ref, got):
    n = len(ref) // 8
    return int(np.any(np.asarray(got).reshape(n, 8) != np.asarray(ref).reshape(n, 8), axis=1).sum())


def reference_hashes(comm, make_engine, prompt, n_check):
    """rank 0: the unsplit engine's logits hashes for n_check rows (the prompt rows teacher-forced,
    then greedy rows) and the smallest relative top-1/top-2 margin; broadcast to every rank."""
    info = {}
    raw = b""
    if comm.rank == 0:
        ref = make_engine(None)
        try:
            ref.begin(prompt)
            lg = ref.step(n_check, want_logits=True, use_graph=True)
            raw = row_hashes(lg).tobytes()
            top2 = np.sort(lg, axis=1)[:, -2:]
            info["margin"] = float(np.min((top2[:, 1] - top2[:, 0]) / np.maximum(np.abs(top2[:, 1]), 1e-30)))
            info["tokens"] = [int(t) for t in ref.tokens()[len(prompt):len(prompt) + 8]]
        finally:
            ref.close()
    return np.frombuffer(comm.bcast_bytes(raw, 8 * n_check), dtype=np.uint8), info


def check_parity(comm, make_engine, make_id, prompt, n_check, ref, layouts=(0,)):
    """Every rank's split engine(s) against the reference hashes; raises ParityError on any mismatch
    of an RCCL layout (after every rank has counted, so all ranks raise together).  World 1: 8
    virtual ranks and a 1-rank RCCL communicator; world N: the N RCCL ranks.  Each layout in
    `layouts` wherever the engine has more than one rank (a 1-rank engine has a single layout).
    A P2P layout that cannot be made, times out or mismatches is dropped (returned in `dropped`
    with the reason), not fatal.  Returns (splits checked, layouts that passed, dropped)."""
    base = [(comm.world, comm.rank, "rccl")] if comm.world > 1 else [(8, 0, None), (1, 0, "rccl")]
    splits = [(sp, f) for f in layouts for sp in base if f == 0 or sp[0] > 1]
    nbad, passed, dropped = 0, [], {}
    for split, flags in splits:
        if flags & TP_P2P:
            ce = make_split(comm, make_engine, make_id, flags)
            if ce is None:
                dropped[LAYOUT_NAMES.get(flags, flags)] = "engine or peer mapping failed on some rank"
                continue
            bad = 0
            try:
                ce.begin(prompt)
                bad = mismatched_rows(ref, row_hashes(ce.step(n_check, want_logits=True, use_graph=True)))
                bad += n_check if ce.p2p_err() else 0
            except Exception:
                bad = n_check
            comm.barrier()
            ce.close()
            total = comm.sum_int(bad)
            if total:
                dropped[LAYOUT_NAMES.get(flags, flags)] = f"{total} mismatched or timed-out rows over all ranks"
            elif flags not in passed:
                passed.append(flags)
            continue
        if split[2] == "rccl":
            split = (split[0], split[1], new_rccl_id(comm, make_id))
        ce = _mk(make_engine, split, flags)
        try:
            ce.begin(prompt)
            nbad += mismatched_rows(ref, row_hashes(ce.step(n_check, want_logits=True, use_graph=True)))
        finally:
            ce.close()
        if flags not in passed:
            passed.append(flags)
    total = comm.sum_int(nbad)
    if total:
        raise ParityError(f"row-split logits differ from the unsplit engine: {total} rows over all ranks")
    return splits, passed, dropped


def timed_steps(comm, engine, steps, device_sync):
    """barrier + device sync, exactly `steps` decode steps, device sync + barrier; max over ranks (s)"""
    device_sync()
    comm.barrier()
    t0 = time.perf_counter()
    engine.step(steps, use_graph=True)
    engine.sync()
    device_sync()
    comm.barrier()
    return comm.max_float(time.perf_counter() - t0)


def run_stream(comm, make_engine, make_id, prompt, steps, warmup, tune=True, tune_iters=6,
               check_prompt=None, n_check=20, device_sync=lambda: None, unsplit_rate=True, kernel_iters=0,
               layouts=(0,)):
    """The whole row-split leg: parity of every rank against the unsplit engine, one timed stream
    row-split over comm.world ranks per layout (the faster is the result), and (rank 0) the unsplit
    1-GPU rate beside it.  Returns a dict (meaningful on rank 0); raises ParityError on a mismatch."""
    check_prompt = prompt[:16] if check_prompt is None else check_prompt
    layouts = tuple(layouts) if comm.world > 1 else (0,)  # one rank: one layout
    ref, info = reference_hashes(comm, make_engine, check_prompt, n_check)
    checked, layouts, dropped = check_parity(comm, make_engine, make_id, check_prompt, n_check, ref, layouts)

    tok_s_1, plan_1 = None, None
    if unsplit_rate and comm.rank == 0:  # the same treatment (tuned or not) as the split engine
        ue = make_engine(None)
        try:
            plan_1 = ue.tune(tune_iters) if tune else ue.plan()
            ue.begin(prompt)
            ue.step(len(prompt) + warmup, use_graph=True)
            ue.sync()
            t1 = time.perf_counter()
            ue.step(steps, use_graph=True)
            ue.sync()
            tok_s_1 = steps / (time.perf_counter() - t1)
        finally:
            ue.close()

    runs = {}
    for flags in layouts:  # every rank runs the same layouts in the same order (lockstep)
        te = make_split(comm, make_engine, make_id, flags)
        if te is None:
            dropped[LAYOUT_NAMES.get(flags, flags)] = "engine or peer mapping failed on some rank (timed run)"
            continue
        try:
            plan = share_plan(comm, te, tune, tune_iters)
            te.begin(prompt)
            te.step(len(prompt) + warmup, use_graph=True)  # the prompt token by token, then W warmup steps
            dt = timed_steps(comm, te, steps, device_sync)
            toks = [int(t) for t in te.tokens()]
            kern = {}
            for k in range(5 if kernel_iters > 0 else 0):
                try:
                    us, algo = te.time_kernel(k, kernel_iters)
                    kern[k] = (us, algo)
                except Exception:  # reported as missing, never fatal
                    pass
            bad = comm.sum_int(1 if (flags & TP_P2P and te.p2p_err()) else 0)
        finally:
            comm.barrier()
            te.close()
        if bad:
            dropped[LAYOUT_NAMES.get(flags, flags)] = "a flag wait timed out in the timed run"
            continue
        runs[flags] = (dt, plan, toks, kern)
    if not runs:
        raise ParityError(f"no row-split layout passed: {dropped}")
    best = min(runs, key=lambda f: runs[f][0])  # dt is the max over ranks: every rank picks the same
    dt, plan, toks, kern = runs[best]
    tok_s = steps / dt
    out = {"ranks": comm.world, "tok_s": tok_s, "ms_per_token": dt / steps * 1e3, "steps": steps, "warmup": warmup,
           "timed_s": dt, "tok_s_unsplit_1gpu": tok_s_1, "launch_plan": plan, "launch_plan_unsplit": plan_1,
           "tokens": toks, "kernels": kern, "layout": LAYOUT_NAMES.get(best, best),
           "layouts_tok_s": {LAYOUT_NAMES.get(f, f): steps / runs[f][0] for f in runs},
           "layouts_dropped": dropped,
           "parity_check": {"rows": n_check, "mismatched_rows_all_ranks": 0,
                            "reference": "unsplit 1-GPU engine (rank 0), logits sha1 per row",
                            "split_checked": (f"{comm.world} ranks, layouts "
                                              f"{[LAYOUT_NAMES.get(f, f) for f in layouts]}") if comm.world > 1
                            else "8 virtual ranks + the 1-rank RCCL engine",
                            "min_top1_top2_rel_margin": info.get("margin"),
                            "tokens_unsplit": info.get("tokens"), "splits": len(checked)}}
    return out
