"""CPU, world_size 2 over gloo: the multi-rank control flow of the row-split decode leg
(scripts/tp_leg.py -> gemma_tp.run_stream) driven end to end with a stub engine.

The stub stands in for the HIP engine: a split engine (tp = (N, rank, id)) runs one gloo all-reduce
per decode step, as the real engine runs its RCCL all-gathers, so ranks whose step counts diverge
(tuning, parity, warmup or timed steps out of lockstep) would hang the test instead of passing.
Checked: the RCCL id is made once by rank 0 per communicator and every rank receives the same bytes;
every rank runs rank 0's tuned plan; the unsplit-engine hash check passes on equal logits; a forced
one-row mismatch on rank 1 makes BOTH ranks exit 3 with rank 0 printing the error object; rank 0's
JSON line carries the max-over-ranks time; both row-split layouts (every matrix split / the attention
block replicated) are checked and timed in the same order on every rank, and the faster is the line's
rate."""
import contextlib
import io
import json
import os
import socket
import sys
import time

import numpy as np
import torch.distributed as dist
import torch.multiprocessing as mp

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
V = 64


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


class StubEngine:
    log = []

    def __init__(self, tp, comm, corrupt, flags=0):
        self.tp, self.comm, self.corrupt, self.flags = tp, comm, corrupt, flags
        self.split = tp is not None and (tp[0] > 1 or tp[2] is not None)
        assert not (flags & 2) or (tp is not None and tp[2] is None), "p2p engines take no RCCL id"
        self.rccl = tp is not None and tp[2] is not None
        self._plan = {k: (1, 1, 0) for k in ("qkv", "attn_out", "gate_up", "down", "logits")}
        self._plan["attention"] = 0
        self.toks = []
        StubEngine.log.append(("create", None if tp is None else (tp[0], tp[1], bytes(tp[2]) if tp[2] else None), flags))

    def _collective(self):  # the real engine's all-gathers (RCCL or p2p): every rank must take part
        if (self.rccl or self.flags & 2) and self.comm.world > 1:
            self.comm.sum_int(1)

    def begin(self, prompt):
        self.toks = list(prompt)
        self.pos = 0

    def _row(self, pos):
        rng = np.random.default_rng(int(self.toks[pos]) * 1000003 + pos)
        return rng.standard_normal(V).astype(np.float32)

    def step(self, n, want_logits=False, use_graph=True):
        out = np.zeros((n, V), dtype=np.float32) if want_logits else None
        if n == 5 and self.tp and self.tp[1] == 1:  # rank 1 is the slow one in the timed region
            time.sleep({0: 0.3, 1: 0.15, 2: 0.25, 3: 0.2}[self.flags])  # (the replicated-attention layout "fastest")
        for i in range(n):
            self._collective()
            lg = self._row(self.pos)
            if self.corrupt and self.split and i == 3 and (self.corrupt != "p2p" or self.flags & 2):
                lg[7] = np.nextafter(lg[7], np.float32(np.inf))  # one ulp on one logit of one row
            if want_logits:
                out[i] = lg
            self.pos += 1
            if self.pos >= len(self.toks):
                self.toks.append(int(np.argmax(lg)))
        return out

    def tune(self, iters):
        for _ in range(iters):  # trial steps with collectives, a fixed schedule on every rank
            self._collective()
        # ranks "measure" different winners; run_stream must install rank 0's everywhere
        self._plan["gate_up"] = (1, 1 + (self.tp[1] if self.tp else 0), 0)
        return self.plan()

    def plan(self):
        return dict(self._plan)

    def set_plan(self, plan):
        self._plan = dict(plan)
        StubEngine.log.append(("set_plan", tuple(plan["gate_up"])))

    def sync(self):
        pass

    def p2p_handle(self):  # the GEMMA_TP_P2P engine's inbox handle
        return bytes([0x50, self.tp[1]]) * 32

    def p2p_open(self, handles):
        StubEngine.log.append(("p2p_open", tuple(h[1] for h in handles)))

    def p2p_err(self):
        return 0

    def tokens(self):
        return np.array(self.toks, dtype=np.int32)

    def time_kernel(self, k, iters):
        return 10.0 + k, 1.0e6

    def close(self):
        pass


def _work(rank, world, port, corrupt, q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    sys.path.insert(0, os.path.join(ROOT, "gemma.ggml_amd", "python"))
    sys.path.insert(0, os.path.join(ROOT, "scripts"))
    sys.path.insert(0, ROOT)
    import gemma_tp as T
    import tp_leg
    dist.init_process_group("gloo", rank=rank, world_size=world)
    comm = T.Comm(world, rank, dist)
    made = []

    def make_id():
        made.append(rank)
        return bytes([0xA5, rank + 1]) * 64

    buf = io.StringIO()
    with contextlib.redirect_stdout(buf):
        rc = tp_leg.main(["5", "q4_0", "1", "2b", "3", "8"],
                         make_engine=lambda tp, flags=0: StubEngine(tp, comm, corrupt if rank == 1 else False, flags),
                         make_id=make_id, comm=comm)
    q.put((rank, rc, buf.getvalue(), made, StubEngine.log))


def _worker(rank, world, port, corrupt, q):
    try:
        _work(rank, world, port, corrupt, q)
    except Exception as ex:  # report instead of hanging the parent
        q.put((rank, -1, repr(ex), [], []))


def _run(corrupt):
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, corrupt, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = {}
    for _ in range(world):
        r = q.get(timeout=120)
        res[r[0]] = r[1:]
    for p in procs:
        p.join(timeout=60)
    return res


def test_tp_leg_control_flow_world2():
    res = _run(corrupt=False)
    assert res[0][0] == 0 and res[1][0] == 0, res
    line = json.loads(res[0][1].strip().splitlines()[-1])
    assert line["ranks"] == 2 and line["steps"] == 5 and line["warmup"] == 3
    assert line["parity_check"]["mismatched_rows_all_ranks"] == 0
    assert line["launch_plan"]["gate_up"] == [1, 1, 0] or tuple(line["launch_plan"]["gate_up"]) == (1, 1, 0)
    assert "roofline" in line and line["roofline"]["kernel"]
    # the max over ranks (rank 1 slept in the timed region), of the faster layout
    assert 0.15 <= line["timed_s"] < 0.3
    assert line["layout"] == "rep_attn"
    assert set(line["layouts_tok_s"]) == {"split", "rep_attn", "p2p", "p2p_rep_attn"} and not line["layouts_dropped"]
    assert line["layouts_tok_s"]["rep_attn"] > line["layouts_tok_s"]["split"]
    assert res[1][1] == ""  # only rank 0 prints
    # ids: made on rank 0 only (one per communicator: a parity and a timed engine per layout), same
    # bytes everywhere
    assert res[0][2] == [0, 0, 0, 0] and res[1][2] == []
    for r in (0, 1):  # split engines in the same layout order on every rank (RCCL ones with an id)
        assert [e[2] for e in res[r][3] if e[0] == "create" and e[1] and e[1][2]] == [0, 1, 0, 1]
        assert [e[2] for e in res[r][3] if e[0] == "create" and e[1] and e[1][0] == 2] == [0, 1, 2, 3, 0, 1, 2, 3]
        # p2p engines: every rank's handle, in rank order, once per p2p engine
        assert [e[1] for e in res[r][3] if e[0] == "p2p_open"] == [(0, 1)] * 4
    ids = [[e[1][2] for e in res[r][3] if e[0] == "create" and e[1] and e[1][2]] for r in (0, 1)]
    assert ids[0] == ids[1] and len(ids[0]) == 4 and ids[0][0] == bytes([0xA5, 1]) * 64
    # every rank installed rank 0's plan (rank 1 tuned a different one), once per timed layout
    for r in (0, 1):
        assert [e[1] for e in res[r][3] if e[0] == "set_plan"] == [(1, 1, 0)] * 4


def test_tp_leg_p2p_mismatch_drops_the_p2p_layouts_only():
    """a mismatch confined to the (experimental) peer-to-peer transport drops its layouts; the RCCL
    layouts still give the line, and no rank exits 3"""
    res = _run(corrupt="p2p")
    assert res[0][0] == 0 and res[1][0] == 0, res
    line = json.loads(res[0][1].strip().splitlines()[-1])
    assert set(line["layouts_tok_s"]) == {"split", "rep_attn"} and line["layout"] == "rep_attn"
    assert set(line["layouts_dropped"]) == {"p2p", "p2p_rep_attn"}


def test_tp_leg_forced_mismatch_exits_3_on_every_rank():
    res = _run(corrupt=True)
    assert res[0][0] == 3 and res[1][0] == 3, res
    err = json.loads(res[0][1].strip().splitlines()[-1])
    assert "error" in err and "rows over all ranks" in err["error"]
    assert res[1][1] == ""


def test_bench_merges_the_rccl_and_p2p_legs():
    """bench.py --gpus N runs the RCCL layouts and the p2p layouts as separate child legs
    (bench.merge_legs): the faster successful leg is the headline, per-layout rates and drops are
    merged, and a failed leg (a fault, a timeout, exit 3) is kept under failed_legs without costing
    the other's number."""
    sys.path.insert(0, ROOT)
    from bench import merge_legs
    rccl = {"tok_s": 2000.0, "ms_per_token": 0.5, "layout": "split",
            "layouts_tok_s": {"split": 2000.0, "rep_attn": 1900.0}, "layouts_dropped": {}}
    p2p = {"tok_s": 2500.0, "ms_per_token": 0.4, "layout": "p2p_rep_attn",
           "layouts_tok_s": {"p2p_rep_attn": 2500.0}, "layouts_dropped": {"p2p_split": "timed out"}}
    m = merge_legs(rccl, p2p)
    assert m["tok_s"] == 2500.0 and m["layout"] == "p2p_rep_attn"
    assert m["layouts_tok_s"] == {"split": 2000.0, "rep_attn": 1900.0, "p2p_rep_attn": 2500.0}
    assert m["layouts_dropped"] == {"p2p_split": "timed out"} and "failed_legs" not in m
    crashed = {"error": "Memory access fault", "exit": -6}
    m = merge_legs(rccl, crashed)
    assert m["tok_s"] == 2000.0 and m["failed_legs"] == {"p2p": crashed}
    m = merge_legs({"error": "timed out after 360 s"}, p2p)
    assert m["tok_s"] == 2500.0 and "rccl" in m["failed_legs"]
    both = merge_legs({"error": "a"}, {"error": "b"})
    assert "tok_s" not in both and both["error"] == "a"
    assert merge_legs(None, None) is None
    assert rccl["layouts_tok_s"] == {"split": 2000.0, "rep_attn": 1900.0}  # inputs untouched
