"""CPU, world_size 2 over gloo: the row-split partition math of the TP engine.

Each rank computes its contiguous row shard of every Gemma matrix with the oracle's mul_mat
(restatement of src/hpc.cpp) and all-gathers; the result equals the single-process product bit for
bit (row split has no cross-rank reduction).  The argmax merge mirrors k_reduce_keys: per-rank
(ordered value, ~global index) keys, gathered, max taken — the first maximum wins as in
src/gemma_model.cpp:538-543, including ties that straddle ranks."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

import oracle_ctypes as O


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _key(v, idx):
    u = np.float32(v).view(np.uint32).item()
    u = (~u & 0xFFFFFFFF) if (u & 0x80000000) else (u | 0x80000000)
    return (u << 32) | (0xFFFFFFFF - idx)


def _worker(rank, world, port, q):
    try:
        _work(rank, world, port, q)
    except Exception as ex:  # report instead of hanging the parent
        q.put((rank, repr(ex)))


def _work(rank, world, port, q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    rng = np.random.default_rng(7)
    ok = True
    # (rows, K) of Gemma-2B's matrices scaled down 4x in K: fused qkv, o, gate, down, output
    for rows, K in [(2560, 512), (2048, 512), (16384, 256), (2048, 1024), (4096, 256)]:
        assert rows % (8 * world) == 0
        W = O.quantize((rng.standard_normal((rows, K)) * 0.05).astype(np.float32), "q4_0_ref")
        x = rng.standard_normal((1, K)).astype(np.float32)
        wdata, rs = O.mul_mat_init(O.Q4_0, x)
        full = O.mul_mat(W, O.Q4_0, rows, W.shape[1], K, wdata, rs, 1)[0]
        sh = rows // world
        mine = O.mul_mat(np.ascontiguousarray(W[rank * sh:(rank + 1) * sh]), O.Q4_0, sh, W.shape[1], K, wdata, rs, 1)[0]
        parts = [torch.zeros(sh) for _ in range(world)]
        dist.all_gather(parts, torch.from_numpy(mine.copy()))
        got = torch.cat(parts).numpy()
        ok &= np.array_equal(got.view(np.uint32), full.view(np.uint32))
    # argmax merge with a tie across the rank boundary: the lower global index must win
    V = 64
    logits = rng.standard_normal(V).astype(np.float32)
    logits[V // world + 3] = logits[5] = np.float32(9.0)  # same max on two ranks
    sh = V // world
    loc = logits[rank * sh:(rank + 1) * sh]
    i = int(np.argmax(loc))  # numpy argmax: first max, like the kernel's strict '>'
    key = _key(loc[i], rank * sh + i)
    k = torch.tensor([key - (1 << 64) if key >= (1 << 63) else key], dtype=torch.int64)  # u64 bits in int64
    keys = [torch.zeros(1, dtype=torch.int64) for _ in range(world)]
    dist.all_gather(keys, k)
    best = max(int(t.item()) & 0xFFFFFFFFFFFFFFFF for t in keys)
    ok &= (0xFFFFFFFF - (best & 0xFFFFFFFF)) == int(np.argmax(logits)) == 5
    q.put((rank, bool(ok)))
    dist.destroy_process_group()


def test_row_split_allgather_world2():
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = dict(q.get(timeout=90) for _ in range(world))
    for p in procs:
        p.join(timeout=60)
    assert res == {0: True, 1: True}, res
