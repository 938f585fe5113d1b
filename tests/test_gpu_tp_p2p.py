"""The peer-to-peer transport of the row-split engine (GEMMA_TP_P2P) on ONE GPU.

Two processes, one rank each, both on device 0 (the box has one GPU; RCCL refuses two ranks per
device, the IPC path does not): every rank creates its row-split engine with tp = (2, rank, None)
and TP_P2P, publishes its uncached inbox arena as an IPC handle, the handles are exchanged over
gloo, each rank maps the other's arena (hipIpcOpenMemHandle) and decodes.  Every all-gather of the
step (q|k|v, sa, the h image, x, the argmax keys; the logits when asked for) is then a push into
the peer's inbox + a flag, inside the captured hipGraph, exactly the code an N-GPU node runs.  Bar:
tokens and every logit of BOTH ranks bit-identical to the CPU oracle (src/gemma_model.cpp:231-286
with the row partition of src/hpc.cpp:245-269).  The peers here share one device's memory, so
these runs check the protocol (inbox offsets, flags, sequence, copy-out), not xGMI coherence or
speed."""
import os
import socket
import sys

import numpy as np
import pytest

import oracle_ctypes as O

gpu = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _child(rank, world, port, shape, prompt, n_decode, n_ctx, flags, graph, q):
    try:
        os.environ["MASTER_ADDR"] = "127.0.0.1"
        os.environ["MASTER_PORT"] = str(port)
        sys.path.insert(0, os.path.join(ROOT, "gemma.ggml_amd", "python"))
        import torch.distributed as dist

        import gemma_hip as G
        import gemma_tp as T
        dist.init_process_group("gloo", rank=rank, world_size=world)
        comm = T.Comm(world, rank, dist)
        e = G.Engine(shape, n_ctx=n_ctx, device=0, tp=(world, rank, None), tp_flags=flags)
        assert e.tp_flags() == flags and e.tp_info()[:2] == [world, rank]
        T.open_p2p(comm, e)
        e.begin(prompt)
        lg = e.step(len(prompt) + n_decode, want_logits=True, use_graph=graph)
        toks = [int(t) for t in e.tokens()]
        e.begin(prompt)  # back-to-back replays without logits: tokens fed back through the key gather
        e.step(len(prompt) + n_decode, use_graph=graph)
        toks2 = [int(t) for t in e.tokens()]
        err = e.p2p_err()
        comm.barrier()  # no rank unmaps its arena while a peer may still push into it
        e.close()
        comm.close()
        q.put((rank, lg, toks, toks2, err, None))
    except Exception as ex:  # reported to the parent instead of hanging it
        q.put((rank, None, None, None, None, repr(ex)))


def _run(shape, n_prompt, n_decode, n_ctx, flags, graph=True, world=2):
    import torch.multiprocessing as mp
    O.lib().orc_set_threads(16)
    prompt = O.make_prompt(n_prompt, shape["n_vocab"])
    m = O.Model(O.make_config(shape, n_ctx=n_ctx))
    seq_ref, lg_ref = m.generate(prompt, n_decode)
    m.close()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_child, args=(r, world, port, shape, prompt, n_decode, n_ctx, flags, graph, q))
             for r in range(world)]
    for p in procs:
        p.start()
    res = {}
    try:
        for _ in range(world):
            r = q.get(timeout=240)
            res[r[0]] = r[1:]
    finally:
        for p in procs:
            p.join(timeout=30)
            if p.is_alive():
                p.kill()
    for r in range(world):
        lg, toks, toks2, err, ex = res[r]
        assert ex is None, f"rank {r}: {ex}"
        assert err == 0, f"rank {r}: a p2p flag wait timed out"
        assert toks[: len(seq_ref)] == list(seq_ref), f"rank {r} tokens"
        assert toks2[: len(seq_ref)] == list(seq_ref), f"rank {r} tokens (no logits)"
        got = lg[len(prompt) - 1:]
        bad = np.argwhere(got.view(np.uint32) != lg_ref.view(np.uint32))
        assert bad.size == 0, f"rank {r}: {len(bad)} logits differ, first {bad[:5]}"


@gpu
@pytest.mark.parametrize("rep_attn", [0, 1], ids=["split", "rep_attn"])
def test_p2p_two_ranks_tiny(rep_attn):
    import gemma_hip as G
    _run(dict(O.TINY), 6, 6, 128, G.TP_P2P | G.TP_REP_ATTN * rep_attn)


@gpu
def test_p2p_two_ranks_tiny_eager():
    import gemma_hip as G
    _run(dict(O.TINY), 5, 4, 128, G.TP_P2P, graph=False)


@gpu
@pytest.mark.parametrize("rep_attn", [0, 1], ids=["split", "rep_attn"])
def test_p2p_two_ranks_gemma2b_shapes(rep_attn):
    """Gemma-2B shapes (18 layers, the 256,000-row output split 2 ways), 2 prompt + 2 decode rows."""
    import gemma_hip as G
    _run(dict(O.GEMMA_2B), 3, 2, 64, G.TP_P2P | G.TP_REP_ATTN * rep_attn)


@gpu
def test_p2p_four_ranks_tiny():
    """Four ranks on the one device: three pushes and three flag waits per gather."""
    import gemma_hip as G
    _run(dict(O.TINY), 4, 4, 128, G.TP_P2P, world=4)
