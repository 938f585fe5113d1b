"""The RCCL transport of the row-split engine (BASELINE config 4) on ONE GPU.

The box has one GPU and RCCL refuses two ranks per device, so N > 1 runs only on the driver's
8-GPU node.  A 1-rank communicator (gemma_tp_unique_id + ncclCommInitRank(nranks = 1)) sends the
engine down exactly the code the N-GPU ranks run: every activation vector and the h image through
in-place ncclAllGather (grouped for the image), the per-rank argmax key through ncclAllGather +
the key merge, RCCL inside the captured decode hipGraph.  Bar: tokens and every logit bit-identical
to the CPU oracle (the reference's per-token graph, src/gemma_model.cpp:231-286 with the row
partition of src/hpc.cpp:245-269 restated in oracle/), as the virtual-rank tests require.
"""
import numpy as np
import pytest

import oracle_ctypes as O

gpu = pytest.mark.gpu

GEMMA_7B_LAYERS = dict(n_layer=3, n_embd=3072, n_head=16, n_head_kv=16, head_dim=256, n_ff=24576, n_vocab=8192)


def _rccl_engine(shape, n_ctx, **kw):
    import gemma_hip as G
    uid = G.tp_unique_id()
    e = G.Engine(shape, n_ctx=n_ctx, device=0, tp=(1, 0, uid), **kw)
    info = e.tp_info()
    assert info == [1, 0, 1, 1], f"expected a 1-rank RCCL communicator, got tp_info {info}"
    return e


def _check(shape, n_prompt, n_decode, n_ctx=64, graph=True):
    O.lib().orc_set_threads(16)
    prompt = O.make_prompt(n_prompt, shape["n_vocab"])
    m = O.Model(O.make_config(shape, n_ctx=n_ctx))
    seq_ref, lg_ref = m.generate(prompt, n_decode)
    m.close()
    e = _rccl_engine(shape, n_ctx)
    e.begin(prompt)
    lg = e.step(len(prompt) + n_decode, want_logits=True, use_graph=graph)
    toks = list(e.tokens()[: len(seq_ref)])
    # without logits: graph replays back to back, tokens fed back on the device through the key gather
    e.begin(prompt)
    e.step(len(prompt) + n_decode, want_logits=False, use_graph=graph)
    toks2 = list(e.tokens()[: len(seq_ref)])
    e.close()
    assert toks == list(seq_ref)
    assert toks2 == list(seq_ref)
    got = lg[len(prompt) - 1:]
    bad = np.argwhere(got.view(np.uint32) != lg_ref.view(np.uint32))
    assert bad.size == 0, f"{len(bad)} logits differ, first {bad[:5]}"


@gpu
def test_rccl_one_rank_tiny_eager_and_graph():
    for graph in (False, True):
        _check(dict(O.TINY), 6, 6, n_ctx=128, graph=graph)


@gpu
def test_rccl_one_rank_gemma2b():
    _check(dict(O.GEMMA_2B), 5, 3)


@gpu
def test_rccl_one_rank_gemma7b_layers():
    _check(dict(GEMMA_7B_LAYERS), 5, 3)


@gpu
def test_rccl_one_rank_declines_prefill_and_kquant():
    import gemma_hip as G
    e = _rccl_engine(dict(O.TINY), 64)
    e.begin(O.make_prompt(4, O.TINY["n_vocab"]))
    with pytest.raises(RuntimeError):
        e.prefill(4)
    assert not e.set_persist(1)  # the persistent launch is single-engine only
    e.close()
    with pytest.raises(RuntimeError):
        G.Engine(dict(O.GEMMA_2B, n_layer=1), n_ctx=64, wtype=G.GGML_TYPE_Q4_K, tp=(1, 0, G.tp_unique_id()))


@gpu
def test_rccl_unique_id_serves_one_communicator():
    """Two communicators in one process each need their own id (the bench's TP leg builds a parity
    engine and then the timed engine): a fresh id per engine works, in sequence and side by side."""
    import gemma_hip as G
    shape = dict(O.TINY)
    a = G.Engine(shape, n_ctx=64, device=0, tp=(1, 0, G.tp_unique_id()))
    b = G.Engine(shape, n_ctx=64, device=0, tp=(1, 0, G.tp_unique_id()))
    assert a.tp_info() == [1, 0, 1, 1] and b.tp_info() == [1, 0, 1, 1]
    prompt = O.make_prompt(4, shape["n_vocab"])
    outs = []
    for e in (a, b):
        e.begin(prompt)
        outs.append(e.step(len(prompt) + 2, want_logits=True, use_graph=True))
        e.close()
    assert np.array_equal(outs[0].view(np.uint32), outs[1].view(np.uint32))


@gpu
def test_bench_tp_leg_runs_at_one_gpu():
    """bench.py's config-4 leg (scripts/tp_leg.py) end to end at N = 1: unsplit reference, 8 virtual
    ranks and a 1-rank RCCL engine checked bit-exact, then the timed 1-rank RCCL engine."""
    import json
    import os
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env = dict(os.environ, WORLD_SIZE="1", RANK="0", LOCAL_RANK="0")
    r = subprocess.run([sys.executable, os.path.join(root, "scripts", "tp_leg.py"), "4", "q4_0", "0"],
                       capture_output=True, text=True, timeout=240, env=env)
    assert r.returncode == 0, r.stderr[-2000:]
    line = json.loads(r.stdout.strip().splitlines()[-1])
    assert "error" not in line, line
    assert line["parity_check"]["mismatched_rows_all_ranks"] == 0 and line["tok_s"] > 0


@gpu
def test_bench_tp_leg_2b_headline_at_one_gpu():
    """The N > 1 headline leg (Gemma-2B row-split, scripts/tp_leg.py 2b) end to end at N = 1 with the
    bench's prompt length: parity vs the unsplit engine (8 virtual ranks + a 1-rank RCCL engine),
    rank 0's tuned plan installed, the timed 1-rank RCCL stream and its per-shard roofline."""
    import json
    import os
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env = dict(os.environ, WORLD_SIZE="1", RANK="0", LOCAL_RANK="0")
    r = subprocess.run([sys.executable, os.path.join(root, "scripts", "tp_leg.py"), "8", "q4_0", "1", "2b", "2", "128"],
                       capture_output=True, text=True, timeout=240, env=env)
    assert r.returncode == 0, r.stderr[-2000:]
    line = json.loads(r.stdout.strip().splitlines()[-1])
    assert "error" not in line, line
    assert line["parity_check"]["mismatched_rows_all_ranks"] == 0 and line["tok_s"] > 0
    assert line["steps"] == 8 and line["warmup"] == 2 and line["prompt"] == 128
    assert line["roofline"]["classes"] and line["roofline"]["avg_us"] > 0
