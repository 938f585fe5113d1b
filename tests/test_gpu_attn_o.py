"""The decode attention + attn-out (+ residual) as ONE launch per layer (layer_front.hip k_attn_o:
the attention launch's idle workgroups run attn-out's row tiles behind an in-launch sc1 hand-off)
against the oracle (src/gemma_model.cpp:454-497, :723 restated) and against the two separate launches,
bit for bit; the launch count drops by one per layer and no hand-off may time out.  The counters
reset themselves inside each launch, so long runs (hundreds of launches per layer) must stay exact."""
import numpy as np
import pytest

import oracle_ctypes as O

gpu = pytest.mark.gpu


def _engine(shape, **kw):
    import gemma_hip as G
    return G.Engine(shape, **kw)


@gpu
@pytest.mark.parametrize("kv", [1, 8], ids=["gqa_2b", "mha"])
def test_attn_o_bitexact_vs_oracle(kv):
    O.lib().orc_set_threads(16)
    shape = dict(O.GEMMA_2B, n_layer=3, n_vocab=8192, n_head_kv=kv)
    m = O.Model(O.make_config(shape, n_ctx=256))
    prompt = O.make_prompt(9, shape["n_vocab"])
    seq_ref, lg_ref = m.generate(prompt, 40)
    m.close()
    e = _engine(shape, n_ctx=256)
    p = e.plan()
    p.update(attn_out=(9, 1, 1), attention=0)
    e.set_plan(p)
    e.set_att_o(0)
    e.begin(prompt)
    e.step(2, use_graph=True)
    n_two = e.graph_kernels()
    assert e.set_att_o(1)
    e.begin(prompt)
    lg = e.step(len(prompt) + 40, want_logits=True, use_graph=True)
    assert e.graph_kernels() == n_two - shape["n_layer"], "the fused launch did not replace attention + attn-out"
    assert list(e.tokens()[: len(seq_ref)]) == list(seq_ref)
    bad = np.argwhere(lg[len(prompt) - 1:].view(np.uint32) != lg_ref.view(np.uint32))
    assert bad.size == 0, f"{len(bad)} logits differ, first {bad[:5]}"
    e.close()


@gpu
def test_attn_o_gemma2b_bench_positions_bitexact():
    """BASELINE config 2 as bench.py runs it, with the fused launch: the tuned plan, the 128-token
    prompt through the hipGraph, 24 greedy steps; every logit against the oracle."""
    O.lib().orc_set_threads(16)
    prompt = O.make_prompt(128, O.GEMMA_2B["n_vocab"])
    m = O.Model(O.make_config(O.GEMMA_2B, n_ctx=512))
    seq_ref, lg_ref = m.generate(prompt, 24)
    m.close()
    e = _engine(O.GEMMA_2B, n_ctx=512)
    e.tune(6)
    p = e.plan()
    p.update(attn_out=(9, 1, 1), attention=0)
    e.set_plan(p)
    assert e.set_att_o(1)
    e.begin(prompt)
    lg = e.step(len(prompt) + 24, want_logits=True, use_graph=True)
    toks = list(e.tokens()[: len(seq_ref)])
    e.close()
    assert toks == list(seq_ref)
    bad = np.argwhere(lg[len(prompt) - 1:].view(np.uint32) != lg_ref.view(np.uint32))
    assert bad.size == 0, f"{len(bad)} logits differ, first {bad[:5]}"


@gpu
def test_attn_o_long_run_equals_two_launches():
    """300 graph replays (each layer's counters used 300 times, reset inside every launch): every
    logit equal with and without the fused launch, eager and graph."""
    shape = dict(O.GEMMA_2B, n_layer=2, n_vocab=4096)
    prompt = O.make_prompt(5, shape["n_vocab"])
    outs = []
    for fused, graph in ((0, True), (1, True), (1, False)):
        e = _engine(shape, n_ctx=512)
        p = e.plan()
        p.update(attn_out=(9, 1, 1), attention=0)
        e.set_plan(p)
        e.set_att_o(fused)
        e.begin(prompt)
        outs.append(e.step(300, want_logits=True, use_graph=graph))
        e.close()
    assert np.array_equal(outs[0].view(np.uint32), outs[1].view(np.uint32))
    assert np.array_equal(outs[0].view(np.uint32), outs[2].view(np.uint32))
