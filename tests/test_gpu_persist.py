"""GPU parity of the persistent token launch (csrc/token.hip): the decode step's
layers as ONE launch with in-launch granule hand-offs and LDS-DMA weight rings.

Bar: bit-identical logits and greedy tokens to the CPU oracle (the reference's per-token graph,
src/gemma_model.cpp:231-286 / :665-747) and to the per-layer launch path, and no hand-off timeout.
The launch is built for Gemma-2B's E = 2048 / F = 16384; the shapes here keep those and cut the
layer count and vocabulary so the oracle stays fast.
"""
import numpy as np
import pytest

import oracle_ctypes as O

gpu = pytest.mark.gpu

GEMMA_2B_LAYERS = dict(n_layer=3, n_embd=2048, n_head=8, n_head_kv=1, head_dim=256, n_ff=16384, n_vocab=8192)


def _engine(shape, **kw):
    import gemma_hip as G
    return G.Engine(shape, **kw)


def _decode(e, prompt, n_decode):
    e.begin(prompt)
    lg = e.step(len(prompt) + n_decode, want_logits=True, use_graph=True)
    return lg, list(e.tokens())


@gpu
@pytest.mark.parametrize("wtype", [O.Q4_0, O.Q8_0])
@pytest.mark.parametrize("n_head_kv", [1, 2])
def test_persist_decode_bitexact(wtype, n_head_kv):
    O.lib().orc_set_threads(16)
    shape = dict(GEMMA_2B_LAYERS, n_head_kv=n_head_kv)
    n_ctx = 128
    m = O.Model(O.make_config(shape, n_ctx=n_ctx, wtype=wtype))
    prompt = O.make_prompt(6, shape["n_vocab"])
    seq_ref, lg_ref = m.generate(prompt, 8)
    e = _engine(shape, n_ctx=n_ctx, wtype=wtype)
    assert e.set_persist(1), "the persistent launch should run Gemma-2B layer shapes"
    e.persist_err(reset=True)
    lg, toks = _decode(e, prompt, 8)
    err = e.persist_err()
    e.close()
    assert err[0] == 0, f"hand-off timeout {err}"
    assert toks[: len(seq_ref)] == list(seq_ref)
    got = lg[len(prompt) - 1:]
    bad = np.argwhere(got.view(np.uint32) != lg_ref.view(np.uint32))
    assert bad.size == 0, f"{len(bad)} logits differ, first {bad[:5]} max abs {np.abs(got - lg_ref).max()}"


@gpu
@pytest.mark.parametrize("wtype", [O.Q4_0, O.Q8_0])
def test_persist_matches_launch_path(wtype):
    """every logit of 70 steps (positions across several n_kv paddings) equal with and without the
    persistent launch, on full Gemma-2B shapes"""
    shape = O.GEMMA_2B
    prompt = O.make_prompt(5, shape["n_vocab"])
    e = _engine(shape, n_ctx=256, wtype=wtype)
    assert e.set_persist(1)
    e.persist_err(reset=True)
    lg1, t1 = _decode(e, prompt, 65)
    assert e.persist_err()[0] == 0
    assert not e.set_persist(0)
    lg0, t0 = _decode(e, prompt, 65)
    e.close()
    assert t1 == t0
    assert np.array_equal(lg1.view(np.uint32), lg0.view(np.uint32))


@gpu
def test_persist_gemma2b_bitexact():
    """full Gemma-2B (18 layers, 256000 vocab) against the oracle through the persistent launch"""
    O.lib().orc_set_threads(16)
    shape = O.GEMMA_2B
    m = O.Model(O.make_config(shape, n_ctx=256))
    prompt = O.make_prompt(6, shape["n_vocab"])
    seq_ref, lg_ref = m.generate(prompt, 4)
    e = _engine(shape, n_ctx=256)
    assert e.set_persist(1)
    lg, toks = _decode(e, prompt, 4)
    assert e.persist_err()[0] == 0
    e.close()
    assert toks[: len(seq_ref)] == list(seq_ref)
    assert np.array_equal(lg[len(prompt) - 1:].view(np.uint32), lg_ref.view(np.uint32))


@gpu
def test_persist_declines_unsupported_shapes():
    """shapes outside the launch's build (tiny model) fall back to the per-layer launches"""
    e = _engine(O.TINY, n_ctx=64)
    assert not e.set_persist(1)
    e.close()


@gpu
def test_persist_declines_kquant():
    """K-quant layers never take the launch: set_persist reports 0 and steps run the K-quant path"""
    import gemma_hip as G
    e = _engine(dict(GEMMA_2B_LAYERS, n_layer=1), n_ctx=64, wtype=G.GGML_TYPE_Q4_K)
    assert not e.set_persist(1)
    assert "K-quant" in G.last_error()
    e.close()


@gpu
def test_persist_timeout_reported():
    """a hand-off timeout inside the launch (forced with a 10 ns per-wait bound) must
    fail the step, leave the launch off, and the restarted sequence must be the oracle's again"""
    import gemma_hip as G
    O.lib().orc_set_threads(16)
    shape = GEMMA_2B_LAYERS
    m = O.Model(O.make_config(shape, n_ctx=64))
    prompt = O.make_prompt(4, shape["n_vocab"])
    seq_ref, lg_ref = m.generate(prompt, 3)
    e = _engine(shape, n_ctx=64)
    assert e.set_persist(1)
    assert e.set_persist_timeout(1) == 0
    e.persist_err(reset=True)
    e.begin(prompt)
    with pytest.raises(RuntimeError, match="hand-off timeout"):
        e.step(len(prompt) + 3, want_logits=False, use_graph=True)
    assert not e.set_persist(-1), "the launch must be off after a timeout"
    assert e.persist_err()[0] == 0, "the sticky word is cleared once reported"
    lg, toks = _decode(e, prompt, 3)
    e.close()
    assert toks[: len(seq_ref)] == list(seq_ref)
    assert np.array_equal(lg[len(prompt) - 1:].view(np.uint32), lg_ref.view(np.uint32))
