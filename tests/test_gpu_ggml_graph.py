"""The ggml operator surface: the reference's graph code restated against
include/ggml.h (tests/ggml_driver/gemma_graph_driver.cpp, same API calls as src/gemma_model.cpp)
runs on the MI355X graph executor, and its logits — prefill (last row) and every decode step — and
greedy tokens are bit-identical to the CPU oracle."""
import os
import subprocess

import numpy as np
import pytest

import oracle_ctypes as O

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
DRIVER = os.path.join(ROOT, "tests", "ggml_driver", "gemma_graph_driver")
gpu = pytest.mark.gpu


def test_driver_built():
    assert os.path.exists(DRIVER), "make -C gemma.ggml_amd builds the ggml graph driver"


def _run(tmp_path, shape, wtype, n_prompt, n_decode, ctx):
    m = O.Model(O.make_config(shape, n_ctx=ctx, wtype=wtype))
    wpath, ppath, opath = tmp_path / "w.bin", tmp_path / "p.bin", tmp_path / "o.bin"
    with open(wpath, "wb") as f:
        f.write(m.tensor(0).tobytes())  # token_embd (also the tied output)
        f.write(m.tensor(1).tobytes())  # output_norm
        for il in range(shape["n_layer"]):
            for k in range(9):  # attn_norm q k v o ffn_norm gate up down
                f.write(m.tensor(16 + il * 16 + k).tobytes())
    prompt = np.array(O.make_prompt(n_prompt, shape["n_vocab"]), dtype=np.int32)
    prompt.tofile(ppath)
    args = [DRIVER, str(wpath), str(ppath), str(opath)] + [str(shape[k]) for k in
            ("n_layer", "n_embd", "n_head", "n_head_kv", "head_dim", "n_ff", "n_vocab")] + [str(ctx), str(wtype),
                                                                                          str(n_decode)]
    r = subprocess.run(args, capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr[-2000:]
    raw = np.fromfile(opath, dtype=np.float32)
    V = shape["n_vocab"]
    logits = raw[: (n_decode + 1) * V].reshape(n_decode + 1, V)
    toks = raw[(n_decode + 1) * V:].view(np.int32)
    # oracle: the reference's inference() sequence (PREFILL, then DECODE per token)
    seq = list(prompt)
    t0, l0, _ = m.inference(seq, 0)
    refs, rtoks = [l0], [t0]
    seq.append(t0)
    for _ in range(n_decode):
        t, lg, _ = m.inference(seq, 1)
        refs.append(lg)
        rtoks.append(t)
        seq.append(t)
    m.close()
    for i, ref in enumerate(refs):
        assert np.array_equal(logits[i].view(np.uint32), ref.view(np.uint32)), (i, np.abs(logits[i] - ref).max())
    assert list(toks) == rtoks


@gpu
def test_ggml_graph_tiny_q4_0(tmp_path):
    _run(tmp_path, dict(O.TINY), O.Q4_0, 20, 4, 128)


@gpu
def test_ggml_graph_gqa_q8_0(tmp_path):
    _run(tmp_path, dict(O.TINY, n_head=4, n_head_kv=2), O.Q8_0, 37, 3, 128)


@gpu
def test_ggml_graph_gemma2b_layers(tmp_path):
    shape = dict(O.GEMMA_2B, n_layer=2, n_vocab=8192)
    _run(tmp_path, shape, O.Q4_0, 40, 2, 128)
