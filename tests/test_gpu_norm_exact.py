"""ggml-exact RMSNorm on adversarial inputs (VERDICT r4 "Next round" #1(a)).

ggml's rms_norm sums (double)(x*x) in index order (src/gemma_model.cpp:438-442).  Every
kernel here sums the same terms in a tree and keeps the tree's mean only when rms_mean_certain
proves it equal to the sequential one, else it runs the sequential sum (csrc/device_util.h).
tests/norm_adversary.py builds embedding rows on which ANY summation tree of depth <= 32 and the
sequential sum give different means (checked on the CPU: test_rows_are_adversarial), plus a norm
weight w0 that carries the one-ulp scale difference into the quantized activation.  Each GPU run
below must equal the oracle bit for bit — which a tree mean cannot:

  * the two norm kernels alone (ggml executor RMS_NORM, k_norm_q8K) on host rows;
  * the decode engine (Q4_0, Q8_0: the matvec prologue, PRO_EMBED / PRO_NORM) and its exact batched
    prefill (k_quant_rows), on a GGUF whose token_embd row and attn_norm carry the adversary;
  * the K-quant engine (Q4_K / Q6_K layers, Q6_K token_embd) under the Q8_K INIT plans that put the
    norm in the consumer's prologue (kq_pro_build), in a launch (k_norm_q8K) or in a hand-off tail;
  * the ggml graph executor, node by node (k_g_rms_norm) and on its fast path;
  * the persistent token launch (token.hip norm_quant).
"""
import ctypes as C

import numpy as np
import pytest

import norm_adversary as A
import oracle_ctypes as O

gpu = pytest.mark.gpu
EPS = 1e-6
ADV_TOKEN = 77


def _adversary(fmt, n, kind, seed=1):
    row, x, info = A.build_row(fmt, n, eps=EPS, seed=seed)
    w0 = A.pick_norm_weight(x[0], info, kind)
    return row, x, info, w0


def test_rows_are_adversarial():
    """CPU: the rows really separate tree and sequential means, and w0 makes the quantized
    activation's block scale depend on which mean is used."""
    for fmt, n, kind in (("q8_0", 512, "q8_0"), ("q4_0", 512, "q8_0"), ("q6_K", 512, "q8_K"), ("q8_0", 2048, "q8_0")):
        row, x, info, w0 = _adversary(fmt, n, kind)
        ok, info2 = A.verify(x, EPS)
        assert ok and info2["ulps"] > 2 * A.TREE_ULPS, (fmt, n, info2)
        # numpy's pairwise sum (one more tree) lands on the tree side, the loop on the sequential side
        t = (x * x).astype(np.float64)
        assert A.mean_of(float(np.sum(t)), n) == info["mean_tree"] != info["mean_seq"]
        ys = np.float32(np.float32(x[0]) * info["scale_seq"]) * w0
        yt = np.float32(np.float32(x[0]) * info["scale_tree"]) * w0
        if kind == "q8_0":
            assert np.float16(np.abs(ys) / np.float32(127)) != np.float16(np.abs(yt) / np.float32(127))
        else:
            assert np.float32(1.0 / np.float64(np.float32(-127.0 / np.float64(ys)))) != \
                np.float32(1.0 / np.float64(np.float32(-127.0 / np.float64(yt))))


def _rms_rows(x):
    L = O.lib()
    y = np.zeros_like(x)
    for r in range(x.shape[0]):
        L.orc_rms_norm(O.ptr(x[r]), O.ptr(y[r]), x.shape[1], EPS)
    return y


def _test_rows(n, fmt):
    rng = np.random.default_rng(n)
    _, xa, _, _ = _adversary(fmt, n, "q8_K")
    rows = [xa]
    rows += [rng.standard_normal(n).astype(np.float32) for _ in range(6)]
    rows += [(rng.standard_normal(n) * np.exp(rng.uniform(-12, 12, n))).astype(np.float32) for _ in range(6)]
    for seed in (2, 3):
        rows.append(A.build_row(fmt, n, eps=EPS, seed=seed)[1])
    return np.ascontiguousarray(np.stack(rows), dtype=np.float32)


@gpu
@pytest.mark.parametrize("n", [512, 2048, 3072])
def test_ggml_rms_norm_kernel_adversarial(n):
    import gemma_hip as G
    L = G.lib()
    L.gemma_test_rms_norm.restype = C.c_int
    L.gemma_test_rms_norm.argtypes = [C.c_int, C.c_void_p, C.c_void_p, C.c_int, C.c_int, C.c_float, C.c_void_p]
    x = _test_rows(n, "q8_0")
    out = np.zeros_like(x)
    assert L.gemma_test_rms_norm(0, x.ctypes.data, None, x.shape[0], n, EPS, out.ctypes.data) == 0, G.last_error()
    ref = _rms_rows(x)
    bad = np.argwhere(out.view(np.uint32) != ref.view(np.uint32))
    assert bad.size == 0, f"rows {sorted(set(bad[:, 0].tolist()))} differ from ggml's sequential sum"


@gpu
@pytest.mark.parametrize("n", [512, 2048])
def test_norm_q8K_kernel_adversarial(n):
    import gemma_hip as G
    L = G.lib()
    L.gemma_test_rms_norm.restype = C.c_int
    L.gemma_test_rms_norm.argtypes = [C.c_int, C.c_void_p, C.c_void_p, C.c_int, C.c_int, C.c_float, C.c_void_p]
    x = _test_rows(n, "q6_K")
    _, xa, info, w0 = _adversary("q6_K", n, "q8_K")
    w = np.ones(n, dtype=np.float32)
    w[0] = w0
    out = np.zeros((x.shape[0], n // 256 * 292), dtype=np.uint8)
    assert L.gemma_test_rms_norm(1, x.ctypes.data, w.ctypes.data, x.shape[0], n, EPS, out.ctypes.data) == 0, G.last_error()
    ref = O.quantize_q8_K(_rms_rows(x) * w)
    bad = [r for r in range(x.shape[0]) if not np.array_equal(out[r], ref[r])]
    assert not bad, f"Q8_K rows {bad} differ from the oracle"


# ---- whole models carrying the adversarial row --------------------------------------------------
SHAPE = dict(n_layer=2, n_embd=512, n_head=2, n_head_kv=1, head_dim=256, n_ff=1024, n_vocab=2048)
KSHAPE = dict(n_layer=2, n_embd=512, n_head=2, n_head_kv=1, head_dim=256, n_ff=512, n_vocab=1024)


def _poke_model(m, fmt, kind, n_embd):
    """token ADV_TOKEN's embedding row := the adversarial row; layer 0's attn_norm[0] := w0"""
    row, x, info, w0 = _adversary(fmt, n_embd, kind)
    m.poke(0, ADV_TOKEN * row.size, row)
    m.poke(16, 0, np.array([w0], dtype=np.float32))
    return info


def _prompt(n_vocab, n):
    p = list(O.make_prompt(n, n_vocab))
    p[1] = ADV_TOKEN  # the adversary at a prompt row and as a decode input
    p[n // 2] = ADV_TOKEN
    p[-1] = ADV_TOKEN
    return p


def _engine_vs_oracle(e, m, prompt, n_decode):
    seq_ref, lg_ref = m.generate(prompt, n_decode)
    e.begin(prompt)
    lg = e.step(len(prompt) + n_decode, want_logits=True)
    got = lg[len(prompt) - 1:]
    bad = np.argwhere(got.view(np.uint32) != lg_ref.view(np.uint32))
    assert bad.size == 0, f"decode: {len(bad)} logits differ, first {bad[:5]}"
    assert list(e.tokens()[: len(seq_ref)]) == list(seq_ref)
    # the batched exact prefill over the same prompt
    m.reset()
    tok_ref, _, all_ref = m.inference(prompt, 0, want_all=True)
    e.begin(prompt)
    tok, _, allv = e.prefill(len(prompt), want_all=True)
    bad = np.argwhere(allv.view(np.uint32) != all_ref.view(np.uint32))
    assert bad.size == 0, f"prefill: {len(bad)} logits differ, first {bad[:5]}"
    assert tok == tok_ref


@gpu
@pytest.mark.parametrize("wtype,fmt", [(O.Q4_0, "q4_0"), (O.Q8_0, "q8_0")])
def test_engine_adversarial_embedding(tmp_path, wtype, fmt):
    import gemma_hip as G
    from test_gpu_ggml_graph import write_gguf
    m = O.Model(O.make_config(SHAPE, n_ctx=128, wtype=wtype))
    _poke_model(m, fmt, "q8_0", SHAPE["n_embd"])
    path = tmp_path / "adv.gguf"
    write_gguf(m, SHAPE, path, 0)
    e = G.Engine.from_gguf(str(path), n_ctx=128)
    _engine_vs_oracle(e, m, _prompt(SHAPE["n_vocab"], 12), 6)
    e.close()
    m.close()


@gpu
@pytest.mark.parametrize("fuse", [5, 0, 2])
def test_kquant_engine_adversarial_embedding(tmp_path, fuse):
    """Q8_K INIT plans (engine.cpp enqueue_step_kq): 5 norms in the consumers' prologues, 0 as
    k_norm_q8K launches, 2 in the producers' hand-off tails"""
    import gemma_hip as G
    from test_gpu_ggml_graph import write_gguf
    m = O.Model(O.make_config(KSHAPE, n_ctx=128, kmix=1))
    _poke_model(m, "q6_K", "q8_K", KSHAPE["n_embd"])
    path = tmp_path / "adv_kq.gguf"
    write_gguf(m, KSHAPE, path, 1)
    e = G.Engine.from_gguf(str(path), n_ctx=128)
    e.set_option("kq_fuse", fuse)
    _engine_vs_oracle(e, m, _prompt(KSHAPE["n_vocab"], 10), 5)
    e.close()
    m.close()


@gpu
@pytest.mark.parametrize("fast", [0, 1])
def test_ggml_graph_adversarial_embedding(tmp_path, fast):
    from test_gpu_ggml_graph import _run
    _run(tmp_path, dict(SHAPE), O.Q8_0, 0, 3, 128, gguf=True, fast=fast,
         poke=lambda m: _poke_model(m, "q8_0", "q8_0", SHAPE["n_embd"]), prompt=_prompt(SHAPE["n_vocab"], 9))


@gpu
def test_persist_adversarial_embedding(tmp_path):
    import gemma_hip as G
    from test_gpu_ggml_graph import write_gguf
    shape = dict(n_layer=1, n_embd=2048, n_head=8, n_head_kv=1, head_dim=256, n_ff=16384, n_vocab=1024)
    m = O.Model(O.make_config(shape, n_ctx=64))
    _poke_model(m, "q4_0", "q8_0", shape["n_embd"])
    path = tmp_path / "adv_p.gguf"
    write_gguf(m, shape, path, 0)
    e = G.Engine.from_gguf(str(path), n_ctx=64)
    assert e.set_persist(1), "the persistent launch should take Gemma-2B layer shapes"
    e.persist_err(reset=True)
    prompt = _prompt(shape["n_vocab"], 6)
    seq_ref, lg_ref = m.generate(prompt, 4)
    e.begin(prompt)
    lg = e.step(len(prompt) + 4, want_logits=True, use_graph=True)
    assert e.persist_err()[0] == 0
    got = lg[len(prompt) - 1:]
    assert np.array_equal(got.view(np.uint32), lg_ref.view(np.uint32))
    assert list(e.tokens()[: len(seq_ref)]) == list(seq_ref)
    e.close()
    m.close()
