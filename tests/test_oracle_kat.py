"""CPU tests of the ORACLE: analytic known-answer tests (the only pins available for the ggml
semantics), internal consistency (ordered vs AVX2 paths), and format round trips."""
import numpy as np
import pytest

import oracle_ctypes as O


def test_fp16_conversion_matches_numpy():
    rng = np.random.default_rng(0)
    vals = np.concatenate([rng.standard_normal(20000).astype(np.float32) * s for s in (1e-8, 1e-5, 1, 1e3, 7e4)])
    vals = np.concatenate([vals, np.array([0.0, -0.0, 65504.0, 65520.0, 1e9, -1e9, 2.0 ** -24, 2.0 ** -25,
                                           3 * 2.0 ** -26, np.inf, -np.inf], dtype=np.float32)])
    got = O.fp32_to_fp16_bits(vals)
    ref = vals.astype(np.float16).view(np.uint16)
    assert np.array_equal(got, ref)
    L = O.lib()
    allh = np.arange(65536, dtype=np.uint16)
    back = np.array([L.orc_fp16_to_fp32(int(h)) for h in allh[::97]], dtype=np.float32)
    ref_back = allh[::97].view(np.float16).astype(np.float32)
    same = (back == ref_back) | (np.isnan(back) & np.isnan(ref_back))
    assert same.all()


def test_fp16_f16c_matches_portable_restatement():
    """the F16C conversions (ggml's x86 GGML_FP32_TO_FP16 / GGML_FP16_TO_FP32) and the portable RNE
    restatement agree on every fp16 pattern and a strided sweep of fp32 patterns + rounding edges"""
    assert O.lib().orc_fp16_selfcheck(4099) == 0


def test_q4_0_constant_block_known_answer():
    # all-constant weights w: max = w, d = -w/8 -> every code = min(15, (int)(-8 + 8.5)) = 0 -> value -8*d = w
    x = np.full((1, 64), 0.75, dtype=np.float32)
    q = O.quantize(x, "q4_0_ref")
    deq = np.zeros(64, dtype=np.float32)
    O.lib().orc_dequantize_row_q4_0(O.ptr(q[0]), O.ptr(deq), 64)
    assert np.all(deq == 0.75)
    # dot with an all-ones activation: q8 scale 1/127, codes 127 -> 64 * 0.75 * (fp16(1/127)*127)
    a = O.quantize(np.ones((1, 64), dtype=np.float32), "q8_0")
    d_a = np.float32(np.float16(np.float32(1.0) / np.float32(127.0)))
    s = O.vec_dot(O.Q4_0, q[0], a[0], 64)
    # per lane per block: 4*(-8)*127 * d_w*d_a with d_w = -0.09375 -> exact in fp32
    lane = np.float32(-0.09375) * d_a
    acc = np.zeros(8, dtype=np.float32)
    for _ in range(2):
        acc = (lane * np.float32(-8 * 127 * 4) + acc).astype(np.float32)
    assert s == np.float32(((acc[0] + acc[4]) + (acc[2] + acc[6])) + ((acc[1] + acc[5]) + (acc[3] + acc[7])))
    assert abs(s - 64 * 0.75) < 0.05


def test_quantize_q8_0_avx2_semantics():
    # AVX2 path: id = 127/amax and round-half-even; scalar reference: id = 1/d and roundf
    x = np.zeros((1, 32), dtype=np.float32)
    x[0, 0] = 127.0
    x[0, 1] = 0.5
    x[0, 2] = 1.5
    x[0, 3] = -2.5
    q = O.quantize(x, "q8_0")
    vals = q[0, 2:].view(np.int8)
    assert list(vals[:4]) == [127, 0, 2, -2]          # ties to even
    qr = O.quantize(x, "q8_0_ref")
    assert list(qr[0, 2:].view(np.int8)[:4]) == [127, 1, 2, -3]  # ties away from zero


@pytest.mark.parametrize("wtype", [O.Q4_0, O.Q8_0])
def test_vec_dot_ordered_equals_avx2(wtype):
    rng = np.random.default_rng(1)
    for k in (32, 256, 2048, 16384):
        W = O.quantize((rng.standard_normal((4, k)) * 0.05).astype(np.float32),
                       "q4_0_ref" if wtype == O.Q4_0 else "q8_0_ref")
        A = O.quantize(rng.standard_normal((4, k)).astype(np.float32), "q8_0")
        for r in range(4):
            a = O.vec_dot(wtype, W[r], A[r], k, avx2=False)
            b = O.vec_dot(wtype, W[r], A[r], k, avx2=True)
            assert np.float32(a).view(np.uint32) == np.float32(b).view(np.uint32)


def test_vec_dot_f16_ordered_equals_avx2():
    rng = np.random.default_rng(2)
    for k in (32, 256, 544, 2080):
        x = rng.standard_normal(k).astype(np.float16).view(np.uint16)
        y = rng.standard_normal(k).astype(np.float16).view(np.uint16)
        a = O.vec_dot(O.F16, x, y, k, avx2=False)
        b = O.vec_dot(O.F16, x, y, k, avx2=True)
        assert np.float32(a).view(np.uint32) == np.float32(b).view(np.uint32)
        ref = float(np.dot(x.view(np.float16).astype(np.float64), y.view(np.float16).astype(np.float64)))
        assert abs(a - ref) <= 1e-4 * max(1.0, abs(ref))


def test_lane_sums_known_answer():
    w = O.quantize(np.arange(32, dtype=np.float32)[None] - 16.0, "q8_0_ref")[0]
    a = O.quantize(np.ones((1, 32), dtype=np.float32), "q8_0")[0]
    lanes = np.zeros(8, dtype=np.int32)
    O.lib().orc_block_lane_sums(O.Q8_0, O.ptr(w), O.ptr(a), O.ptr(lanes))
    wq = w[2:].view(np.int8).astype(np.int32)
    assert list(lanes) == [int(wq[4 * l:4 * l + 4].sum() * 127) for l in range(8)]


def test_softmax_rows_sum_to_one_and_mask():
    L = O.lib()
    O.lib().orc_init_tables(0)
    x = np.linspace(-3, 3, 64).astype(np.float32)
    mask = np.zeros(64, dtype=np.float32)
    mask[40:] = -np.inf
    y = np.zeros(64, dtype=np.float32)
    L.orc_soft_max_row(O.ptr(x), O.ptr(mask), O.ptr(y), 64, 1.0)
    assert np.all(y[40:] == 0)
    assert abs(y.sum() - 1.0) < 2e-3
    ref = np.exp(x[:40] - x[:40].max())
    ref /= ref.sum()
    assert np.abs(y[:40] - ref).max() < 2e-3  # fp16 exp table


def test_rms_norm_and_rope_known_answers():
    L = O.lib()
    x = np.full(256, 2.0, dtype=np.float32)
    y = np.zeros(256, dtype=np.float32)
    L.orc_rms_norm(O.ptr(x), O.ptr(y), 256, 0.0)
    assert np.all(y == 1.0)
    # rope at position 0 is the identity; at position p pair 0 rotates by p radians
    v = np.arange(256, dtype=np.float32)
    r = v.copy()
    L.orc_rope_neox(O.ptr(r), 256, 1, 0, 10000.0)
    assert np.array_equal(r, v)
    r = v.copy()
    L.orc_rope_neox(O.ptr(r), 256, 1, 3, 10000.0)
    c, s = np.cos(np.float32(3)), np.sin(np.float32(3))
    assert abs(r[0] - (v[0] * c - v[128] * s)) < 1e-4 and abs(r[128] - (v[0] * s + v[128] * c)) < 1e-4


def test_gelu_table():
    L = O.lib()
    O.lib().orc_init_tables(0)
    x = np.linspace(-6, 6, 101).astype(np.float32)
    y = np.zeros_like(x)
    L.orc_gelu(O.ptr(x), O.ptr(y), x.size)
    ref = 0.5 * x * (1 + np.tanh(0.7978845608 * x * (1 + 0.044715 * x * x)))
    assert np.abs(y - ref).max() < 5e-3


def test_mul_mat_thread_split_invariant():
    """src/hpc.cpp:245-273 row split: results independent of the worker count and pool kind."""
    rng = np.random.default_rng(3)
    rows, k, ncols = 37, 256, 3
    W = O.quantize((rng.standard_normal((rows, k)) * 0.05).astype(np.float32), "q4_0_ref")
    X = rng.standard_normal((ncols, k)).astype(np.float32)
    wdata, rs = O.mul_mat_init(O.Q4_0, X)
    outs = []
    for pool in (0, 1):  # the reference task pool and the bench's spin fork-join pool
        O.lib().orc_set_pool(pool)
        for nt in (1, 4, 7):
            O.lib().orc_set_threads(nt)
            outs.append(O.mul_mat(W, O.Q4_0, rows, W.shape[1], k, wdata, rs, ncols))
    O.lib().orc_set_pool(0)
    O.lib().orc_set_threads(4)
    assert all(np.array_equal(outs[0], o) for o in outs[1:])
    # and equals the per-element vec_dot
    for c in range(ncols):
        for r in range(rows):
            assert outs[0][c, r] == np.float32(O.vec_dot(O.Q4_0, W[r], wdata[c], k))


def test_tiny_model_generation_is_deterministic_and_avx2_consistent():
    cfg = O.make_config(O.TINY, n_ctx=128)
    m = O.Model(cfg)
    p = O.make_prompt(9, cfg.n_vocab)
    s1, l1 = m.generate(p, 6, avx2=True)
    s2, l2 = m.generate(p, 6, avx2=False)
    assert s1 == s2 and np.array_equal(l1, l2)
    assert np.isfinite(l1).all()


def test_prefill_equals_tokenwise_decode():
    """Batched PREFILL and token-by-token DECODE give identical logits (n_kv padding is inert)."""
    cfg = O.make_config(O.TINY, n_ctx=128)
    m = O.Model(cfg)
    p = O.make_prompt(12, cfg.n_vocab)
    m.reset()
    _, last_prefill, _ = m.inference(p, 0)
    m.reset()
    m.inference(p[:1], 0)
    for i in range(2, len(p) + 1):
        _, last, _ = m.inference(p[:i], 1)
    assert np.array_equal(last, last_prefill)


def test_graph_wiring_matches_transformers_gemma_golden():
    """Oracle forward (ggml semantics, Q8_0 weights and activations) vs the float forward of a
    locally built transformers GemmaForCausalLM on the same (dequantized) weights — fixture made by
    tests/golden/make_hf_wiring_golden.py.  Pins the graph wiring of src/gemma_model.cpp:665-747
    (embedding scale, '+1' RMSNorm weights, RoPE-NEOX pairs, MQA, q scale, GeGLU, residuals, tied
    output); the tolerance covers Q8_0 activation quantization only (measured: corr >= 0.9998,
    max |diff| 0.066 at logit std 0.99)."""
    import os
    g = np.load(os.path.join(os.path.dirname(__file__), "golden", "hf_wiring_tiny.npz"))
    keys = ("n_layer", "n_embd", "n_head", "n_head_kv", "head_dim", "n_ff", "n_vocab")
    shape = dict(zip(keys, (int(v) for v in g["shape"])))
    m = O.Model(O.make_config(shape, n_ctx=64, wtype=O.Q8_0, seed=int(g["seed"][0])))
    _, _, ours = m.inference(g["prompt"], 0, want_all=True)
    ref = g["logits"]
    corr = min(np.corrcoef(ours[i], ref[i])[0, 1] for i in range(len(ref)))
    assert corr > 0.999, corr
    assert np.abs(ours - ref).max() < 0.15 * ref.std()
    assert (ours.argmax(1) == ref.argmax(1)).mean() >= 0.9
