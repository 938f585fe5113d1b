"""The exact prefill GEMM on the K = 4 multi-block MFMA (prefill.hip k_gemm_x4, hpc_set_gemm_x4(1)):
bit-identical to mul_mat's AVX2 lane order (the oracle's restatement of src/hpc.cpp:15-41 over
ggml's vec_dot_q4_0_q8_0 / q8_0_q8_0) at ragged shapes, and whole exact prefills (every prompt row's
logits, the decode that continues from the cache) equal to the oracle and to the W32 form."""
import numpy as np
import pytest

import oracle_ctypes as O
from test_gpu_prefill import _gemm, _prefill_exact_case

gpu = pytest.mark.gpu


DEFAULT = 3  # hpc_set_gemm_x4's default form


@pytest.fixture(params=[0, 1, 2, 3, 4], ids=["w32", "x4_32x64", "x4_64x32", "x4_i8", "x4_64x32_i8"])
def x4(request):
    """every exact GEMM form: the lane-masked W32 kernel (0), the K = 4 kernel with 32 rows x 64
    tokens (1, the default) and 64 x 32 (2)"""
    import gemma_hip as G
    G.lib().hpc_set_gemm_x4(request.param)
    yield request.param
    G.lib().hpc_set_gemm_x4(DEFAULT)


@gpu
@pytest.mark.parametrize("wtype", [O.Q4_0, O.Q8_0], ids=["q4_0", "q8_0"])
@pytest.mark.parametrize("rows,K,T", [(64, 256, 64), (100, 512, 37), (72, 2048, 130), (2560, 2048, 96),
                                      (256, 16384, 70), (40, 96, 3), (8, 32, 1), (96, 1312, 65)])
def test_gemm_x4_bit_identical(x4, wtype, rows, K, T):
    import gemma_hip as G
    L = G.lib()
    rng = np.random.default_rng(rows * 13 + K + T)
    Wf = (rng.standard_normal((rows, K)) * 0.05).astype(np.float32)
    W = O.quantize(Wf, "q4_0_ref" if wtype == O.Q4_0 else "q8_0_ref")
    X = (rng.standard_normal((T, K)) * rng.uniform(0.1, 3.0, (T, 1))).astype(np.float32)
    X[0, :min(37, K)] = 0.0
    r, Y, xq, da = _gemm(L, wtype, W, X, rows, K, T, exact=True)
    assert r == 0, G.last_error()
    wdata, rs = O.mul_mat_init(wtype, X)
    ref = O.mul_mat(W, wtype, rows, W.shape[1], K, wdata, rs, T)
    assert np.array_equal(Y.view(np.uint32), ref.view(np.uint32)), np.abs(Y - ref).max()


@gpu
def test_gemm_x4_extreme_blocks(x4):
    """the isum bounds: Q8_0 weights and activations at +-127 / -128 (4 products of 128*128 = 65,536),
    Q4_0 nibbles 0 / 15 (-8 / +7), all in one row"""
    import gemma_hip as G
    L = G.lib()
    rows, K, T = 16, 256, 17
    for wtype, q in ((O.Q8_0, "q8_0_ref"), (O.Q4_0, "q4_0_ref")):
        Wf = np.zeros((rows, K), np.float32)
        Wf[0::2] = 1.0
        Wf[1::2] = -1.0
        Wf[3, ::3] = 0.01
        W = O.quantize(Wf, q)
        X = np.zeros((T, K), np.float32)
        X[0::2] = -1.0
        X[1::2] = 1.0
        X[5, 7::5] = 0.3
        r, Y, _, _ = _gemm(L, wtype, W, X, rows, K, T, exact=True)
        assert r == 0, G.last_error()
        wdata, rs = O.mul_mat_init(wtype, X)
        ref = O.mul_mat(W, wtype, rows, W.shape[1], K, wdata, rs, T)
        assert np.array_equal(Y.view(np.uint32), ref.view(np.uint32)), (wtype, np.abs(Y - ref).max())


@gpu
def test_prefill_exact_x4_gemma2b_shapes(x4):
    _prefill_exact_case(dict(O.GEMMA_2B), 96, 256, n_decode=2)


@gpu
def test_prefill_exact_x4_q8_0_gqa(x4):
    _prefill_exact_case(dict(O.TINY, n_head=4, n_head_kv=2), 70, 256, wtype=O.Q8_0)


@gpu
def test_prefill_x4_full_size_equals_w32():
    """BASELINE config 3 at full size (Gemma-2B, T = 2048): every prompt row's logits from the K = 4
    form equal the lane-masked W32 form's (both bit-exact restatements; a size-independent check)."""
    import gemma_hip as G
    T = 2048
    shape = dict(O.GEMMA_2B)
    prompt = O.make_prompt(T, shape["n_vocab"], seed=2)
    out = []
    try:
        for on in (0, 1, 2, 3, 4):
            G.lib().hpc_set_gemm_x4(on)
            e = G.Engine(shape, n_ctx=T + 64, device=0)
            e.begin(prompt)
            tok, last = e.prefill(T)
            out.append((tok, last, e.step(2, want_logits=True, use_graph=True)))
            e.close()
    finally:
        G.lib().hpc_set_gemm_x4(DEFAULT)
    for o in out[1:]:
        assert out[0][0] == o[0]
        assert np.array_equal(out[0][1].view(np.uint32), o[1].view(np.uint32))
        assert np.array_equal(out[0][2].view(np.uint32), o[2].view(np.uint32))
