"""GPU parity of the K-quant matvec: mul_mat with Q4_K / Q6_K src0 and Q8_K wdata
through the C-ABI drop-in, bit-identical to the oracle's ggml AVX2-order vec_dot (every row, every
column; ragged row counts, several super-block counts, an all-zero activation block)."""
import numpy as np
import pytest

import oracle_ctypes as O

gpu = pytest.mark.gpu


@gpu
@pytest.mark.parametrize("wtype", [O.Q4_K, O.Q6_K], ids=["q4_K", "q6_K"])
@pytest.mark.parametrize("rows,K,ncols", [(8, 256, 1), (100, 2048, 3), (37, 16384, 1), (2048, 2048, 2),
                                          (1000, 4096, 1),
                                          # >= 4 columns: the T-column kernel (4 columns share each
                                          # weight load), ragged column tails, > 64 KiB of LDS
                                          (72, 2048, 4), (300, 4096, 7), (64, 16384, 9),
                                          # >= 8 columns: the MFMA GEMM (prefill_kq.hip) on ggml's
                                          # row-major blocks; ragged row / column tiles
                                          (100, 2048, 8), (130, 4096, 65), (64, 16384, 33), (257, 256, 70)])
def test_kquant_mul_mat_bit_exact(wtype, rows, K, ncols):
    import gemma_hip as G
    G.lib().hpc_set_error_mode(0)
    W = O.synth_kquant(wtype, rows * 31 + K, rows, K)
    rng = np.random.default_rng(rows + K)
    X = (rng.standard_normal((ncols, K)) * rng.uniform(0.1, 4.0, (ncols, 1))).astype(np.float32)
    X[0, :256] = 0.0  # one all-zero Q8_K block (d = 0)
    wdata, rs = O.mul_mat_init(wtype, X)
    ref = O.mul_mat(W, wtype, rows, W.shape[1], K, wdata, rs, ncols)
    got = G.mul_mat(W, wtype, rows, W.shape[1], K, wdata, rs, ncols)
    bad = np.nonzero(got.view(np.uint32) != ref.view(np.uint32))
    assert bad[0].size == 0, (bad[0][:5], bad[1][:5], np.abs(got - ref).max())


@gpu
def test_kquant_rejects_bad_k():
    import gemma_hip as G
    L = G.lib()
    L.hpc_set_error_mode(0)
    W = O.synth_kquant(O.Q4_K, 1, 8, 256)
    X = np.ones((1, 256), np.float32)
    wdata, rs = O.mul_mat_init(O.Q4_K, X)
    G.mul_mat(W, O.Q4_K, 8, W.shape[1], 200, wdata, rs, 1)
    assert "K-quant" in G.last_error()


def _extreme_blocks(wtype, W, K):
    """Overwrite rows of W (ggml row-major blocks) with the extreme super-blocks of the exactness
    argument in prefill_kq.hip: Q6_K (q6 - 32) * scale = 4096 (the 2^24 lane-sum bound with
    activations of -128), odd products just below it, and mixed signs; Q4_K all nibbles 15 with
    six-bit scales and mins 63."""
    W = W.copy()
    nsb = K // 256
    for r in range(W.shape[0]):
        for sb in range(nsb):
            if wtype == O.Q6_K:
                b = W[r, sb * 210:(sb + 1) * 210]
                kind = (r + sb) % 4
                if kind == 0:    # q6 = 0 -> -32, scale -128: every product 4096
                    b[:192] = 0
                    b[192:208] = np.uint8(0x80)
                elif kind == 1:  # q6 = 1 -> -31, scale -127: odd products 3937
                    b[:128] = 0x11
                    b[128:192] = 0
                    b[192:208] = np.uint8(0x81)
                elif kind == 2:  # q6 = 63 -> 31, scale 127
                    b[:192] = 0xFF
                    b[192:208] = 127
                # kind 3: the random block stays
            else:
                b = W[r, sb * 144:(sb + 1) * 144]
                if (r + sb) % 3 != 2:
                    b[4:] = 0xFF  # scales, mins 63; nibbles 15
    return W


@gpu
@pytest.mark.parametrize("wtype", [O.Q4_K, O.Q6_K], ids=["q4_K", "q6_K"])
def test_kquant_mul_mat_extreme_blocks(wtype):
    # lane sums at the f16/fp32 exactness bounds the MFMA GEMM relies on (and the dot4 matvec for
    # fewer columns): columns of all-equal activations quantize to -128 everywhere
    import gemma_hip as G
    G.lib().hpc_set_error_mode(0)
    rows, K = 96, 4096
    W = _extreme_blocks(wtype, O.synth_kquant(wtype, 7, rows, K), K)
    rng = np.random.default_rng(5)
    for ncols in (3, 12):
        X = rng.standard_normal((ncols, K)).astype(np.float32)
        X[0] = 1.0
        X[1] = -1.0
        X[2, ::2] = 1.0
        wdata, rs = O.mul_mat_init(wtype, X)
        ref = O.mul_mat(W, wtype, rows, W.shape[1], K, wdata, rs, ncols)
        got = G.mul_mat(W, wtype, rows, W.shape[1], K, wdata, rs, ncols)
        bad = np.nonzero(got.view(np.uint32) != ref.view(np.uint32))
        assert bad[0].size == 0, (ncols, bad[0][:5], bad[1][:5], np.abs(got - ref).max())


@gpu
@pytest.mark.parametrize("wtype", [O.Q4_K, O.Q6_K], ids=["q4_K", "q6_K"])
def test_kquant_gemm_extreme_activation_scales(wtype):
    """the Q4_K MFMA GEMM folds 2^24 into x.d (its A operand is f16 denormals); it rounds
    d = y.d * x.d unscaled, as ggml does, and scales it by 2^24 afterwards, so columns whose Q8_K scales
    make d subnormal (column 0 here: |d| ~ 1e-40) still give ggml's bits.  The documented bound is
    |y.d * x.d| < 2^104 (the largest column here reaches 9.8e30 of 2.0e31).  >= 8 columns: the GEMM."""
    import gemma_hip as G
    G.lib().hpc_set_error_mode(0)
    rows, K = 64, 2048
    W = O.synth_kquant(wtype, 11, rows, K)
    rng = np.random.default_rng(9)
    scales = np.array([1e-36, 3e-38, 1e-33, 1e-30, 1e-20, 1.0, 1e20, 1e30, 1e33, 2e34, 1e35, 1.0], np.float32)
    X = (rng.standard_normal((len(scales), K)) * scales[:, None]).astype(np.float32)
    X[5, 256:512] *= np.float32(1e-37)  # one super-block tiny inside an ordinary column
    wdata, rs = O.mul_mat_init(wtype, X)
    ref = O.mul_mat(W, wtype, rows, W.shape[1], K, wdata, rs, len(scales))
    got = G.mul_mat(W, wtype, rows, W.shape[1], K, wdata, rs, len(scales))
    assert np.isfinite(ref).all()
    bad = np.nonzero(got.view(np.uint32) != ref.view(np.uint32))
    assert bad[0].size == 0, (bad[0][:5], bad[1][:5])
