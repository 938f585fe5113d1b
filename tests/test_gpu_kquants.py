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
                                          (72, 2048, 4), (300, 4096, 7), (64, 16384, 9)])
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
