"""ggml graph executor, K-quant ops one node at a time through the ggml API (include/ggml.h, via
ctypes): get_rows of Q4_0 / Q8_0 / Q4_K / Q6_K rows (ggml dequantize_row_*) and mul_mat with Q4_K /
Q6_K src0 (device Q8_K INIT + the AVX2-lane-order K-quant dot), bit-identical to the oracle."""
import ctypes as C

import numpy as np
import pytest

import gemma_hip as G
import oracle_ctypes as O

gpu = pytest.mark.gpu


class InitParams(C.Structure):
    _fields_ = [("mem_size", C.c_size_t), ("mem_buffer", C.c_void_p), ("no_alloc", C.c_bool)]


def _api():
    L = G.lib()
    T = C.POINTER(G.GgmlTensor)
    L.ggml_init.restype = C.c_void_p
    L.ggml_init.argtypes = [InitParams]
    L.ggml_new_tensor_1d.restype = T
    L.ggml_new_tensor_1d.argtypes = [C.c_void_p, C.c_int, C.c_int64]
    L.ggml_new_tensor_2d.restype = T
    L.ggml_new_tensor_2d.argtypes = [C.c_void_p, C.c_int, C.c_int64, C.c_int64]
    L.ggml_get_rows.restype = T
    L.ggml_get_rows.argtypes = [C.c_void_p, T, T]
    L.ggml_mul_mat.restype = T
    L.ggml_mul_mat.argtypes = [C.c_void_p, T, T]
    L.ggml_new_graph.restype = C.c_void_p
    L.ggml_new_graph.argtypes = [C.c_void_p]
    L.ggml_build_forward_expand.argtypes = [C.c_void_p, T]
    L.ggml_graph_compute_with_ctx.restype = C.c_int
    L.ggml_graph_compute_with_ctx.argtypes = [C.c_void_p, C.c_void_p, C.c_int]
    return L


def _put(t, arr):
    b = np.ascontiguousarray(arr).view(np.uint8).ravel()
    C.memmove(t.contents.data, b.ctypes.data, b.size)


def _get(t, n):
    return np.ctypeslib.as_array((C.c_float * n).from_address(t.contents.data)).copy()


def _compute(L, ctx, out):
    g = L.ggml_new_graph(ctx)
    L.ggml_build_forward_expand(g, out)
    assert L.ggml_graph_compute_with_ctx(ctx, g, 1) == 0, G.last_error()


@gpu
@pytest.mark.parametrize("wtype", [O.Q4_0, O.Q8_0, O.Q4_K, O.Q6_K])
def test_get_rows_dequantizes_like_ggml(wtype):
    L = _api()
    rows, K = 37, 1024
    rng = np.random.default_rng(wtype)
    if wtype in (O.Q4_K, O.Q6_K):
        w = O.synth_kquant(wtype, 5, rows, K).ravel()
    else:
        w = O.quantize(rng.standard_normal((rows, K)).astype(np.float32), "q4_0_ref" if wtype == O.Q4_0 else "q8_0_ref")
    w = w.ravel()
    rb = w.size // rows
    idx = np.array([0, 36, 5, 5, 17, 1], np.int32)
    ctx = L.ggml_init(InitParams(64 << 20, None, False))
    a = L.ggml_new_tensor_2d(ctx, wtype, K, rows)
    b = L.ggml_new_tensor_1d(ctx, 26, len(idx))  # GGML_TYPE_I32
    _put(a, w)
    _put(b, idx)
    out = L.ggml_get_rows(ctx, a, b)
    _compute(L, ctx, out)
    got = _get(out, K * len(idx)).reshape(len(idx), K)
    for r, i in enumerate(idx):
        ref = O.dequantize(wtype, w[i * rb:(i + 1) * rb], K)
        assert np.array_equal(got[r].view(np.uint32), ref.view(np.uint32)), (wtype, r)
    L.ggml_free(ctx)


@gpu
@pytest.mark.parametrize("wtype", [O.Q4_K, O.Q6_K])
@pytest.mark.parametrize("rows,K,cols", [(64, 256, 1), (200, 2048, 3), (33, 4096, 17), (2048, 16384, 2)])
def test_mul_mat_kquant_in_graph(wtype, rows, K, cols):
    L = _api()
    rng = np.random.default_rng(rows + cols)
    w = O.synth_kquant(wtype, rows * 7 + K, rows, K).ravel()
    x = rng.standard_normal((cols, K)).astype(np.float32)
    x[0, :256] = 0.0  # an all-zero super-block: Q8_K d = 0
    if cols > 1:
        x[1, 7] = -50.0  # a negative max
    ctx = L.ggml_init(InitParams(256 << 20, None, False))
    a = L.ggml_new_tensor_2d(ctx, wtype, K, rows)
    b = L.ggml_new_tensor_2d(ctx, 0, K, cols)
    _put(a, w)
    _put(b, x)
    out = L.ggml_mul_mat(ctx, a, b)
    _compute(L, ctx, out)
    got = _get(out, rows * cols).reshape(cols, rows)
    wd, rs = O.mul_mat_init(wtype, x)
    ref = O.mul_mat(w, wtype, rows, w.size // rows, K, wd, rs, cols)
    assert np.array_equal(got.view(np.uint32), ref.view(np.uint32))
    L.ggml_free(ctx)
