"""GPU per-op parity: single kernels of the decode step against the oracle's restatement."""
import ctypes as C

import numpy as np
import pytest

import oracle_ctypes as O

gpu = pytest.mark.gpu


def _attn_case(rng, pos, H, Hkv, hd, ctx, scale_q=1.0):
    qkv = (rng.standard_normal((H + 2 * Hkv) * hd) * scale_q).astype(np.float32)
    kvw = Hkv * hd
    kc = np.zeros(ctx * kvw, dtype=np.uint16)
    vc = np.zeros(ctx * kvw, dtype=np.uint16)
    # history positions < pos hold fp16 keys/values
    kc[: pos * kvw] = rng.standard_normal(pos * kvw).astype(np.float16).view(np.uint16)
    vhist = rng.standard_normal((kvw, ctx)).astype(np.float16).view(np.uint16)
    vhist[:, pos:] = 0
    vc[:] = vhist.ravel()
    return qkv, kc, vc


@gpu
@pytest.mark.parametrize("mode", [0, 1, 2, 3], ids=["per_head", "split", "per_head_d2", "per_head_d4"])
@pytest.mark.parametrize("H,Hkv", [(8, 1), (2, 1), (4, 2), (16, 16)])
def test_attn_decode_bitexact(H, Hkv, mode):
    import gemma_hip as G
    L = G.lib()
    L.gemma_test_attn_decode.restype = C.c_int
    L.gemma_test_attn_decode.argtypes = [C.c_void_p] * 3 + [C.c_int] * 5 + [C.c_float] + [C.c_void_p] * 5 + [C.c_int]
    OL = O.lib()
    OL.orc_attn_decode.argtypes = [C.c_void_p] * 3 + [C.c_int] * 5 + [C.c_float] + [C.c_void_p] * 4
    hd, ctx = 256, 512
    rng = np.random.default_rng(H * 100 + Hkv)
    fails = []
    for pos in list(range(0, 70)) + [127, 128, 255, 300, 480, 510]:
        for scale_q in (0.5, 4.0):
            qkv, kc, vc = _attn_case(rng, pos, H, Hkv, hd, ctx, scale_q)
            k1, v1, k2, v2 = kc.copy(), vc.copy(), kc.copy(), vc.copy()
            ref = np.zeros(H * hd, dtype=np.float32)
            got = np.zeros(H * hd, dtype=np.float32)
            w1 = np.zeros(H * ctx, np.float32); w2 = np.zeros(H * ctx, np.float32)
            p1 = np.zeros(H * ctx, np.uint16); p2 = np.zeros(H * ctx, np.uint16)
            OL.orc_attn_decode(qkv.ctypes.data, k1.ctypes.data, v1.ctypes.data, pos, H, Hkv, hd, ctx, 10000.0,
                               ref.ctypes.data, w1.ctypes.data, p1.ctypes.data, None)
            r = L.gemma_test_attn_decode(qkv.ctypes.data, k2.ctypes.data, v2.ctypes.data, pos, H, Hkv, hd, ctx,
                                         10000.0, got.ctypes.data, w2.ctypes.data, p2.ctypes.data, None, None, mode)
            assert r == 0, G.last_error()
            assert np.array_equal(k1, k2) and np.array_equal(v1, v2), f"cache update differs at pos {pos}"
            nd = int((got.view(np.uint32) != ref.view(np.uint32)).sum())
            if nd:
                n_kv = min(ctx, 32 * ((pos + 1) // 32 + 1))
                w1 = w1.reshape(H, ctx)[:, :n_kv]; w2 = w2.reshape(H, ctx)[:, :n_kv]
                p1 = p1.reshape(H, ctx)[:, :n_kv]; p2 = p2.reshape(H, ctx)[:, :n_kv]
                wd = np.argwhere(w1.view(np.uint32) != w2.view(np.uint32))
                pd = np.argwhere(p1 != p2)
                info = dict(w_diffs=wd[:3].tolist(), p_diffs=pd[:3].tolist())
                if len(pd):
                    h, j = pd[0]
                    info["p_vals"] = (int(p1[h, j]), int(p2[h, j]), float(w1[h, j]), float(w2[h, j]),
                                      float(w1[h].max()), float(w2[h].max()))
                fails.append((pos, scale_q, nd, float(np.abs(got - ref).max()), info))
    assert not fails, fails[:10]


@gpu
def test_exp_f16_matches_table():
    """The attention softmax computes ggml's table_exp_f16 entry (fp16(expf(x)), ggml_init) as
    fp16(f32(exp(double x))); it must equal the glibc-expf table for every input it can see
    (x = f16(w - max) <= 0) — checked here for all non-positive codes, on the device."""
    import gemma_hip as G
    L = G.lib()
    L.gemma_test_exp_f16.restype = C.c_int
    L.gemma_test_exp_f16.argtypes = [C.c_void_p]
    got = np.zeros(65536, np.uint16)
    assert L.gemma_test_exp_f16(got.ctypes.data) == 0, G.last_error()
    libm = C.CDLL("libm.so.6")
    libm.expf.restype = C.c_float
    libm.expf.argtypes = [C.c_float]
    x = np.arange(65536, dtype=np.uint16).view(np.float16).astype(np.float32)
    sel = np.flatnonzero((x <= 0) & np.isfinite(x))
    ref = np.array([libm.expf(float(x[i])) for i in sel], np.float32).astype(np.float16).view(np.uint16)
    bad = sel[got[sel] != ref]
    assert len(bad) == 0, [(int(i), int(got[i])) for i in bad[:8]]
