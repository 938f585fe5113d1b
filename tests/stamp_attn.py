"""Diagnostic: phase stamps of the decode attention kernel (s_memrealtime, 10 ns ticks)."""
import ctypes as C
import sys

import numpy as np

sys.path.insert(0, "gemma.ggml_amd/python")
import gemma_hip as G

L = G.lib()
L.gemma_test_attn_decode.restype = C.c_int
L.gemma_test_attn_decode.argtypes = [C.c_void_p] * 3 + [C.c_int] * 5 + [C.c_float] + [C.c_void_p] * 5 + [C.c_int]
mode = int(sys.argv[1]) if len(sys.argv) > 1 and sys.argv[1].isdigit() else 0
H, Hkv, hd, ctx, pos = 8, 1, 256, 512, 200
rng = np.random.default_rng(0)
qkv = rng.standard_normal((H + 2 * Hkv) * hd).astype(np.float32)
kc = rng.standard_normal(ctx * Hkv * hd).astype(np.float16).view(np.uint16)
vc = rng.standard_normal(ctx * Hkv * hd).astype(np.float16).view(np.uint16)
out = np.zeros(H * hd, np.float32)
st = np.zeros(H * 8 * 8, np.uint64)
r = L.gemma_test_attn_decode(qkv.ctypes.data, kc.ctypes.data, vc.ctypes.data, pos, H, Hkv, hd, ctx, 10000.0,
                             out.ctypes.data, None, None, None, st.ctypes.data, mode)
assert r == 0, G.last_error()
st = st.reshape(H * 8, 8).astype(np.int64)
wg_ids = np.nonzero(st[:, 0])[0]
st = st[st[:, 0] != 0]  # launched workgroups only
rel = (st[:, :8] - st[:, :1]) * 10
if "--per-wg" in sys.argv:  # every workgroup, times from the earliest start
    t0 = st[:, 0].min()
    for i, row in zip(wg_ids, st):
        print("wg %3d" % i, [int((v - t0) * 10) if v else -1 for v in row])
print("phase end times (ns) per WG [start, p1..p7] (mode %d; AH_STAMP / ATT_STAMP order)" % mode)
print("median", np.median(rel, axis=0).astype(int).tolist())
print("max   ", rel.max(axis=0).tolist())
print("WG start spread (ns)", int((st[:, 0].max() - st[:, 0].min()) * 10))
