"""Diagnostic: per-layer residual-stream error of the MFMA prefill vs the oracle (TINY, 2 layers)."""
import ctypes as C
import sys

import numpy as np

sys.path.insert(0, "gemma.ggml_amd/python")
sys.path.insert(0, "tests")
import gemma_hip as G
import oracle_ctypes as O

shape = dict(O.GEMMA_2B if "2b" in sys.argv else O.TINY)
n = int(sys.argv[1]) if len(sys.argv) > 1 else 16
prompt = O.make_prompt(n, shape["n_vocab"])
m = O.Model(O.make_config(shape, n_ctx=256))
m.inference(prompt, 0, want_all=True)
L = G.lib()
L.gemma_engine_prefill_taps.restype = C.c_int
L.gemma_engine_prefill_taps.argtypes = [C.c_void_p, C.c_void_p, C.c_int]
e = G.Engine(shape, n_ctx=256, device=0)
e.begin(prompt)
E = shape["n_embd"]
taps = np.zeros((shape["n_layer"], n, E), np.float32)
assert L.gemma_engine_prefill_taps(e.h, taps.ctypes.data, 0) == 0, G.last_error()
for il in range(shape["n_layer"]):
    ref = m.hidden(il, n)
    err = np.abs(taps[il] - ref).max(axis=1) / np.abs(ref).max(axis=1)
    print("layer", il, "row errs:", " ".join("%d:%.1e" % (i, v) for i, v in enumerate(err[:8])), "max %.1e" % err.max())
