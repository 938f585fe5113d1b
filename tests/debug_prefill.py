"""Diagnostic: prefill vs oracle logits error per prompt length (TINY shape)."""
import sys

import numpy as np

sys.path.insert(0, "gemma.ggml_amd/python")
sys.path.insert(0, "tests")
import gemma_hip as G
import oracle_ctypes as O

shape = dict(O.TINY)
for n in [int(v) for v in sys.argv[1:]] or [1, 2, 3, 5, 8, 16, 17, 31, 32, 33, 40, 64, 65]:
    prompt = O.make_prompt(n, shape["n_vocab"])
    m = O.Model(O.make_config(shape, n_ctx=256))
    tok_ref, last_ref, all_ref = m.inference(prompt, 0, want_all=True)
    e = G.Engine(shape, n_ctx=256, device=0)
    e.begin(prompt)
    tok, last, allv = e.prefill(n, want_all=True)
    err = np.abs(allv - all_ref).max(axis=1) / np.abs(all_ref).max(axis=1)
    print(n, "max err %.2e" % err.max(), "rows>1e-4:", np.flatnonzero(err > 1e-4).tolist()[:20])
    e.close(); m.close()
