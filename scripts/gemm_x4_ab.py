"""A/B of the exact T = 2048 Gemma-2B Q4_0 prefill with the W32 GEMM (hpc_set_gemm_x4(0)) and the
K = 4 multi-block forms (1: 32x64, 2: 64x32), interleaved reps on one engine.  usage: gemm_x4_ab.py [reps] [T] [modes, e.g. 0,1,3]"""
import os
import sys
import time

import torch  # noqa: F401  (the runtime bench.py runs on)

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "gemma.ggml_amd", "python"))
sys.path.insert(0, ROOT)
import gemma_hip as G  # noqa: E402
from bench import GEMMA_2B, make_prompt  # noqa: E402

reps = int(sys.argv[1]) if len(sys.argv) > 1 else 3
T = int(sys.argv[2]) if len(sys.argv) > 2 else 2048
MODES = [int(m) for m in sys.argv[3].split(",")] if len(sys.argv) > 3 else [0, 1, 3]
e = G.Engine(GEMMA_2B, n_ctx=T + 64, device=0)
p = make_prompt(T, GEMMA_2B["n_vocab"], seed=2)
res = {m: [] for m in MODES}
toks = {}
for r in range(reps + 1):
    for on in MODES:
        G.lib().hpc_set_gemm_x4(on)
        e.begin(p)
        e.sync()
        t0 = time.perf_counter()
        tok = e.prefill(T)[0]
        dt = time.perf_counter() - t0
        toks[on] = tok
        if r:
            res[on].append(dt * 1e3)
        print(f"rep {r} x4 {on}: {dt * 1e3:.2f} ms token {tok}", flush=True)
G.lib().hpc_set_gemm_x4(3)  # the default form
NAMES = {0: "W32", 1: "x4 32x64", 2: "x4 64x32", 3: "x4 32x64 int8-staged", 4: "x4 64x32 int8-staged"}
print(" ".join(f"{NAMES[m]} ms {[round(v, 2) for v in res[m]]}" for m in MODES),
      "tokens equal", len(set(toks.values())) == 1)
e.close()
