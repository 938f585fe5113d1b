"""Profile target: batched prefill of a T-token synthetic prompt on Gemma-2B shapes (one warm-up
pass, then `reps` timed passes).  usage: prof_prefill.py [T] [exact 1/0] [reps]"""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "gemma.ggml_amd", "python"))
sys.path.insert(0, ROOT)
import gemma_hip as G  # noqa: E402
from bench import GEMMA_2B, make_prompt  # noqa: E402

T = int(sys.argv[1]) if len(sys.argv) > 1 else 2048
exact = (sys.argv[2] != "0") if len(sys.argv) > 2 else True
reps = int(sys.argv[3]) if len(sys.argv) > 3 else 2
if os.environ.get("X4"):  # the exact GEMM form (hpc_set_gemm_x4: 0 W32, 1 K = 4 (default), 2 K = 4 64 x 32)
    G.lib().hpc_set_gemm_x4(int(os.environ["X4"]))
e = G.Engine(GEMMA_2B, n_ctx=T + 64, device=0)
p = make_prompt(T, GEMMA_2B["n_vocab"], seed=2)
for r in range(reps + 1):
    e.begin(p)
    e.L.gemma_engine_sync(e.h)
    t0 = time.perf_counter()
    tok = e.prefill(T, exact=exact)[0]
    print(f"rep {r}: {(time.perf_counter() - t0) * 1e3:.2f} ms token {tok}", flush=True)
e.close()
