"""K-quant (Q4_K_M layout) batched exact prefill timing at prompt length T: one untimed pass, then
`reps` timed passes.  usage: python scripts/kq_prefill.py [T] [reps]"""
import os
import sys
import time

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "gemma.ggml_amd", "python"))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
import gemma_hip as G  # noqa: E402
from bench import GEMMA_2B, make_prompt  # noqa: E402

T = int(sys.argv[1]) if len(sys.argv) > 1 else 2048
reps = int(sys.argv[2]) if len(sys.argv) > 2 else 2
e = G.Engine(GEMMA_2B, n_ctx=T + 64, wtype=G.GGML_TYPE_Q4_K)
p = make_prompt(T, GEMMA_2B["n_vocab"], seed=2)
for r in range(reps + 1):
    e.begin(p)
    e.L.gemma_engine_sync(e.h)
    t0 = time.perf_counter()
    tok = e.prefill(T)[0]
    print(f"rep {r}: {(time.perf_counter() - t0) * 1e3:.2f} ms ({T / (time.perf_counter() - t0):.0f} tok/s) token {tok}",
          flush=True)
e.close()
