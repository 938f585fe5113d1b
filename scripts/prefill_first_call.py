"""Engine prefill at T = 128: the first call on a fresh engine vs warm calls (one-time costs such as
code-object loading show up in the first).  usage: python scripts/prefill_first_call.py"""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "gemma.ggml_amd", "python"))
sys.path.insert(0, ROOT)
import gemma_hip as G  # noqa: E402
from bench import GEMMA_2B, make_prompt  # noqa: E402

t0 = time.perf_counter()
e = G.Engine(GEMMA_2B, n_ctx=512)
e.L.gemma_engine_sync(e.h)
print(f"create {1e3 * (time.perf_counter() - t0):.1f} ms", flush=True)
p = make_prompt(128, GEMMA_2B["n_vocab"])
for i in range(4):
    e.begin(p)
    e.L.gemma_engine_sync(e.h)
    t0 = time.perf_counter()
    e.prefill(128)
    e.L.gemma_engine_sync(e.h)
    print(f"prefill T=128 call {i}: {1e3 * (time.perf_counter() - t0):.2f} ms", flush=True)
e.close()
