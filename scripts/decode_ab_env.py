"""Decode tok/s of the default engine (64-step graph replays after a 128-token prompt), for A/B runs
of the same build under different environments: python scripts/decode_ab_env.py [steps] [reps]"""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "gemma.ggml_amd", "python"))
sys.path.insert(0, ROOT)
import gemma_hip as G  # noqa: E402
from bench import GEMMA_2B, make_prompt  # noqa: E402

steps = int(sys.argv[1]) if len(sys.argv) > 1 else 64
reps = int(sys.argv[2]) if len(sys.argv) > 2 else 3
e = G.Engine(GEMMA_2B, n_ctx=512)
e.tune(8)
p = make_prompt(128, GEMMA_2B["n_vocab"])
for r in range(reps):
    e.begin(p)
    e.step(len(p) + 8, use_graph=True)
    e.L.gemma_engine_sync(e.h)
    t0 = time.perf_counter()
    e.step(steps, use_graph=True)
    e.L.gemma_engine_sync(e.h)
    dt = time.perf_counter() - t0
    print(f"rep {r}: {steps / dt:.1f} tok/s ({dt / steps * 1e3:.4f} ms/token) env HIP_FORCE_DEV_KERNARG="
          f"{os.environ.get('HIP_FORCE_DEV_KERNARG')}", flush=True)
e.close()
