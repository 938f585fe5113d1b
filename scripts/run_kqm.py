"""Profile target: Gemma-2B in the Q4_K_M layout (Q4_K / Q6_K layers, Q6_K output), greedy decode.
usage: python scripts/run_kqm.py [steps] [prompt tokens (16; the bench leg's positions: 128 + warmup 8)]"""
import os
import sys
import time

import torch  # noqa: F401  (the HIP runtime bench.py runs on)

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "gemma.ggml_amd", "python"))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
import gemma_hip as G  # noqa: E402
from bench import GEMMA_2B, make_prompt  # noqa: E402

steps = int(sys.argv[1]) if len(sys.argv) > 1 else 32
n_prompt = int(sys.argv[2]) if len(sys.argv) > 2 else 16
e = G.Engine(GEMMA_2B, n_ctx=512, wtype=G.GGML_TYPE_Q4_K)
e.begin(make_prompt(n_prompt, GEMMA_2B["n_vocab"]))
e.step(n_prompt + (4 if n_prompt == 16 else 8), use_graph=True)
e.L.gemma_engine_sync(e.h)
t0 = time.perf_counter()
e.step(steps, use_graph=True)
e.L.gemma_engine_sync(e.h)
dt = time.perf_counter() - t0
import zlib  # noqa: E402
toks = e.tokens()
print(f"q4_k_m decode {steps / dt:.1f} tok/s ({dt / steps * 1e3:.3f} ms/token), prompt {n_prompt}, "
      f"tokens crc {zlib.crc32(toks.tobytes()):08x}", flush=True)
e.close()
