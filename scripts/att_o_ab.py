"""A/B of the decode step with the attention + attn-out fused launch (k_attn_o) on and off, on one
engine (bench.py's config 2: Gemma-2B Q4_0, tuned plan, the 128-token prompt), interleaved reps.
usage: att_o_ab.py [reps] [steps]"""
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
steps = int(sys.argv[2]) if len(sys.argv) > 2 else 64
e = G.Engine(GEMMA_2B, n_ctx=512, device=0)
plan = e.tune(8)
p = e.plan()
if p["attn_out"][0] != 9 or not p["attn_out"][2]:
    p.update(attn_out=(9, 1, 1))
    e.set_plan(p)
print("plan", e.plan(), flush=True)
prompt = make_prompt(128, GEMMA_2B["n_vocab"])
res = {0: [], 1: []}
toks = {}
for r in range(reps):
    for on in (0, 1):
        e.set_att_o(on)
        e.begin(prompt)
        e.step(128 + 8, use_graph=True)
        e.sync()
        t0 = time.perf_counter()
        e.step(steps, use_graph=True)
        e.sync()
        dt = time.perf_counter() - t0
        res[on].append(steps / dt)
        toks[on] = list(e.tokens()[128:128 + 8 + steps])
        print(f"rep {r} att_o {on}: {steps / dt:.1f} tok/s  kernels/token {e.graph_kernels()}", flush=True)
print("att_o off", [round(v, 1) for v in res[0]], "on", [round(v, 1) for v in res[1]],
      "tokens equal", toks[0] == toks[1], flush=True)
e.close()
