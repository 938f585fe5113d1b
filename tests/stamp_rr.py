"""Diagnostic: phase timeline of the round-pipelined down matvec inside a decode step (stamps build).
Stamps (10 ns ticks): 0 start, 1 image built, 2..9 loader wave 0 done with round r, 10 image built, 11 weights
issued, 12 carrier done with round 5, 13 carrier done with the last round, 14 epilogue stored, 15 loader 7 done
with the last round."""
import os
import sys

import numpy as np

sys.path.insert(0, "gemma.ggml_amd/python")
sys.path.insert(0, ".")
import gemma_hip as G  # noqa: E402
from bench import GEMMA_2B, make_prompt  # noqa: E402

e = G.Engine(GEMMA_2B, n_ctx=512, device=0)
p = e.plan()
p["down"] = (9, 1, 1)
if os.environ.get("QKV9"):
    p["qkv"] = (9, 1, 0)
e.set_plan(p)
e.begin(make_prompt(128, GEMMA_2B["n_vocab"]))
e.step(140, use_graph=True)
for rep in range(3):
    st = e.stamp_step(9).astype(np.int64)
r = st[4]
r = r[r[:, 0] != 0]
t0 = r[:, 0].min()
rel = (r - t0) * 10
rel[r == 0] = -1
names = ["start", "barrier"] + [f"r{i}" for i in range(8)] + ["imgbuilt", "wissued", "c5", "c7", "epi", "l7last"]
print("WGs", len(r))
for q in (10, 50, 90, 100):
    print(f"p{q:3d} " + " ".join(f"{n}={int(v)}" for n, v in zip(names, np.percentile(rel, q, axis=0))))
e.close()
