"""Diagnostic: phase timeline of the fused layer-front kernel inside a decode step (stamps build).
Stamps (10 ns): 0 start, 1 qkv tile(s) done, 2 qkv signalled, 3 attention poll done, 4 attention
done, 5 attention signalled, 6 attn-out done."""
import sys

import numpy as np

sys.path.insert(0, "gemma.ggml_amd/python")
sys.path.insert(0, ".")
import gemma_hip as G  # noqa: E402
from bench import GEMMA_2B, make_prompt  # noqa: E402

e = G.Engine(GEMMA_2B, n_ctx=512, device=0)
p = e.plan()
p.update(qkv=(9, 1, 0), attn_out=(9, 1, 1), attention=0)
e.set_plan(p)
e.set_fuse(1)
e.begin(make_prompt(128, GEMMA_2B["n_vocab"]))
e.step(140, use_graph=True)
for rep in range(3):
    st = e.stamp_step(9).astype(np.int64)
r = st[0][:256]
t0 = r[r[:, 0] != 0, 0].min()
rel = np.where(r != 0, (r - t0) * 10, -1)
names = ["start", "qkv", "qsig", "apoll", "att", "asig", "o"]
for lo, hi, nm in ((0, 8, "attention WGs"), (8, 256, "attn-out WGs"), (192, 256, "2-tile qkv WGs")):
    sub = rel[lo:hi, :7]
    print(nm)
    for q in (0, 50, 100):
        print(f"  p{q:3d} " + " ".join(f"{n}={int(v)}" for n, v in zip(names, np.percentile(sub, q, axis=0))))
print("err", e.set_fuse(-1))
e.close()
