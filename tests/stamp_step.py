"""Diagnostic: in-step phase timeline of one layer's kernels (s_memrealtime stamps, 10 ns ticks).

Prints, per kernel, the workgroup start spread and the median / max time of each phase end
relative to the kernel's first workgroup start, and the gap from the previous kernel's last
workgroup end to this kernel's first start."""
import sys

import numpy as np

sys.path.insert(0, "gemma.ggml_amd/python")
sys.path.insert(0, ".")
import os

import gemma_hip as G
from bench import GEMMA_2B, GEMMA_7B, make_prompt

layer = int(sys.argv[1]) if len(sys.argv) > 1 else 9
shape = GEMMA_7B if (len(sys.argv) > 2 and sys.argv[2] == "7b") else GEMMA_2B
wtype = G.GGML_TYPE_Q4_K if os.environ.get("KQ") == "1" else G.GGML_TYPE_Q4_0  # KQ=1: the Q4_K_M layout
e = G.Engine(shape, n_ctx=512, device=0, wtype=wtype)
if os.environ.get("PLAN"):  # qkv, o, gate/up, down, logits: ks,rpw,img triples
    v = [int(t) for t in os.environ["PLAN"].split(",")]
    e.set_plan({k: (v[3 * i], v[3 * i + 1], v[3 * i + 2]) for i, k in enumerate(e.PLAN_CLASSES)})
print("plan", e.plan() if wtype == G.GGML_TYPE_Q4_0 else "K-quant")
e.begin(make_prompt(128, shape["n_vocab"]))
e.step(140, use_graph=True)
names = ["qkv", "attention", "attn-out", "gate/up", "down", "logits"]
phases = {0: ["issue", "prologue", "sync", "stream", "end", "own", "carry0", "fma", "store", "sync2"], 1: ["p1", "p2", "p3", "p4", "p5", "p6", "p7"]}  # attention: see AH_STAMP / ATT_STAMP
for rep in range(2):
    st = e.stamp_step(layer).astype(np.int64)
prev_end = None
for k, nm in enumerate(names):
    r = st[k].reshape(-1, 8) if k == 1 else st[k]  # attention writes 8 stamps per workgroup
    r = r[r[:, 0] != 0]
    if len(r) == 0:
        continue
    t0 = r[:, 0].min()
    ph = phases[1] if k == 1 else phases[0]
    n = len(ph) + 1
    rel = (r[:, :n] - t0) * 10
    rel[r[:, :n] == 0] = -1
    end = r[:, :n].max() if k == 1 else r[:, 5].max()
    gap = (t0 - prev_end) * 10 if prev_end is not None else None
    print(f"{nm:10s} WGs={len(r):5d} start spread {int((r[:, 0].max() - t0) * 10):6d} ns  gap {gap} ns  "
          f"span {int((end - t0) * 10)} ns")
    print("   median " + " ".join(f"{p}={int(v)}" for p, v in zip(["start"] + ph, np.median(rel, axis=0))))
    print("   max    " + " ".join(f"{p}={int(v)}" for p, v in zip(["start"] + ph, rel.max(axis=0))))
    if k == 1 and os.environ.get("CLK") == "1":  # stamps build 3: s_memtime beside stamps 0 / 4 (slots 5 / 6: cycles, ticks)
        ghz = r[:, 5] / np.maximum(r[:, 6] * 10, 1)  # cycles / ns of split 0's workgroups
        print(f"   core clock GHz median {np.median(ghz):.3f} min {ghz.min():.3f} max {ghz.max():.3f}")
    prev_end = end
e.close()
