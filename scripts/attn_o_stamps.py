"""Diagnostic (stamps build): the fused attention + attn-out launch (k_attn_o) of one layer, phase by
phase, s_memrealtime (10 ns ticks) relative to the launch's first workgroup start; and the same
layer's separate attention + attn-out launches for comparison.
usage: GHIP_ALLOW_ALT_LIB=1 GHIP_LIB=ab_libs/libstamps.so python scripts/attn_o_stamps.py [layer]"""
import os
import sys

import numpy as np
import torch  # noqa: F401

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "gemma.ggml_amd", "python"))
sys.path.insert(0, ROOT)
import gemma_hip as G  # noqa: E402
from bench import GEMMA_2B, make_prompt  # noqa: E402

layer = int(sys.argv[1]) if len(sys.argv) > 1 else 9
e = G.Engine(GEMMA_2B, n_ctx=512, device=0)
p = e.plan()
p.update(qkv=(9, 1, 0), attn_out=(9, 1, 1), gate_up=(1, 1, 0), down=(9, 1, 1), logits=(1, 8, 0), attention=0)
e.set_plan(p)
for on in (1, 0):
    e.set_att_o(on)
    e.begin(make_prompt(128, GEMMA_2B["n_vocab"]))
    e.step(140, use_graph=True)
    for rep in range(3):
        st = e.stamp_step(layer).astype(np.int64)
    qkv = st[0][st[0][:, 0] != 0]
    q_end = qkv[:, 5].max() if len(qkv) else None
    if on:
        r = st[1][:256]
        att = np.array([b for b in range(256) if b % 8 == 0])
        con = np.array([b for b in range(256) if b % 8 != 0])
        t0 = r[r[:, 0] != 0, 0].min()
        rel = lambda x: (x - t0) * 10  # noqa: E731
        print(f"att_o=1 layer {layer}: qkv end -> launch start {rel(q_end) if q_end else None} ns")
        print(f"  attention WGs: start med {np.median(rel(r[att, 0])):.0f} end med {np.median(rel(r[att, 5])):.0f} max {rel(r[att, 5]).max()}")
        for k, nm in ((0, "start"), (1, "weights issued"), (2, "poll passed"), (3, "image built"), (4, "rr done")):
            v = rel(r[con, k])
            print(f"  consumers {nm:15s} median {np.median(v):7.0f}  min {v.min():7.0f}  max {v.max():7.0f} ns")
        g = st[3][st[3][:, 0] != 0]
        if len(g):
            print(f"  next launch (gate/up) first start {rel(g[:, 0].min())} ns")
    else:
        a = st[1].reshape(-1, 8)
        a = a[a[:, 0] != 0]
        o = st[2][st[2][:, 0] != 0]
        t0 = a[:, 0].min()
        rel = lambda x: (x - t0) * 10  # noqa: E731
        print(f"att_o=0 layer {layer}: attention start -> end {rel(a[:, :5].max())} ns; attn-out first start "
              f"{rel(o[:, 0].min())}, end {rel(o[:, 5].max())} ns")
        g = st[3][st[3][:, 0] != 0]
        if len(g):
            print(f"  next launch (gate/up) first start {rel(g[:, 0].min())} ns")
e.close()
