"""Phase stamps of the persistent token launch (token.hip), one decode step after a 128-token prompt.

    GHIP_ALLOW_ALT_LIB=1 GHIP_LIB=ab_libs/libstamps.so python scripts/token_stamps.py [layers-to-print]
(build: bash scripts/build_variant.sh stamps token.hip,engine.cpp -DGHIP_STAMPS=1)

Stamp i of layer l (s_memrealtime, 100 MHz = 10 ns) per workgroup: 0 layer start, 1 x gathered,
2 norm+image, 3 qkv rr done (term waves), 4 attention q|k|v gathered, 5 attention done, 6 attention
image gathered, 7 o rr done, 8 sa gathered, 9 ffn norm, 10 gate/up done, 11 h image gathered,
12 down rr done.  Prints, per layer, each phase's latest workgroup (the critical path) relative to
the layer's earliest start, and the layer-to-layer period.
"""
import ctypes as C
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "gemma.ggml_amd", "python"))
sys.path.insert(0, ROOT)
import gemma_hip as G  # noqa: E402
from bench import GEMMA_2B, make_prompt  # noqa: E402

NAMES = ["start", "x", "norm", "qkv", "att_in", "att", "att_img", "o", "sa", "fnorm", "gu6", "gu", "h_img", "dn0", "dn7", "down"]
ORDER = [0, 1, 2, 3, 4, 5, 6, 7, 8, 9, 13, 10, 11, 14, 15, 12]  # stamp slot of each name


def main():
    nshow = int(sys.argv[1]) if len(sys.argv) > 1 else 3
    L = G.lib()
    L.gemma_engine_token_stamps.argtypes = [C.c_void_p, C.c_void_p]
    e = G.Engine(GEMMA_2B, n_ctx=512)
    assert e.set_persist(1), G.last_error()
    prompt = make_prompt(128, GEMMA_2B["n_vocab"])
    e.begin(prompt)
    e.step(len(prompt) + 4, use_graph=True)
    nl = GEMMA_2B["n_layer"]
    grid = GEMMA_2B["n_embd"] // 8
    out = np.zeros(grid * nl * 16 + 256, dtype=np.uint64)
    for rep in range(2):
        r = L.gemma_engine_token_stamps(e.h, out.ctypes.data_as(C.c_void_p))
        assert r == 0, G.last_error()
    probes = out[grid * nl * 16:].astype(np.int64).reshape(64, 4)
    t = out[: grid * nl * 16].reshape(grid, nl, 16).astype(np.int64)
    t0 = t[:, 0, 0].min()
    att = np.array([(c & 7) == 0 and (c >> 3) < 32 for c in range(grid)])
    print("per layer: phase -> max over workgroups (us from the layer's earliest start); attention rows: the 32 attention WGs")
    starts = [t[:, l, 0].min() for l in range(nl)]
    for l in list(range(min(nshow, nl))) + [nl - 1]:
        base = starts[l]
        row = []
        for i, nm in zip(ORDER, NAMES):
            v = t[:, l, i]
            sel = v[att] if nm in ("att_in", "att") else v
            sel = sel[sel > 0]
            if sel.size == 0:
                continue
            row.append(f"{nm} {(sel.max() - base) / 100:.2f}/{(np.median(sel) - base) / 100:.2f}")
        print(f"L{l}: " + "  ".join(row))
    per = np.diff(starts) / 100
    print("layer start-to-start us:", " ".join(f"{x:.1f}" for x in per))
    end = t[:, nl - 1, 12].max()
    print(f"whole launch (first start -> last down): {(end - t0) / 100:.1f} us")
    # phase durations averaged over layers 1..nl-2 (critical path deltas)
    acc = np.zeros(len(NAMES))
    for l in range(1, nl - 1):
        base = starts[l]
        prev = 0.0
        for jj, (i, nm) in enumerate(zip(ORDER, NAMES)):
            v = t[:, l, i]
            sel = v[att] if nm in ("att_in", "att") else v
            sel = sel[sel > 0]
            m = (sel.max() - base) / 100 if sel.size else prev
            acc[jj] += m - prev
            prev = m
    acc /= max(nl - 2, 1)
    print("mean critical-path increments (us): " + "  ".join(f"{nm} {x:.2f}" for nm, x in zip(NAMES, acc)))
    nz = [i for i in range(64) if probes[i, 0] != 0]
    p0 = probes[nz[0], 0] if nz else 0
    print("workgroup 0 wave 0 layer 1 pops (us from its first pop): start / after refill issue / after vmcnt wait")
    for i in nz:
        print(f"  pop {i:2d}: {(probes[i, 0] - p0) / 100:7.2f} {(probes[i, 1] - p0) / 100:7.2f} {(probes[i, 2] - p0) / 100:7.2f}")
    e.close()


if __name__ == "__main__":
    main()
