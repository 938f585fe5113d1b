import os, sys
sys.path.insert(0, "gemma.ggml_amd/python"); sys.path.insert(0, "tests")
import numpy as np
import gemma_hip as G
import oracle_ctypes as O
shape = dict(O.GEMMA_2B, n_layer=3, n_vocab=8192)
e = G.Engine(shape, n_ctx=256)
p = e.plan(); p.update(qkv=(9, 1, 0), attn_out=(9, 1, 1), attention=0); e.set_plan(p)
print("plan", e.plan(), flush=True)
e.set_fuse(1)
e.begin(O.make_prompt(9, shape["n_vocab"]))
e.step(1, use_graph=False)
e.L.gemma_engine_sync(e.h)
print("err", e.set_fuse(-1), flush=True)
