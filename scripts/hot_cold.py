"""Kernel times with weights streamed cold from HBM (rotating over layers) vs hot (one matrix
repeated, so it is Infinity-Cache resident): how much a cache-warm weight stream would buy."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "gemma.ggml_amd", "python"))
sys.path.insert(0, ROOT)
import gemma_hip as G  # noqa: E402
from bench import GEMMA_2B, make_prompt  # noqa: E402

e = G.Engine(GEMMA_2B, n_ctx=512, device=0)
e.begin(make_prompt(16, GEMMA_2B["n_vocab"]))
e.step(20, use_graph=True)
for mode in ("cold", "hot"):
    e.set_option("time_hot", mode == "hot")
    print(mode, json.dumps({w: round(e.time_kernel(w, 200)[0], 3) for w in range(4)}), flush=True)
e.close()
