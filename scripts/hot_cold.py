"""Kernel times with weights streamed cold from HBM (rotating over layers) vs hot (one matrix
repeated, so it is Infinity-Cache resident): how much a cache-warm weight stream would buy."""
import os
import subprocess
import sys

code = r'''
import sys, json
sys.path.insert(0, "gemma.ggml_amd/python"); sys.path.insert(0, ".")
import gemma_hip as G
from bench import GEMMA_2B, make_prompt
e = G.Engine(GEMMA_2B, n_ctx=512, device=0)
e.begin(make_prompt(16, GEMMA_2B["n_vocab"])); e.step(20, use_graph=True)
print(json.dumps({w: e.time_kernel(w, 200)[0] for w in range(4)}))
'''
for mode in ("cold", "hot"):
    env = dict(os.environ)
    if mode == "hot":
        env["GHIP_TIME_HOT"] = "1"
    r = subprocess.run([sys.executable, "-c", code], env=env, capture_output=True, text=True, timeout=300)
    print(mode, r.stdout.strip().splitlines()[-1] if r.stdout.strip() else r.stderr[-500:])
