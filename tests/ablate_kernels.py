"""Timing-only ablation sweep of the decode matvec kernels (not a test; results differ)."""
import os
import subprocess
import sys

code = r'''
import sys, os, json
sys.path.insert(0, "gemma.ggml_amd/python")
import gemma_hip as G
shape = dict(n_layer=18, n_embd=2048, n_head=8, n_head_kv=1, head_dim=256, n_ff=16384, n_vocab=256000)
e = G.Engine(shape, n_ctx=512)
e.begin([2, 5, 7])
e.step(3, use_graph=False)
out = {}
for k in (0, 1, 2, 3, 4):
    us, b = e.time_kernel(k, 200)
    out[k] = round(us, 2)
print(json.dumps(out))
'''
for ab in (0, 1, 8, 9, 4):
    env = dict(os.environ, GHIP_ABLATE=str(ab))
    r = subprocess.run([sys.executable, "-c", code], env=env, capture_output=True, text=True)
    print("ablate", ab, r.stdout.strip(), r.stderr.strip()[-300:] if r.returncode else "", flush=True)
