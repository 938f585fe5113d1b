"""Timing-only sweep of the big-matvec grid size (not a test)."""
import os
import subprocess
import sys

code = r'''
import sys, json
sys.path.insert(0, "gemma.ggml_amd/python")
import gemma_hip as G
shape = dict(n_layer=18, n_embd=2048, n_head=8, n_head_kv=1, head_dim=256, n_ff=16384, n_vocab=256000)
e = G.Engine(shape, n_ctx=512)
e.begin([2, 5, 7])
e.step(3, use_graph=False)
print(json.dumps({k: round(e.time_kernel(k, 200)[0], 2) for k in (0, 4)}))
'''
for g in (256, 512, 768, 1024, 1536, 2048, 4096, 8192):
    env = dict(os.environ, GHIP_GRID_BIG=str(g))
    r = subprocess.run([sys.executable, "-c", code], env=env, capture_output=True, text=True)
    print("grid", g, r.stdout.strip(), r.stderr.strip()[-300:] if r.returncode else "", flush=True)
for ab in (0, 1, 4, 5):
    env = dict(os.environ, GHIP_ABLATE=str(ab))
    code2 = code.replace("(0, 4)", "(0, 1, 2, 3, 4)")
    r = subprocess.run([sys.executable, "-c", code2], env=env, capture_output=True, text=True)
    print("ablate", ab, r.stdout.strip(), r.stderr.strip()[-300:] if r.returncode else "", flush=True)
