"""Timing-only ablation sweep of the decode matvec kernels (not a test; ablated results differ):
option "ablate" of gemma_engine_time (1 no dot products, 8 no scale loads, 9 both, 4 no prologue)."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "gemma.ggml_amd", "python"))
import gemma_hip as G  # noqa: E402

shape = dict(n_layer=18, n_embd=2048, n_head=8, n_head_kv=1, head_dim=256, n_ff=16384, n_vocab=256000)
e = G.Engine(shape, n_ctx=512)
e.begin([2, 5, 7])
e.step(3, use_graph=False)
for ab in (0, 1, 8, 9, 4):
    e.set_option("ablate", ab)
    print("ablate", ab, json.dumps({k: round(e.time_kernel(k, 200)[0], 2) for k in range(5)}), flush=True)
e.close()
