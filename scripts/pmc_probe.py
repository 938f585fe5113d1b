"""Counter probe: launches each hot decode kernel 36x (rotating over the 18 layers, as in a decode
step) so a `rocprofv3 --pmc` pass can price its HBM traffic per dispatch.  Run under rocprofv3 only."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "gemma.ggml_amd", "python"))
sys.path.insert(0, ROOT)
import gemma_hip as G  # noqa: E402
from bench import GEMMA_2B, make_prompt  # noqa: E402

e = G.Engine(GEMMA_2B, n_ctx=512, device=0)
e.begin(make_prompt(128, GEMMA_2B["n_vocab"]))
e.step(8, use_graph=False)
for k in (0, 1, 2, 3, 4):
    e.time_kernel(k, 36)
e.close()
print("pmc probe done")
