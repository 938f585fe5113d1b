"""Which token_embd / output gain makes the synthetic model's greedy tokens depend on the input?
(the TP leg's check).  With a TIED output, the current token's own embedding rides the
residual stream to the final norm, so a LARGER gain makes logits[t] = |E_t|^2 * sqrt(E) * gain^2
dominate (a copy model: the greedy sequence repeats the last prompt token); a smaller gain lets the
layers' outputs decide.  Prints, per gain, the 16-row teacher-forced argmaxes vs the input tokens,
the greedy continuation and the smallest top-1/top-2 margin.
usage: python scripts/out_gain_scan.py [2b|7b] gain [gain ...]"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "gemma.ggml_amd", "python"))
sys.path.insert(0, ROOT)
import gemma_hip as G  # noqa: E402
from bench import GEMMA_2B, GEMMA_7B, make_prompt  # noqa: E402

shape = GEMMA_7B if sys.argv[1] == "7b" else GEMMA_2B
prompt = make_prompt(16, shape["n_vocab"])
for g in [float(x) for x in sys.argv[2:]]:
    e = G.Engine(shape, n_ctx=256, out_gain=g)
    e.begin(prompt)
    lg = e.step(16 + 16, want_logits=True, use_graph=True)
    am = lg.argmax(axis=1)
    top2 = np.sort(lg, axis=1)[:, -2:]
    margin = float(np.min((top2[:, 1] - top2[:, 0]) / np.maximum(np.abs(top2[:, 1]), 1e-30)))
    toks = [int(t) for t in e.tokens()]
    copy = int(np.sum(am[:16] == np.array(prompt[:16])))
    print(f"gain {g}: prompt rows whose argmax = their input token {copy}/16; greedy {toks[16:32]}; "
          f"distinct {len(set(toks[16:32]))}; min rel margin {margin:.4g}", flush=True)
    e.close()
