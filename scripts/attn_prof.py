"""Profile target for the decode attention: Gemma-2B Q4_0, 128-token prompt fed token by token, then
64 greedy steps (positions 128..191, the bench's range).  usage: python scripts/attn_prof.py"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "gemma.ggml_amd", "python"))
sys.path.insert(0, ROOT)
import gemma_hip as G  # noqa: E402
from bench import GEMMA_2B, make_prompt  # noqa: E402

e = G.Engine(GEMMA_2B, n_ctx=512, device=0)
e.begin(make_prompt(128, GEMMA_2B["n_vocab"]))
# eager by default: a rocprofv3 kernel trace of graph replays crashed once inside the runtime
# (the round-4 SIGSEGV); GHIP_PROF_GRAPH=1 profiles the hipGraph replay itself
e.step(128 + 64, use_graph=os.environ.get("GHIP_PROF_GRAPH", "0") == "1")
e.L.gemma_engine_sync(e.h)
print("tokens", list(e.tokens()[128:136]))
e.close()
