"""Diagnostic: the first decode steps after a batched prefill (graph captured before it)."""
import os, sys, time
sys.path.insert(0, "gemma.ggml_amd/python"); sys.path.insert(0, ".")
import gemma_hip as G
from bench import GEMMA_2B, make_prompt
e = G.Engine(GEMMA_2B, n_ctx=512)
p = make_prompt(128, GEMMA_2B["n_vocab"])
e.begin(p[:4]); e.step(1, use_graph=True); e.L.gemma_engine_sync(e.h)  # graph captured before any prefill
for trial in range(3):
    e.begin(p)
    if trial < 2:
        t0 = time.perf_counter(); e.prefill(128); e.L.gemma_engine_sync(e.h); t1 = time.perf_counter()
    else:
        t0 = time.perf_counter(); e.step(128, use_graph=True); e.L.gemma_engine_sync(e.h); t1 = time.perf_counter()
    ts = []
    for i in range(4):
        a = time.perf_counter(); e.step(1, use_graph=True); e.L.gemma_engine_sync(e.h); ts.append((time.perf_counter() - a) * 1e3)
    print(f"trial {trial}: prompt {(t1-t0)*1e3:.1f} ms, steps", " ".join(f"{x:.3f}" for x in ts), flush=True)
