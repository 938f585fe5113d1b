"""A/B of the persistent token launch against the per-layer launches, same engine, same box.

    python scripts/persist_ab.py [steps] [reps] [wtype q4_0|q8_0]

Prints decode tok/s (64-step hipGraph replays after a 128-token prompt) for each mode, interleaved
reps, and the persistent launch's hand-off timeout words.
"""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "gemma.ggml_amd", "python"))
sys.path.insert(0, ROOT)

import gemma_hip as G  # noqa: E402
from bench import GEMMA_2B, make_prompt  # noqa: E402


def main():
    steps = int(sys.argv[1]) if len(sys.argv) > 1 else 64
    reps = int(sys.argv[2]) if len(sys.argv) > 2 else 3
    wt = G.GGML_TYPE_Q8_0 if len(sys.argv) > 3 and sys.argv[3] == "q8_0" else G.GGML_TYPE_Q4_0
    e = G.Engine(GEMMA_2B, n_ctx=512, wtype=wt)
    prompt = make_prompt(128, GEMMA_2B["n_vocab"])
    res = {0: [], 1: []}
    for rep in range(reps):
        for mode in (1, 0):
            on = e.set_persist(mode)
            assert on == bool(mode), G.last_error()
            e.persist_err(reset=True)
            e.begin(prompt)
            e.step(len(prompt) + 8, use_graph=True)
            e.L.gemma_engine_sync(e.h)
            t0 = time.perf_counter()
            e.step(steps, use_graph=True)
            e.L.gemma_engine_sync(e.h)
            dt = time.perf_counter() - t0
            res[mode].append(steps / dt)
            err = e.persist_err()
            print(f"rep {rep} persist {mode}: {steps / dt:.1f} tok/s  ({dt / steps * 1e3:.4f} ms/token)  err {err}"
                  f"  launches {e.graph_kernels()}", flush=True)
    toks = e.tokens()
    print("tokens", list(toks[128:136]))
    for mode in (1, 0):
        print(f"persist {mode}: best {max(res[mode]):.1f} median {sorted(res[mode])[len(res[mode]) // 2]:.1f} tok/s")
    e.close()


if __name__ == "__main__":
    main()
