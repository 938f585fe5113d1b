"""Timing probe: the gate/up matvec in its paired (k_split 1) and split-wave (k_split 2) forms,
Gemma-2B Q4_0 shapes, hipEvents over launches rotating over the 18 layers (gemma_engine_time)."""
import sys
sys.path.insert(0, "gemma.ggml_amd/python")
sys.path.insert(0, ".")
import gemma_hip as G  # noqa: E402
from bench import GEMMA_2B  # noqa: E402

e = G.Engine(GEMMA_2B, n_ctx=512)
base = e.plan()
for ks, rpw in ((1, 1), (2, 1), (2, 2), (1, 2), (2, 4)):
    e.set_plan(dict(base, gate_up=(ks, rpw, 0)))
    e.begin([2, 5, 7])
    e.step(3, use_graph=False)
    t = [round(e.time_kernel(0, 200)[0], 3) for _ in range(3)]
    e.begin([2, 5, 7])
    import time
    e.step(3 + 8, use_graph=True)
    e.L.gemma_engine_sync(e.h)
    t0 = time.perf_counter()
    e.step(64, use_graph=True)
    e.L.gemma_engine_sync(e.h)
    print("gate_up", (ks, rpw), "us", t, "decode tok/s", round(64 / (time.perf_counter() - t0), 1), flush=True)
