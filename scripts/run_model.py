"""Decode a synthetic model for profiling: python scripts/run_model.py {2b|7b} [steps] [tp_virtual]"""
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "gemma.ggml_amd", "python"))
import gemma_hip as G  # noqa: E402

SHAPES = {"2b": dict(n_layer=18, n_embd=2048, n_head=8, n_head_kv=1, head_dim=256, n_ff=16384, n_vocab=256000),
          "7b": dict(n_layer=28, n_embd=3072, n_head=16, n_head_kv=16, head_dim=256, n_ff=24576, n_vocab=256000)}
name = sys.argv[1]
steps = int(sys.argv[2]) if len(sys.argv) > 2 else 32
tpv = int(sys.argv[3]) if len(sys.argv) > 3 else 1
e = G.Engine(SHAPES[name], n_ctx=256, device=0, tp=(tpv, 0, None) if tpv > 1 else None)
if os.environ.get("PLAN"):  # e.g. PLAN=1,1,0,4,1,0,1,1,0,8,2,0,1,16,0 (qkv, o, gate/up, down, logits: ks,rpw,img)
    v = [int(t) for t in os.environ["PLAN"].split(",")]
    e.set_plan({k: (v[3 * i], v[3 * i + 1], v[3 * i + 2]) for i, k in enumerate(e.PLAN_CLASSES)})
elif os.environ.get("TUNE", "1") == "1":  # tuning replays ~20 captured graphs: under rocprofv3 pass PLAN
    print("plan", e.tune(6))
print("plan", e.plan())
e.begin([2, 100, 200, 300])
e.step(4 + steps, use_graph=os.environ.get("GHIP_PROF_GRAPH", "0") == "1")  # eager under the profiler
e.L.gemma_engine_sync(e.h)
print("tokens", list(e.tokens()[:12]))
e.close()
