"""Decode-only profile target with a FIXED launch plan (VERDICT r4 "Next round" #7): Gemma-2B Q4_0,
the bench's 128-token prompt, then `steps` greedy decode steps — no tuning, no other legs, so a
rocprofv3 kernel trace of this process holds exactly the decode kernels of one plan.

  rocprofv3 --kernel-trace --stats -d OUT -o run -- python3 scripts/decode_prof.py [steps]
  python3 scripts/decode_classes.py OUT/.../run_kernel_trace.csv 128 steps > profiles/r05/decode_kernels.md

PLAN (env, optional): qkv, attn-out, gate/up, down, logits as 15 ints k_split,rows_per_wg,image
(default: the plan the round-4 driver bench tuned to, BENCH_r04 `launch_plan`).  GHIP_PROF_GRAPH=1
replays the hipGraph (the product path); the default runs the same kernels eagerly, because a
rocprofv3 kernel trace of graph replays once crashed inside the runtime (SIGSEGV).
"""
import os
import sys

if os.environ.get("TORCH_FIRST", "0") == "1":
    # torch's bundled HIP runtime (libamdhip64.so.7 of torch/lib, the one bench.py and the tests run on,
    # since they import torch first) instead of /opt/rocm's: the dynamic linker reuses the loaded soname
    import torch  # noqa: F401
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "gemma.ggml_amd", "python"))
sys.path.insert(0, ROOT)
import gemma_hip as G  # noqa: E402
from bench import GEMMA_2B, make_prompt  # noqa: E402

BENCH_R04_PLAN = "9,1,0,9,1,0,1,1,0,9,1,1,1,8,0"


def main():
    steps = int(sys.argv[1]) if len(sys.argv) > 1 else 32
    graph = os.environ.get("GHIP_PROF_GRAPH", "0") == "1"
    e = G.Engine(GEMMA_2B, n_ctx=512, device=0)
    if os.environ.get("PROF_MAPS"):  # the process's mappings (symbolizes a native crash exactly)
        with open("/proc/self/maps") as f, open(os.environ["PROF_MAPS"], "w") as g:
            g.write(f.read())
    v = [int(t) for t in os.environ.get("PLAN", BENCH_R04_PLAN).split(",")]
    e.set_plan({k: (v[3 * i], v[3 * i + 1], v[3 * i + 2]) for i, k in enumerate(e.PLAN_CLASSES)})
    if os.environ.get("ATT_O"):
        e.set_att_o(int(os.environ["ATT_O"]))
    prompt = make_prompt(128, GEMMA_2B["n_vocab"])
    e.begin(prompt)
    e.step(len(prompt) + steps, use_graph=graph)
    e.L.gemma_engine_sync(e.h)
    print("plan", e.plan(), "graph", graph, "tokens", list(e.tokens()[128:136]), flush=True)
    e.close()


if __name__ == "__main__":
    main()
