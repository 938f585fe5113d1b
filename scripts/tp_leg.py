"""Gemma-7B row-split decode leg of bench.py (BASELINE config 4): one process per GPU, weights
row-split across WORLD_SIZE GPUs, RCCL all-gathers.  bench.py runs it as a child
process of every rank with a time limit, so a collective that never completes cannot stall the
bench line.  Rank 0 prints one JSON line.  usage: tp_leg.py <steps> <wtype q4_0|q8_0> <tune 0|1>"""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "gemma.ggml_amd", "python"))
sys.path.insert(0, ROOT)


def main():
    steps, wtype_s, tune = int(sys.argv[1]), sys.argv[2], sys.argv[3] == "1"
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    import torch
    import torch.distributed as dist

    import gemma_hip as G
    from bench import GEMMA_7B, make_prompt
    wtype = G.GGML_TYPE_Q4_0 if wtype_s == "q4_0" else G.GGML_TYPE_Q8_0
    rid = None
    if world > 1:
        dist.init_process_group(backend="gloo", init_method="env://")
        idt = torch.zeros(256, dtype=torch.uint8)
        if rank == 0:
            raw = G.tp_unique_id()
            idt[: len(raw)] = torch.tensor(list(raw), dtype=torch.uint8)
        dist.broadcast(idt, 0)
        rid = bytes(idt.numpy())

    def sync():
        torch.cuda.synchronize(local_rank)
        if world > 1:
            dist.barrier()

    te = G.Engine(GEMMA_7B, n_ctx=256, wtype=wtype, device=local_rank, tp=(world, rank, rid))
    plan = te.tune(6) if tune else te.plan()
    te.begin(make_prompt(16, GEMMA_7B["n_vocab"]))
    te.step(16 + 4, use_graph=True)
    sync()
    t0 = time.perf_counter()
    te.step(steps, use_graph=True)
    te.L.gemma_engine_sync(te.h)
    sync()
    dt = time.perf_counter() - t0
    if world > 1:
        t = torch.tensor([dt], dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        dt = float(t.item())
    toks = list(te.tokens())
    te.close()
    if rank == 0:
        print(json.dumps({"model": "Gemma-7B " + wtype_s.upper(), "ranks": world, "tok_s": round(steps / dt, 2),
                          "ms_per_token": round(dt / steps * 1e3, 4), "steps": steps,
                          "parallelism": f"row-split tp{world} (RCCL all-gather x4/layer)" if world > 1 else "1 GPU",
                          "tokens_head": [int(t) for t in toks[16:24]], "launch_plan": plan}), flush=True)
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
