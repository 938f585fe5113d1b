"""Gemma-7B row-split decode leg of bench.py (BASELINE config 4): one process per GPU, weights
row-split across WORLD_SIZE GPUs, RCCL all-gathers.  bench.py runs it as a child
process of every rank with a time limit, so a collective that never completes cannot stall the
bench line.  Rank 0 prints one JSON line.  usage: tp_leg.py <steps> <wtype q4_0|q8_0> <tune 0|1>

Synthetic Gemma-7B weights with the token_embd / output matrix at 0.25x its default std, so the
greedy tokens follow the input instead of settling on one id.  SURVEY §8(d) suggests x4 for peaked
logits, but the output is TIED to the embedding: the current token's own row rides the residual
stream to the final norm and x4 turns the model into a copy model (every prompt row's argmax is its
input token, the greedy sequence repeats the last prompt token; x1 settles on one id with a 1.2e-5
margin).  Measured with scripts/out_gain_scan.py 7b: x4 / x1 / x0.5 / x0.25 / x0.125 give 1 / 1 / 5
/ 10 / 10 distinct tokens in 16 greedy steps, margins 0.40 / 1.2e-5 / 3.3e-3 / 1.9e-3 / 1.2e-3.  The unsplit 1-GPU reference engine and the split engine under test get the same launch-plan
treatment (both tuned, or both on the default plan), so at N = 1 the efficiency reads ~1.00."""
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
    if world > 1:
        dist.init_process_group(backend="gloo", init_method="env://")

    def new_id():
        """A fresh RCCL unique id for ONE communicator (an id serves a single ncclCommInitRank round:
        its bootstrap root leaves once every rank has joined, so a second init on it fails with
        "remote process exited").  N > 1: rank 0 makes it and broadcasts it over gloo."""
        if world == 1:
            return G.tp_unique_id()
        idt = torch.zeros(256, dtype=torch.uint8)
        if rank == 0:
            raw = G.tp_unique_id()
            idt[: len(raw)] = torch.tensor(list(raw), dtype=torch.uint8)
        dist.broadcast(idt, 0)
        return bytes(idt.numpy())

    def sync():
        torch.cuda.synchronize(local_rank)
        if world > 1:
            dist.barrier()

    import hashlib

    import numpy as np
    n_check, prompt = 20, make_prompt(16, GEMMA_7B["n_vocab"])
    OUT_GAIN = 0.25

    def row_hashes(lg):
        return np.frombuffer(b"".join(hashlib.sha1(r.tobytes()).digest()[:8] for r in lg), dtype=np.uint8).copy()

    # reference (rank 0): the UNSPLIT engine on one GPU, same synthetic weights and prompt; the first
    # 16 rows are the prompt positions (teacher-forced, so they vary with the input tokens), then 4
    # greedy steps.  Its logits hashes are broadcast; every rank compares its own gathered logits.
    # At N = 1 the split under test is 8 virtual ranks on one GPU (the same shards and key merge).
    ref = torch.zeros(n_check * 8, dtype=torch.uint8)
    tok_s_1 = None
    margin = None
    if rank == 0:
        re_ = G.Engine(GEMMA_7B, n_ctx=256, wtype=wtype, device=local_rank, out_gain=OUT_GAIN)
        re_.begin(prompt)
        lg = re_.step(n_check, want_logits=True, use_graph=True)
        ref = torch.from_numpy(row_hashes(lg))
        top2 = np.sort(lg, axis=1)[:, -2:]
        margin = float(np.min((top2[:, 1] - top2[:, 0]) / np.maximum(np.abs(top2[:, 1]), 1e-30)))
        ref_tokens = [int(t) for t in re_.tokens()[16:24]]
        plan_1 = re_.tune(6) if tune else re_.plan()
        re_.begin(prompt)
        re_.step(16 + 4, use_graph=True)
        re_.L.gemma_engine_sync(re_.h)
        t1 = time.perf_counter()
        re_.step(steps, use_graph=True)
        re_.L.gemma_engine_sync(re_.h)
        tok_s_1 = steps / (time.perf_counter() - t1)
        re_.close()
    if world > 1:
        dist.broadcast(ref, 0)
    # checked: the RCCL ranks (N > 1) or, at N = 1, 8 virtual ranks AND a 1-rank RCCL engine (so the
    # timed engine below runs the transport); every communicator gets its own id
    splits = [(world, rank, "rccl")] if world > 1 else [(8, 0, None), (1, 0, "rccl")]
    nbad = 0
    for split in splits:
        if split[2] == "rccl":
            split = (split[0], split[1], new_id())
        ce = G.Engine(GEMMA_7B, n_ctx=256, wtype=wtype, device=local_rank, tp=split, out_gain=OUT_GAIN)
        ce.begin(prompt)
        got = row_hashes(ce.step(n_check, want_logits=True, use_graph=True))
        ce.close()
        nbad += int(np.sum(got.reshape(n_check, 8) != ref.numpy().reshape(n_check, 8), axis=1).astype(bool).sum())
    bad = torch.tensor([nbad])
    if world > 1:
        dist.all_reduce(bad, op=dist.ReduceOp.SUM)
    if int(bad.item()) != 0:
        if rank == 0:
            print(json.dumps({"error": f"row-split logits differ from the unsplit engine: {int(bad.item())} rows over all ranks"}), flush=True)
        sys.exit(3)

    te = G.Engine(GEMMA_7B, n_ctx=256, wtype=wtype, device=local_rank, tp=(world, rank, new_id()), out_gain=OUT_GAIN)
    plan = te.tune(6) if tune else te.plan()
    te.begin(prompt)
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
        tok_s = steps / dt
        print(json.dumps({"model": "Gemma-7B " + wtype_s.upper(), "ranks": world, "tok_s": round(tok_s, 2),
                          "ms_per_token": round(dt / steps * 1e3, 4), "steps": steps,
                          "parallelism": f"row-split tp{world} (RCCL all-gather x4/layer)" if world > 1
                          else "1 GPU, 1-rank RCCL communicator (every gather through ncclAllGather in the hipGraph)",
                          "tok_s_unsplit_1gpu": round(tok_s_1, 2),
                          # scaling fields only where ranks > 1; at N = 1 the ratio is the 1-rank RCCL
                          # communicator's overhead against the unsplit engine
                          "speedup_vs_1gpu": round(tok_s / tok_s_1, 3) if world > 1 else None,
                          "strong_scaling_efficiency": round(tok_s / tok_s_1 / world, 3) if world > 1 else None,
                          "rccl_overhead_vs_unsplit": round(tok_s / tok_s_1, 3) if world == 1 else None,
                          "parity_check": {"rows": n_check, "mismatched_rows_all_ranks": 0,
                                           "reference": "unsplit 1-GPU engine (rank 0), logits sha1 per row",
                                           "split_checked": f"{world} RCCL ranks" if world > 1
                                           else "8 virtual ranks + the 1-rank RCCL engine",
                                           "min_top1_top2_rel_margin": round(margin, 6)},
                          "tokens_head": [int(t) for t in toks[16:24]], "tokens_head_unsplit": ref_tokens,
                          "distinct_tokens_head": len(set(int(t) for t in toks[16:24])),
                          "synthetic_output_gain": OUT_GAIN, "launch_plan": plan, "launch_plan_unsplit": plan_1,
                          "plans": "both tuned" if tune else "both default"}), flush=True)
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
