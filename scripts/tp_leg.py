"""Row-split decode leg of bench.py: one process per GPU, every weight matrix row-split
across WORLD_SIZE GPUs, RCCL all-gathers inside the decode hipGraph.  bench.py runs it as a child
process of every rank with a time limit, so a collective that never completes cannot stall the bench
line.  Rank 0 prints one JSON line; a parity mismatch on any rank prints an error object and every
rank exits 3.

usage: tp_leg.py <steps> <wtype q4_0|q8_0> <tune 0|1> [model 2b|7b] [warmup] [prompt] [layouts] [shared]

  layouts  comma list of engine layout flags to check and time (default 2b: 0,1,2,3; 7b: 0,1):
           0 split / 1 attention replicated, +2 = peer-to-peer gathers instead of RCCL
  shared   every rank on device 0 (a one-GPU box: only the p2p layouts, RCCL refuses two ranks
           per device) — the p2p transport's end-to-end check, not a scaling measurement

  2b  Gemma-2B (BASELINE config 2 row-split over N GPUs: the headline of `bench.py --gpus N`, N > 1),
      the bench's synthetic weights and prompt
  7b  Gemma-7B (BASELINE config 4), synthetic weights with the token_embd / output matrix at 0.25x
      its default std, so the greedy tokens follow the input instead of settling on one id.  SURVEY
      §8(d) suggests x4 for peaked logits, but the output is TIED to the embedding: the current
      token's own row rides the residual stream to the final norm and x4 turns the model into a copy
      model (every prompt row's argmax is its input token; x1 settles on one id with a 1.2e-5
      margin).  Measured with scripts/out_gain_scan.py 7b: x4 / x1 / x0.5 / x0.25 / x0.125 give 1 /
      1 / 5 / 10 / 10 distinct tokens in 16 greedy steps, margins 0.40 / 1.2e-5 / 3.3e-3 / 1.9e-3 /
      1.2e-3.

The control flow (RCCL id broadcast, lockstep tuning with rank 0's plan broadcast, the unsplit-engine
hash check, max-over-ranks timing) is gemma_tp.run_stream; tests/test_tp_control.py drives it with a
stub engine over gloo.  The unsplit 1-GPU engine and the split engine get the same launch-plan
treatment (both tuned, or both on the default plan), so at N = 1 the ratio reads ~1.00."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "gemma.ggml_amd", "python"))
sys.path.insert(0, ROOT)

# per class: kernel id of gemma_engine_time -> name, launches per token
KERNELS = {0: ("ffn gate/up matvec (+norm, +gelu*mul)", "n_layer"), 1: ("ffn down matvec (+resid)", "n_layer"),
           2: ("qkv matvec (+norm)", "n_layer"), 3: ("attn-out matvec (+resid)", "n_layer"),
           4: ("logits matvec (+argmax)", 1)}


def main(argv=None, make_engine=None, make_id=None, comm=None, device_sync=None):
    argv = sys.argv[1:] if argv is None else argv
    steps, wtype_s, tune = int(argv[0]), argv[1], argv[2] == "1"
    model = argv[3] if len(argv) > 3 else "7b"
    warmup = int(argv[4]) if len(argv) > 4 else 4
    n_prompt = int(argv[5]) if len(argv) > 5 else 16
    layouts = tuple(int(v) for v in argv[6].split(",")) if len(argv) > 6 else ((0, 1, 2, 3) if model == "2b" else (0, 1))
    shared = len(argv) > 7 and argv[7] == "shared"
    import gemma_tp as T
    from bench import GEMMA_2B, GEMMA_7B, HBM_PEAK_GBS, make_prompt
    shape = GEMMA_2B if model == "2b" else GEMMA_7B
    out_gain = 0.0 if model == "2b" else 0.25
    comm = comm or T.Comm.from_env("gloo")
    if make_engine is None:  # the product: the HIP engine on this rank's GPU
        import torch

        import gemma_hip as G
        local_rank = 0 if shared else int(os.environ.get("LOCAL_RANK", "0"))
        wtype = G.GGML_TYPE_Q4_0 if wtype_s == "q4_0" else G.GGML_TYPE_Q8_0
        n_ctx = ((n_prompt + warmup + steps + 64) // 32 + 1) * 32

        def make_engine(tp, flags=0):
            return G.Engine(shape, n_ctx=max(256, n_ctx), wtype=wtype, device=local_rank, tp=tp, out_gain=out_gain,
                            tp_flags=flags)
        make_id = G.tp_unique_id
        device_sync = lambda: torch.cuda.synchronize(local_rank)  # noqa: E731
    prompt = make_prompt(n_prompt, shape["n_vocab"])
    try:
        r = T.run_stream(comm, make_engine, make_id, prompt, steps, warmup, tune=tune,
                         check_prompt=make_prompt(16, shape["n_vocab"]), device_sync=device_sync or (lambda: None),
                         kernel_iters=30 if model == "2b" else 0, layouts=layouts)
    except T.ParityError as ex:
        if comm.rank == 0:
            print(json.dumps({"error": str(ex)}), flush=True)
        comm.close()
        return T.EXIT_PARITY
    if comm.rank == 0:
        world, tok_s, tok_s_1 = comm.world, r["tok_s"], r["tok_s_unsplit_1gpu"]
        toks = r["tokens"][n_prompt:n_prompt + 8]
        line = {"model": f"Gemma-{model.upper()} {wtype_s.upper()}", "ranks": world, "tok_s": round(tok_s, 2),
                "ms_per_token": round(r["ms_per_token"], 4), "steps": steps, "warmup": warmup, "prompt": n_prompt,
                "timed_s": round(r["timed_s"], 6),
                "parallelism": (f"row-split tp{world}, layout {r['layout']} ("
                                f"{'peer-to-peer pushes' if 'p2p' in r['layout'] else 'RCCL all-gathers'} per layer: "
                                f"{2 if 'rep_attn' in r['layout'] else 4})") if world > 1
                else "1 GPU, 1-rank RCCL communicator (every gather through ncclAllGather in the hipGraph)",
                "tok_s_unsplit_1gpu": round(tok_s_1, 2) if tok_s_1 else None,
                # scaling fields only where ranks > 1; at N = 1 the ratio is the 1-rank RCCL
                # communicator's overhead against the unsplit engine
                "speedup_vs_1gpu": round(tok_s / tok_s_1, 3) if world > 1 and tok_s_1 else None,
                "strong_scaling_efficiency": round(tok_s / tok_s_1 / world, 3) if world > 1 and tok_s_1 else None,
                "rccl_overhead_vs_unsplit": round(tok_s / tok_s_1, 3) if world == 1 and tok_s_1 else None,
                "layout": r["layout"] if world > 1 else None,
                "layouts_tok_s": {k: round(v, 2) for k, v in r["layouts_tok_s"].items()} if world > 1 else None,
                "layouts_dropped": r["layouts_dropped"] if world > 1 else None,
                "parity_check": r["parity_check"], "tokens_head": toks,
                "distinct_tokens_head": len(set(toks)), "synthetic_output_gain": out_gain or None,
                "launch_plan": r["launch_plan"], "launch_plan_unsplit": r["launch_plan_unsplit"],
                "plans": ("both tuned; every rank runs rank 0's plan" if tune else "both default")}
        if r["kernels"]:  # per-N roofline: rank 0's shard kernels timed alone (hipEvents)
            cls = {}
            for k, (us, algo) in r["kernels"].items():
                name, calls = KERNELS[k]
                gbs = algo / (us * 1e-6) / 1e9
                cls[name] = {"avg_us": round(us, 3), "algo_bytes": int(algo), "GB/s": round(gbs, 1),
                             "frac": round(gbs / HBM_PEAK_GBS, 4),
                             "launches_per_token": shape["n_layer"] if calls == "n_layer" else calls}
            dom = max(cls, key=lambda n: cls[n]["avg_us"] * cls[n]["launches_per_token"])
            line["roofline"] = dict(bound="hbm", kernel=dom, achieved=cls[dom]["GB/s"], peak=HBM_PEAK_GBS, unit="GB/s",
                                    frac=cls[dom]["frac"], avg_us=cls[dom]["avg_us"], algo_bytes=cls[dom]["algo_bytes"],
                                    per="rank 0's row shard (1/N of every matrix's rows)", classes=cls)
        print(json.dumps(line), flush=True)
    comm.close()
    return 0


if __name__ == "__main__":
    sys.exit(main())
