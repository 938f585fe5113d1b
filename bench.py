#!/usr/bin/env python3
"""bench.py — decode (and prefill) throughput of the MI355X hot path, BASELINE config 2.

One *step* = one greedy decode token of Gemma-2B Q4_0 at batch 1 through the device-resident engine
(all 18 layers: fused norm+quantize+matvec kernels, decode attention, logits+argmax, token feedback;
one hipGraph replay), after a 128-token synthetic prompt.  Weights are synthetic (seeded, Gemma-2B
shapes, generated on the GPU; DESIGN.md §Synthetic weights) — no checkpoint is available offline.

    python bench.py [--gpus N] [--steps K] [--warmup W] [--no-cpu] [--profile-out PATH]

N > 1: one process per GPU (torch.distributed.run).  The headline `value` is ONE Gemma-2B Q4_0
decode stream with every weight matrix row-split across the N GPUs and RCCL all-gathers inside the
decode hipGraph (the north star's partition; strong scaling: the same stream at every N), timed in
scripts/tp_leg.py children (one per rank, time-limited) with the bench's prompt, warmup and steps,
every rank's logits checked against the unsplit engine first (a mismatch exits 3 and the line says
so).  `replicas` keeps N independent streams (one per GPU, weak scaling); the `tp_decode` leg runs
BASELINE config 4 — Gemma-7B, row-split the same way.  Rank 0 prints ONE JSON line.
"""
import argparse
import ctypes as C
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "gemma.ggml_amd", "python"))

METRIC = "decode tok/s + prefill tok/s, Gemma-2B Q4_0, 1/2/4/8 MI355X; %HBM roofline"
GEMMA_2B = dict(n_layer=18, n_embd=2048, n_head=8, n_head_kv=1, head_dim=256, n_ff=16384, n_vocab=256000)
GEMMA_7B = dict(n_layer=28, n_embd=3072, n_head=16, n_head_kv=16, head_dim=256, n_ff=24576, n_vocab=256000)
HBM_PEAK_GBS = 8000.0          # MI355X_MICROARCH.md: HBM3E 8.0 TB/s spec (6.29 TB/s measured copy)
KERNEL_NAMES = {0: "ffn gate/up matvec (+norm, +gelu*mul)", 1: "ffn down matvec (+resid)",
                2: "qkv matvec (+norm)", 3: "attn-out matvec (+resid)", 4: "logits matvec (+argmax)"}
KERNEL_CALLS_PER_TOKEN = {0: 18, 1: 18, 2: 18, 3: 18, 4: 1}


def log(msg):
    """progress on stderr (the JSON line stays the only stdout line)"""
    print(f"[bench {time.strftime('%H:%M:%S')}] {msg}", file=sys.stderr, flush=True)


def make_prompt(n, n_vocab, seed=1):
    """Synthetic prompt: BOS=2 then uniform ids in [3, n_vocab) (DESIGN.md §Synthetic inputs)."""
    M = (1 << 64) - 1

    def sm(x):
        x = (x + 0x9E3779B97F4A7C15) & M
        z = x
        z = ((z ^ (z >> 30)) * 0xBF58476D1CE4E5B9) & M
        z = ((z ^ (z >> 27)) * 0x94D049BB133111EB) & M
        return z ^ (z >> 31)

    base = sm(seed)
    return [2] + [3 + sm((base + i) & M) % (n_vocab - 3) for i in range(1, n)]


def _cpu_model():
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown"


def _pick_cpus(n):
    """n CPUs of this process's affinity set, one per physical core (SMT siblings skipped), lowest
    ids first: the CPU legs run pinned so that repeated runs see the same cores."""
    try:
        allowed = sorted(os.sched_getaffinity(0))
    except AttributeError:
        return None
    picked, seen = [], set()
    for c in allowed:
        try:
            with open(f"/sys/devices/system/cpu/cpu{c}/topology/thread_siblings_list") as f:
                sib = f.read().strip()
        except OSError:
            sib = str(c)
        if sib in seen:
            continue
        seen.add(sib)
        picked.append(c)
        if len(picked) == n:
            return picked
    for c in allowed:  # fewer physical cores than n: SMT siblings too (never fewer CPUs than threads)
        if len(picked) == n:
            break
        if c not in picked:
            picked.append(c)
    return sorted(picked)


def cpu_baseline(n_prompt=128, n_decode=32, threads=4, q8_decode=16, reps=3):
    """Oracle (CPU restatement of the reference CPU + thread_pool path) on the host cores, BASELINE.md §2.

    Config 1: Gemma-2B Q4_0 synthetic weights, the 128-token synthetic prompt (seed 1) as ONE prefill
    graph (logits for every row, as src/gemma_model.cpp:740 computes them), then n_decode greedy
    DECODE steps (bounded sample of the 128 of config 1: each step's cost is flat in this range).
    Timed with std::chrono like src/gemma_model.cpp:552-572.  Every leg runs pinned
    (os.sched_setaffinity before its pool's threads start) to one CPU per physical core.  Runs (other
    ops always on one thread, src/macro.h:20):
      ref_pool x4   mul_mat on the reference's 4-worker task pool (src/macro.h:21), `reps` times:
                    "value" is the MEDIAN, "spread" = (max - min) / median
      ref_pool xN   the same pool with every core this process may use (nproc, capped by the box's share)
      spin_pool xN  the same row split on a spin fork-join pool (oracle/hpc_cpu.cpp spin_pool; NOT the
                    reference's pool, the "fixed" figure)
    and the Q8_0 weights (config 5) on ref_pool x4 and spin_pool xN.  Each run carries the decode
    steps' mul_mat profile: wall time, the slowest share's compute time, and the rest ("pool_s": the
    wake/hand-off latency of the pool; 415 mul_mat calls per token, 288 of them tiny per-head
    attention products).  Configs 3 and 4 on the CPU are bounded samples (cpu_prefill_2048 and
    cpu_decode_7b below), extrapolated from a 1- or 2-layer model with a 16,000-row output."""
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    import ctypes as C
    import numpy as np
    import oracle_ctypes as O
    nproc = os.cpu_count() or 1
    try:
        allowed = len(os.sched_getaffinity(0))
        saved_aff = os.sched_getaffinity(0)
    except AttributeError:
        allowed, saved_aff = nproc, None
    share = int(os.environ.get("OMP_NUM_THREADS", "0") or 0) or allowed
    all_threads = max(1, min(allowed, share))
    L = O.lib()
    prompt = np.array(make_prompt(n_prompt, GEMMA_2B["n_vocab"]), dtype=np.int32)

    def pin(th):
        """the reference-pool x4 legs run pinned (reproducible medians); the all-core diagnostics run on
        the process's whole affinity set: a spin pool pinned to as many CPUs as it has threads shares
        them with the runtime's own threads and measured 0.28 tok/s on the box (2 min)"""
        if saved_aff is None:
            return None
        if th != threads:
            os.sched_setaffinity(0, saved_aff)
            return None
        cpus = _pick_cpus(th)
        if cpus:
            os.sched_setaffinity(0, cpus)  # the pool's threads start after this and inherit it
        return cpus

    def run(m, pool, th, nd, prm=prompt, n_pr=n_prompt):
        log(f"cpu run: {('ref_pool', 'spin_pool')[pool]} x{th}, prompt {n_pr}, {nd} decode steps")
        cpus = pin(th)
        toks = np.zeros(n_pr + nd + 2, dtype=np.int32)
        pre = C.c_double()
        prof = np.zeros(6)
        L.orc_set_pool(pool)
        dec_s = L.orc_bench_run(m.h, O.ptr(prm), n_pr, nd, th, O.ptr(toks), C.byref(pre), O.ptr(prof))
        L.orc_set_pool(0)
        L.orc_set_threads(1)  # the next leg's pool is created afresh under its own affinity
        return {"pool": ("ref_pool", "spin_pool")[pool], "threads": th, "pinned_cpus": cpus,
                "decode_tok_s": round(nd / dec_s, 3) if nd else None, "decode_s": dec_s, "prefill_s": pre.value,
                "prefill_tok_s": round(n_pr / pre.value, 3), "first_tokens": toks[n_pr:n_pr + 4].tolist(),
                "decode_profile_ms_per_token": {
                    "total": round(dec_s / nd * 1e3, 3),
                    "mul_mat_wall": round(prof[1] / nd * 1e3, 3),
                    "mul_mat_slowest_share": round(prof[2] / nd * 1e3, 3),
                    "pool_s": round((prof[1] - prof[2]) / nd * 1e3, 3),
                    "attention_mul_mat_wall": round(prof[4] / nd * 1e3, 3),
                    "serial_ops": round((dec_s - prof[1]) / nd * 1e3, 3),
                    "mul_mat_calls": int(round((prof[0] + prof[3]) / nd))} if nd else None}

    def logits_mm_s(E, V, T, th):
        """one orc_mul_mat of a V x E Q4_0 output matrix over T columns on the reference pool (s)."""
        pin(th)
        rng = np.random.default_rng(3)
        W = O.quantize((rng.standard_normal((V, E)) * 0.02).astype(np.float32), "q4_0_ref")
        X = rng.standard_normal((T, E)).astype(np.float32)
        wdata, rs = O.mul_mat_init(O.Q4_0, X)
        dst = np.zeros((T, V), dtype=np.float32)
        L.orc_set_threads(th)
        t0 = time.perf_counter()
        L.orc_mul_mat(V, T, 1, W.shape[1], T, V * 4, V * 4 * T, rs, E, O.ptr(W), O.ptr(dst), O.Q4_0, O.ptr(wdata), 1)
        dt = time.perf_counter() - t0
        L.orc_set_threads(1)
        return dt

    try:
        log("cpu: oracle model (Gemma-2B Q4_0)")
        m = O.Model(O.make_config(GEMMA_2B, n_ctx=512))
        heads = [run(m, 0, threads, n_decode) for _ in range(reps)]
        vals = sorted(r["decode_tok_s"] for r in heads)
        med = vals[len(vals) // 2]
        pvals = sorted(r["prefill_tok_s"] for r in heads)
        runs = list(heads)
        if all_threads != threads:
            runs.append(run(m, 0, all_threads, n_decode))
        runs.append(run(m, 1, all_threads, n_decode))
        m.close()
        q8 = []
        if q8_decode > 0:
            m = O.Model(O.make_config(GEMMA_2B, n_ctx=512, wtype=O.Q8_0))
            q8 = [run(m, 0, threads, q8_decode), run(m, 1, all_threads, q8_decode)]
            m.close()

        # config 3 on the CPU: T = 2048 prefill, bounded sample = ONE layer + a 16,000-row output at
        # T = 2048 on the reference pool; full = 18 x layer + (256,000 / 16,000) x output GEMM
        V_S, T3 = 16000, 2048
        c3 = None
        try:
            log('cpu: config 3 sample (1 layer at T = 2048)')
            one = dict(GEMMA_2B, n_layer=1, n_vocab=V_S)
            m = O.Model(O.make_config(one, n_ctx=T3 + 64))
            pr3 = np.array(make_prompt(T3, V_S, seed=2), dtype=np.int32)
            r3 = run(m, 0, threads, 0, prm=pr3, n_pr=T3)
            m.close()
            lg = logits_mm_s(GEMMA_2B["n_embd"], V_S, T3, threads)
            layer = max(r3["prefill_s"] - lg, 1e-9)
            full = GEMMA_2B["n_layer"] * layer + (GEMMA_2B["n_vocab"] / V_S) * lg
            c3 = {"value": round(T3 / full, 3), "unit": "tok/s", "est_s": round(full, 2), "cores": threads,
                  "sample_layer_s": round(layer, 3), "sample_output_gemm_s": round(lg, 3),
                  "sample": f"BASELINE config 3 on the CPU, extrapolated: one Gemma-2B Q4_0 layer + a {V_S}-row tied "
                            f"output at T = {T3} through the oracle's prefill graph on the reference's {threads}-worker "
                            f"pool ({r3['prefill_s']:.2f} s), minus that output GEMM timed alone; full = 18 x layer + "
                            f"{GEMMA_2B['n_vocab'] // V_S} x output GEMM"}
        except Exception as ex:
            c3 = {"error": str(ex)[:200]}

        # config 4 on the CPU: Gemma-7B Q4_0 batch-1 decode (one process, the reference pool; the
        # reference has no multi-device path), bounded sample = 2 of 28 layers + a 16,000-row output
        c4 = None
        try:
            nl, nd7, np7 = 2, 16, 16
            log('cpu: config 4 sample (2 Gemma-7B layers)')
            two = dict(GEMMA_7B, n_layer=nl, n_vocab=V_S)
            m = O.Model(O.make_config(two, n_ctx=128))
            pr7 = np.array(make_prompt(np7, V_S), dtype=np.int32)
            r7 = run(m, 0, threads, nd7, prm=pr7, n_pr=np7)
            m.close()
            lg7 = logits_mm_s(GEMMA_7B["n_embd"], V_S, 1, threads)
            step = r7["decode_s"] / nd7
            layer7 = max(step - lg7, 1e-9) / nl
            full7 = GEMMA_7B["n_layer"] * layer7 + (GEMMA_7B["n_vocab"] / V_S) * lg7
            c4 = {"value": round(1.0 / full7, 3), "unit": "tok/s", "est_ms_per_token": round(full7 * 1e3, 2),
                  "cores": threads, "sample_layer_ms": round(layer7 * 1e3, 3), "sample_output_ms": round(lg7 * 1e3, 3),
                  "sample": f"BASELINE config 4 on the CPU (one host, reference pool x{threads}), extrapolated: "
                            f"{nl} Gemma-7B Q4_0 layers + a {V_S}-row output, {nd7} greedy decode steps after a "
                            f"{np7}-token prompt, minus that output matvec timed alone; full = 28 x layer + "
                            f"{GEMMA_7B['n_vocab'] // V_S} x output"}
        except Exception as ex:
            c4 = {"error": str(ex)[:200]}
    finally:
        if saved_aff is not None:
            os.sched_setaffinity(0, saved_aff)
    for r in runs + q8:
        r.pop("decode_s", None), r.pop("prefill_s", None)
    return {"value": med, "unit": "tok/s", "cores": threads, "kind": "port",
            "reps": reps, "reps_decode_tok_s": [r["decode_tok_s"] for r in heads],
            "spread": round((vals[-1] - vals[0]) / med, 4) if med else None,
            "sample": f"BASELINE config 1: Gemma-2B Q4_0 synthetic weights, {n_prompt}-token prompt prefilled as one graph, "
                      f"then {n_decode} greedy decode steps (of config 1's 128; per-step cost is flat), mul_mat on "
                      f"the reference's {threads}-worker task pool (oracle/ restatement of src/hpc.cpp + src/thread_pool.cpp, "
                      f"AVX2 vec_dot), other ops on 1 thread; median of {reps} runs pinned to {threads} physical cores",
            "prefill_tok_s": pvals[len(pvals) // 2], "cpu_model": _cpu_model(), "nproc": nproc,
            "affinity_cpus": allowed, "runs": runs,
            "q8_0": {"value": q8[0]["decode_tok_s"] if q8 else None, "unit": "tok/s",
                     "sample": f"BASELINE config 5: Gemma-2B Q8_0, same prompt, {q8_decode} decode steps", "runs": q8},
            "prefill_2048": c3, "decode_7b": c4,
            "thread_scaling_note": ("decode does not scale past ~4 reference-pool workers because each of the 415 "
                                    "mul_mat calls per token pays a packaged_task + mutex + condvar wake per worker "
                                    "(pool_s grows with the worker count, and the 288 per-head attention products are "
                                    "almost all pool_s); prefill (T = 128 columns per call) amortises it. spin_pool "
                                    "removes the wake cost with the same row split and bit-identical tokens")}


# MFMA dense peaks (MI355X_MICROARCH §Matrix cores): BF16/F16 ~2.5 PF; I8 = 2x the BF16 rate per clock
MFMA_PEAK_TOPS = {"i8": 5000.0, "f16": 2500.0}
GEMMA_2B_MACS_PER_TOKEN = 2506096640  # every weight of the 18 layers + the tied output


def prefill_roofline(T, prefill):
    """Prefill against the MFMA roofline: algorithmic ops = 2*T*MACs/token for the weight
    GEMMs (logits for every row, src/gemma_model.cpp:740) + the full masked attention, 18 layers x
    (KQ + KQV) x 2 flops x 8 heads x 256 x T^2; plus the PMC MFMA/LDS utilisation of the exact GEMM
    from the committed profile (profiles/r02/pmc_prefill.json, scripts/pmc_prefill.sh)."""
    gemm_ops = 2.0 * T * GEMMA_2B_MACS_PER_TOKEN
    attn_ops = 18 * 4 * 8 * 256 * float(T) * T
    out = {"bound": "mfma", "unit": "TOP/s", "algo_ops": gemm_ops + attn_ops, "gemm_ops": gemm_ops, "attn_ops": attn_ops,
           "peak_i8_dense": MFMA_PEAK_TOPS["i8"], "peak_f16_dense": MFMA_PEAK_TOPS["f16"]}
    for name in ("exact", "fast"):
        if name in prefill:
            a = out["algo_ops"] / (prefill[name]["ms"] * 1e-3) / 1e12
            out[name] = {"achieved": round(a, 1), "frac_i8": round(a / MFMA_PEAK_TOPS["i8"], 4),
                         "frac_f16": round(a / MFMA_PEAK_TOPS["f16"], 4)}
    out["achieved"] = out["exact"]["achieved"]
    out["peak"] = MFMA_PEAK_TOPS["i8"]
    out["frac"] = out["exact"]["frac_i8"]
    out["pmc_exact_gemm"] = None
    out["pmc_exact_attention"] = None
    path = latest_profile("pmc_prefill_q4_0.json")
    try:
        with open(path) as f:
            pmc = json.load(f)
        keys = ("mfma_util", "lds_busy", "lds_bank_conflict_frac", "valu_inst_per_wave_cycle", "wait_any_frac", "what")
        src = os.path.relpath(path, ROOT)
        for names, field in ((("k_gemm_x4", "k_gemm_x<", "k_gemm_x"), "pmc_exact_gemm"),
                             (("k_attn_mx", "k_attn_rows"), "pmc_exact_attention")):
            k_name = next((n for n in names if n in pmc), None)
            if k_name:
                out[field] = dict({k: pmc[k_name][k] for k in keys if k in pmc[k_name]}, kernel=k_name, source=src)
    except Exception:
        pass
    return out


def latest_profile(name):
    """profiles/rNN/<name> of the newest round that has it (committed and shipped with the tree)."""
    pdir = os.path.join(ROOT, "profiles")
    try:
        rounds = sorted((d for d in os.listdir(pdir) if d.startswith("r") and d[1:].isdigit()), reverse=True)
    except OSError:
        rounds = []
    for d in rounds:
        path = os.path.join(pdir, d, name)
        if os.path.exists(path):
            return path
    return os.path.join(pdir, name)


def load_graph_profile():
    """the per-class table of the benched path (hipGraph replays under rocprofv3 --kernel-trace,
    scripts/decode_prof.py + scripts/decode_classes.py) from the newest profiles/rNN, or None"""
    path = latest_profile("decode_kernels_graph.json")
    try:
        with open(path) as f:
            d = json.load(f)
        d["source_file"] = os.path.relpath(path, ROOT)
        return d
    except Exception:
        return None


def load_traffic(kernel_id):
    """HBM bytes per launch of the roofline kernel from the committed PMC summary (or None)."""
    path = latest_profile("pmc_traffic.json")
    try:
        with open(path) as f:
            d = json.load(f)
        return d.get("per_launch_bytes", {}).get(str(kernel_id))
    except Exception:
        return None


def run_tp_leg(args, world, rank, model="7b", steps=None, warmup=4, prompt=16, port_offset=1009, layouts=None):
    """Every rank starts scripts/tp_leg.py as a child (its own gloo rendezvous on another port) and
    waits with a time limit: a hung RCCL collective costs the leg, never the bench line."""
    import subprocess
    env = dict(os.environ)
    if world > 1:
        env["MASTER_PORT"] = str(int(os.environ.get("MASTER_PORT", "29500")) + port_offset)
    cmd = [sys.executable, os.path.join(ROOT, "scripts", "tp_leg.py"), str(steps or args.tp_steps), args.wtype,
           "0" if args.no_tune else "1", model, str(warmup), str(prompt)]
    if layouts:
        cmd.append(",".join(str(v) for v in layouts))
    try:
        r = subprocess.run(cmd, env=env, capture_output=True, text=True, timeout=args.tp_timeout)
    except subprocess.TimeoutExpired:
        return {"error": f"timed out after {args.tp_timeout} s"}
    if r.returncode != 0:
        if r.returncode == 3 and rank == 0:  # parity mismatch: the leg's own error object
            try:
                return dict(json.loads(r.stdout.strip().splitlines()[-1]), exit=3)
            except Exception:
                pass
        return {"error": (r.stderr or r.stdout)[-300:], "exit": r.returncode}
    if rank != 0:
        return None
    try:
        return json.loads(r.stdout.strip().splitlines()[-1])
    except Exception as ex:  # reported, never fatal to the headline line
        return {"error": f"unparsable leg output: {ex}"}


def merge_legs(rccl, p2p):
    """The row-split headline from its two child legs: the RCCL layouts (0, 1) and the peer-to-peer
    layouts (2, 3) run in separate processes, so a p2p transport that faults over a node's xGMI costs
    only its own layouts.  The faster successful leg is the line; the other's per-layout rates and
    drops are merged in, and a failed leg's error is kept under `failed_legs`."""
    ok = [d for d in (rccl, p2p) if d and "tok_s" in d]
    bad = {name: d for name, d in (("rccl", rccl), ("p2p", p2p)) if d and "tok_s" not in d}
    if not ok:
        return rccl if rccl is not None else p2p
    best = dict(max(ok, key=lambda d: d["tok_s"]))
    rates, dropped = {}, {}
    for d in ok:
        rates.update(d.get("layouts_tok_s") or {})
        dropped.update(d.get("layouts_dropped") or {})
    best["layouts_tok_s"] = rates or None
    best["layouts_dropped"] = dropped
    if bad:
        best["failed_legs"] = bad
    return best


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=64)
    ap.add_argument("--warmup", type=int, default=8)
    ap.add_argument("--prompt", type=int, default=128)
    ap.add_argument("--ctx", type=int, default=512)
    ap.add_argument("--wtype", choices=["q4_0", "q8_0"], default="q4_0")
    ap.add_argument("--no-cpu", action="store_true", help="skip the CPU baseline leg")
    ap.add_argument("--kernel-iters", type=int, default=50)
    ap.add_argument("--prefill", type=int, default=2048, help="prefill leg prompt length (0 = skip)")
    ap.add_argument("--ggml-steps", type=int, default=64, help="decode steps of the ggml-API drop-in leg (0 = skip)")
    ap.add_argument("--no-tune", action="store_true", help="default launch plan instead of the measured one")
    ap.add_argument("--tp-steps", type=int, default=48, help="Gemma-7B row-split decode leg steps (0 = skip)")
    ap.add_argument("--q8-steps", type=int, default=48, help="Gemma-2B Q8_0 decode leg steps (0 = skip)")
    ap.add_argument("--tp-timeout", type=int, default=360, help="time limit of the TP leg's child processes (s)")
    args = ap.parse_args()

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    dist = None
    if world > 1:
        import torch.distributed as dist_mod
        dist = dist_mod
        dist.init_process_group(backend="gloo", init_method="env://")
    import torch

    import gemma_hip as G
    wtype = G.GGML_TYPE_Q4_0 if args.wtype == "q4_0" else G.GGML_TYPE_Q8_0
    if args.prompt + args.warmup + args.steps + 8 >= args.ctx:
        args.ctx = ((args.prompt + args.warmup + args.steps + 64) // 32 + 1) * 32

    def barrier_sync():
        torch.cuda.synchronize(local_rank) if torch.cuda.is_available() else None
        if dist is not None:
            dist.barrier()

    # N > 1: the headline stream, Gemma-2B row-split over the N GPUs (children, before this
    # process's own engines take the GPUs' time)
    tp2 = None
    if world > 1:
        log(f'row-split Gemma-2B stream over {world} GPUs')
        tp2 = run_tp_leg(args, world, rank, model="2b", steps=args.steps, warmup=args.warmup, prompt=args.prompt,
                         port_offset=1013, layouts=(0, 1))
        log(f'row-split Gemma-2B stream over {world} GPUs, peer-to-peer layouts')
        tp2p = run_tp_leg(args, world, rank, model="2b", steps=args.steps, warmup=args.warmup, prompt=args.prompt,
                          port_offset=1017, layouts=(2, 3))
        tp2 = merge_legs(tp2, tp2p) if rank == 0 else None

    log('engine: Gemma-2B decode')
    eng = G.Engine(GEMMA_2B, n_ctx=args.ctx, wtype=wtype, device=local_rank)
    plan = eng.tune(8) if not args.no_tune else eng.plan()  # engine setup (untimed): launch shapes
    prompt = make_prompt(args.prompt, GEMMA_2B["n_vocab"])
    eng.begin(prompt)
    # prompt pass on the ordered (bit-exact) per-token path; timed as the serial prefill figure
    t0 = time.perf_counter()
    eng.step(args.prompt, use_graph=True)
    prefill_serial_s = time.perf_counter() - t0
    prefill_tok_s = None
    eng.step(args.warmup, use_graph=True)

    barrier_sync()
    t0 = time.perf_counter()
    eng.step(args.steps, use_graph=True)
    eng.L.gemma_engine_sync(eng.h)
    barrier_sync()
    dt = time.perf_counter() - t0
    try:  # kernel launches per decode token (the captured graph's kernel nodes; outside the timed region)
        launches = eng.graph_kernels()
    except Exception:  # reported as null, never fatal
        launches = None
    if dist is not None:
        t = torch.tensor([dt], dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        dt = float(t.item())

    # row-split TP leg (BASELINE config 4): Gemma-7B Q4_0 batch-1 decode, weights row-split across
    # the job's GPUs with RCCL all-gathers (one rank per GPU; at N = 1 the same engine unsplit)
    log('tp leg')
    tp = None
    if args.tp_steps > 0:
        tp = run_tp_leg(args, world, rank)

    # second quant format (BASELINE config 5): the same decode with Q8_0 weights (2.66 GB/token)
    log('q8_0 leg')
    q8 = None
    if args.wtype == "q4_0" and args.q8_steps > 0:
        try:
            qe = G.Engine(GEMMA_2B, n_ctx=args.ctx, wtype=G.GGML_TYPE_Q8_0, device=local_rank)
            qplan = qe.tune(6) if not args.no_tune else qe.plan()
            qe.begin(prompt)
            qe.step(args.prompt + args.warmup, use_graph=True)
            qe.L.gemma_engine_sync(qe.h)
            t0 = time.perf_counter()
            qe.step(args.q8_steps, use_graph=True)
            qe.L.gemma_engine_sync(qe.h)
            qdt = time.perf_counter() - t0
            qus, qalgo = qe.time_kernel(0, args.kernel_iters)
            qe.close()
            q8 = {"model": "Gemma-2B Q8_0", "tok_s": round(args.q8_steps / qdt, 2),
                  "ms_per_token": round(qdt / args.q8_steps * 1e3, 4), "steps": args.q8_steps,
                  "token_weight_bytes": 2662727680,
                  "gate_up_matvec": {"avg_us": round(qus, 3), "GB/s": round(qalgo / (qus * 1e-6) / 1e9, 1)},
                  "launch_plan": qplan}
        except Exception as ex:  # reported, never fatal to the headline line
            q8 = {"error": str(ex)[:300]}

    # llama.cpp's Q4_0 file layout: the same decode with a Q6_K token_embd / tied output
    # (1,544,847,360 weight bytes per token; logits through Q8_K INIT + the K-quant matvec)
    log('q6_K output leg')
    q6o = None
    if args.wtype == "q4_0" and args.q8_steps > 0:
        try:
            ke = G.Engine(GEMMA_2B, n_ctx=args.ctx, wtype=G.GGML_TYPE_Q4_0, device=local_rank,
                          out_type=G.GGML_TYPE_Q6_K)
            kplan = ke.tune(6) if not args.no_tune else ke.plan()
            ke.begin(prompt)
            ke.step(args.prompt + args.warmup, use_graph=True)
            ke.L.gemma_engine_sync(ke.h)
            t0 = time.perf_counter()
            ke.step(args.q8_steps, use_graph=True)
            ke.L.gemma_engine_sync(ke.h)
            kdt = time.perf_counter() - t0
            ke.close()
            q6o = {"model": "Gemma-2B Q4_0 layers + Q6_K token_embd/output (llama.cpp layout)",
                   "tok_s": round(args.q8_steps / kdt, 2), "ms_per_token": round(kdt / args.q8_steps * 1e3, 4),
                   "steps": args.q8_steps, "token_weight_bytes": 1544847360, "launch_plan": kplan}
        except Exception as ex:  # reported, never fatal to the headline line
            q6o = {"error": str(ex)[:300]}

    # the reference's shipped format (src/app.cpp:36, gemma-2b-it-q4_k_m): K-quant layers (Q4_K q/k/o/
    # gate/up, Q6_K v/down) and a Q6_K token_embd / output, token by token through the K-quant matvecs
    log('q4_k_m leg')
    kqm = None
    if args.wtype == "q4_0" and args.q8_steps > 0:
        try:
            E, F, qw, kvw, V = (GEMMA_2B[k] for k in ("n_embd", "n_ff", "n_head", "n_head_kv", "n_vocab"))
            qw, kvw = qw * GEMMA_2B["head_dim"], kvw * GEMMA_2B["head_dim"]
            q4k = (qw * E + kvw * E + E * qw + 2 * F * E) * 144 // 256
            q6k = (kvw * E + E * F) * 210 // 256
            kbytes = GEMMA_2B["n_layer"] * (q4k + q6k) + V * E * 210 // 256
            ke = G.Engine(GEMMA_2B, n_ctx=args.ctx, wtype=G.GGML_TYPE_Q4_K, device=local_rank)
            # the prompt through the batched K-quant prefill (all prompt columns per launch; timed
            # after one untimed pass), then greedy decode
            ke.begin(prompt)
            ke.prefill(args.prompt)
            ke.begin(prompt)
            ke.L.gemma_engine_sync(ke.h)
            tp0 = time.perf_counter()
            ke.prefill(args.prompt)
            kpf_s = time.perf_counter() - tp0
            ke.step(args.warmup, use_graph=True)
            ke.L.gemma_engine_sync(ke.h)
            t0 = time.perf_counter()
            ke.step(args.q8_steps, use_graph=True)
            ke.L.gemma_engine_sync(ke.h)
            kdt = time.perf_counter() - t0
            k_launches = ke.graph_kernels()
            ke.close()
            # BASELINE config 3's prompt length in the shipped format: the batched exact prefill at
            # T = args.prefill (one untimed pass, then one timed)
            kp2 = None
            if args.prefill > 0:
                kpe = G.Engine(GEMMA_2B, n_ctx=args.prefill + 64, wtype=G.GGML_TYPE_Q4_K, device=local_rank)
                kpp = make_prompt(args.prefill, GEMMA_2B["n_vocab"], seed=2)
                kpe.begin(kpp)
                kpe.prefill(args.prefill)
                kpe.begin(kpp)
                kpe.L.gemma_engine_sync(kpe.h)
                tp0 = time.perf_counter()
                kpe.prefill(args.prefill)
                kp2_s = time.perf_counter() - tp0
                kpe.close()
                kp2 = {"T": args.prefill, "ms": round(kp2_s * 1e3, 3), "tok_s": round(args.prefill / kp2_s, 1),
                       "exact": True}
            kqm = {"model": "Gemma-2B Q4_K_M layout (Q4_K/Q6_K layers, Q6_K output; the reference's shipped format)",
                   "launches_per_token": k_launches,
                   "tok_s": round(args.q8_steps / kdt, 2), "ms_per_token": round(kdt / args.q8_steps * 1e3, 4),
                   "steps": args.q8_steps, "token_weight_bytes": kbytes,
                   "weight_GB_s": round(kbytes * args.q8_steps / kdt / 1e9, 1),
                   "prefill": {"T": args.prompt, "ms": round(kpf_s * 1e3, 3),
                               "tok_s": round(args.prompt / kpf_s, 1), "exact": True},
                   "prefill_long": kp2}
        except Exception as ex:  # reported, never fatal to the headline line
            kqm = {"error": str(ex)[:300]}

    # prefill leg (BASELINE config 3): batched prefill of a 2048-token synthetic prompt, logits for
    # every row as the reference computes them.  "exact": bit-identical to the CPU path (the
    # headline prefill_tok_s); "fast": int8/f16 MFMA, fp32 summation order differs
    log('prefill leg')
    prefill = None
    if args.prefill > 0:
        pe = G.Engine(GEMMA_2B, n_ctx=args.prefill + 64, wtype=wtype, device=local_rank)
        pprompt = make_prompt(args.prefill, GEMMA_2B["n_vocab"], seed=2)
        prefill = {"T": args.prefill}
        for name, exact in (("exact", True), ("fast", False)):
            times = []
            for rep in range(3):
                pe.begin(pprompt)
                pe.L.gemma_engine_sync(pe.h)
                t0 = time.perf_counter()
                pe.prefill(args.prefill, exact=exact)
                times.append(time.perf_counter() - t0)
            best = min(times[1:])
            prefill[name] = {"tok_s": round(args.prefill / best, 1), "ms": round(best * 1e3, 3)}
        pe.close()
        prefill["exact"]["path"] = ("ggml AVX2 lane order: v_mfma_f32_16x16x4_4b_f16 GEMMs (one instruction block = one AVX2 "
                                    "lane) + fmaf lane chains, exact attention on f32 MFMA; bit-identical logits to the CPU path")
        prefill["fast"]["path"] = ("int8 MFMA GEMMs + f16 MFMA attention; fp32 order differs from the CPU "
                                   "path (DESIGN.md Prefill)")
        prefill["tok_s"] = prefill["exact"]["tok_s"]
        prefill["ms"] = prefill["exact"]["ms"]
        prefill["roofline"] = prefill_roofline(args.prefill, prefill)

    # ggml-API drop-in leg: the reference's graph code (tests/ggml_driver, restating
    # src/gemma_model.cpp) driving ggml_graph_compute_with_ctx on a Gemma-2B Q4_0 GGUF of the same
    # synthetic weights; timed like src/gemma_model.cpp:552-572 (graph build + compute + greedy sample)
    log('ggml path leg')
    ggml_leg = None
    if args.ggml_steps > 0 and rank == 0 and world == 1:
        import re
        import subprocess
        import tempfile
        with tempfile.TemporaryDirectory(dir=os.environ.get("TMPDIR", "/tmp")) as td:
            try:
                r = subprocess.run([sys.executable, os.path.join(ROOT, "scripts", "ggml_path_bench.py"), str(args.ggml_steps), td],
                                   capture_output=True, text=True, timeout=600)
                mt = re.search(r"prefill_ms ([0-9.]+) prompt (\d+) decode_ms ([0-9.]+) steps (\d+) decode_tok_s ([0-9.]+)"
                               r"(?: upload_ms ([0-9.]+))?(?: first_prefill_ms ([0-9.]+) rounds (\d+))?", r.stdout)
                if mt:
                    ggml_leg = {"decode_tok_s": float(mt.group(5)), "prefill_tok_s": round(int(mt.group(2)) / float(mt.group(1)) * 1e3, 1),
                                "prefill_ms": float(mt.group(1)),
                                "upload_ms": float(mt.group(6)) if mt.group(6) else None,
                                "first_round_prefill_ms": float(mt.group(7)) if mt.group(7) else None,
                                "rounds": int(mt.group(8)) if mt.group(8) else 1,
                                "prefill_timing": "the last of `rounds` begin_one_round_inference rounds on the loaded model "
                                                  "(compute: graph build, executor, the 128 x 256000 logits rows written to the "
                                                  "host tensor); the first round also creates the device engine "
                                                  "(first_round_prefill_ms)",
                                "upload": "hpc_register_weight of every quantized weight at model load (INTEGRATION.md §1), "
                                          "outside the reference loop's prefill timer; the first graph's engine copies them "
                                          "device to device",
                                "prompt": int(mt.group(2)), "steps": int(mt.group(4)),
                                "path": "ggml_graph_compute_with_ctx recognises the Gemma graph and runs the device-resident engine "
                                        "over the graph's weights and KV-cache mirrors (ggml_api.cpp try_fast); includes the "
                                        "reference loop's host graph build and greedy sample"}
                else:
                    ggml_leg = {"error": (r.stderr or r.stdout)[-300:]}
            except Exception as ex:  # reported, never fatal to the headline line
                ggml_leg = {"error": str(ex)[:300]}

    # K-quant leg: Q4_K / Q6_K x Q8_K matvec alone at Gemma-2B shapes, cold weights
    log('kquant matvec leg')
    kquant = {}
    for t, name in ((G.GGML_TYPE_Q4_K, "q4_K"), (G.GGML_TYPE_Q6_K, "q6_K")):
        for rows, K, nm in ((16384, 2048, "gate"), (2048, 16384, "down"), (256000, 2048, "output")):
            ab = C.c_double()
            us = G.lib().gemma_kq_time(t, rows, K, 30, C.byref(ab))
            if us > 0:
                kquant[f"{name}_{nm}"] = {"us": round(us, 3), "GB/s": round(ab.value / us / 1e3, 1)}

    # roofline leg: each hot matvec timed alone with hipEvents on the engine stream
    log('roofline leg')
    kern = {}
    for k in (0, 1, 2, 3, 4):
        us, algo = eng.time_kernel(k, args.kernel_iters)
        kern[k] = (us, algo)
    dominant = max(kern, key=lambda k: kern[k][0] * KERNEL_CALLS_PER_TOKEN[k])
    us, algo = kern[dominant]
    achieved = algo / (us * 1e-6) / 1e9
    traffic = load_traffic(dominant)
    # measured HBM read roofline on this box: streaming read of 4 GiB (defeats the Infinity Cache)
    hbm_probes = [eng.L.gemma_hbm_read_probe(local_rank, 4 << 30, 5, v) for v in (0, 1)]
    hbm_measured = max(hbm_probes)

    log('cpu baseline')
    cpu = None
    if rank == 0 and world == 1 and not args.no_cpu:
        try:
            cpu = cpu_baseline()
        except Exception as ex:  # the CPU baseline is reported, never the target
            cpu = {"value": None, "error": str(ex)}
    eng.close()

    if rank == 0:
        n_tok = args.steps * world
        rep_tok_s = n_tok / dt  # N independent streams (at N = 1: the headline itself)
        line = {
            "metric": METRIC,
            "value": round(n_tok / dt, 2),
            "unit": "tok/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(dt / args.steps * 1e3, 4),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "i8xi8->i32, f32 accumulate (Q4_0 weights x Q8_0 activations)",
            "data": "synthetic (seeded Gemma-2B-shaped Q4_0 weights generated on device; synthetic prompt)",
            "config": {"workload": f"Gemma-2B {args.wtype.upper()} greedy decode, batch 1, after a "
                                   f"{args.prompt}-token prompt (BASELINE config 2); ordered bit-exact path",
                       "n_ctx": args.ctx, "prompt": args.prompt, "parallelism": f"replicas x{world}"},
            "decode_tok_s": round(n_tok / dt, 2),
            "launches_per_token": launches,
            "prefill_tok_s": prefill["tok_s"] if prefill else None,
            "prefill": prefill,
            "kquant_matvec": kquant,
            "q8_0_decode": q8,
            "q4_0_q6k_output_decode": q6o,
            "q4_k_m_decode": kqm,
            "tp_decode": tp,
            "ggml_path": ggml_leg,
            "ggml_path_decode_tok_s": ggml_leg.get("decode_tok_s") if ggml_leg else None,
            "launch_plan": {k: ({"k_split": v[0], "rows_per_wg": v[1], "image": v[2]} if isinstance(v, tuple) else
                                ("split" if v else "per_head")) for k, v in plan.items()},
            "prefill_serial_tok_s": round(args.prompt / prefill_serial_s, 2),
            "roofline": {"bound": "hbm", "kernel": KERNEL_NAMES[dominant], "achieved": round(achieved, 1),
                         "peak": HBM_PEAK_GBS, "unit": "GB/s", "frac": round(achieved / HBM_PEAK_GBS, 4),
                         "traffic": traffic, "avg_us": round(us, 3), "algo_bytes": int(algo),
                         "measured_peak": round(hbm_measured, 1),
                         "measured_peak_probes": {"vgpr_loads_nt": round(hbm_probes[0], 1), "lds_dma_nt": round(hbm_probes[1], 1),
                                                  "what": "4 GiB streaming reads; measured_peak = the faster (the guide's "
                                                          "float4 copy: 6.29 TB/s)"},
                         "frac_of_measured": round(achieved / hbm_measured, 4) if hbm_measured > 0 else None,
                         "timing": "hipEvents over back-to-back launches rotating over the 18 layers' matrices",
                         "graph_profile": load_graph_profile(),
                         "classes": {KERNEL_NAMES[k]: {"avg_us": round(v[0], 3), "algo_bytes": int(v[1]),
                                                       "GB/s": round(v[1] / (v[0] * 1e-6) / 1e9, 1),
                                                       "frac": round(v[1] / (v[0] * 1e-6) / 1e9 / HBM_PEAK_GBS, 4),
                                                       "frac_of_measured": (round(v[1] / (v[0] * 1e-6) / 1e9 / hbm_measured, 4)
                                                                            if hbm_measured > 0 else None),
                                                       "launches_per_token": KERNEL_CALLS_PER_TOKEN[k],
                                                       "traffic": load_traffic(k)}
                                     for k, v in kern.items()}},
            "kernels_us": {KERNEL_NAMES[k]: round(v[0], 3) for k, v in kern.items()},
            "token_weight_bytes": 1409679360 if args.wtype == "q4_0" else 2662727680,
            "cpu_baseline": cpu,
        }
        line["token_hbm_frac"] = round(line["token_weight_bytes"] * line["value"] / world / 1e9 / HBM_PEAK_GBS, 4)
        line["token_hbm_frac_of_measured"] = (round(line["token_weight_bytes"] * line["value"] / world / 1e9 / hbm_measured, 4)
                                              if hbm_measured > 0 else None)
        if world > 1:
            line["replicas"] = {"value": round(rep_tok_s, 2), "unit": "tok/s", "scaling": "weak",
                                "ms_per_step": round(dt / args.steps * 1e3, 4),
                                "what": f"{world} independent Gemma-2B Q4_0 streams, one per GPU (tokens over all "
                                        f"ranks / max-over-ranks time)", "roofline": line["roofline"]}
            if tp2 and "tok_s" in tp2:
                line["value"] = line["decode_tok_s"] = tp2["tok_s"]
                line["ms_per_step"] = tp2["ms_per_token"]
                line["scaling"] = "strong"
                line["config"]["parallelism"] = tp2.get("parallelism") or f"row-split tp{world}"
                line["config"]["workload"] = (f"ONE Gemma-2B {args.wtype.upper()} greedy decode stream, batch 1, every "
                                              f"weight matrix row-split over {world} GPUs, after a {args.prompt}-token "
                                              f"prompt (BASELINE config 2 partitioned as the north star asks)")
                line["row_split"] = tp2
                if tp2.get("roofline"):
                    line["roofline"] = dict(tp2["roofline"], traffic=None)
                # each token reads the weights once, spread over the N GPUs: against the N GPUs' combined peak
                line["token_hbm_frac"] = round(line["token_weight_bytes"] * line["value"] / world / 1e9 / HBM_PEAK_GBS, 4)
                line["token_hbm_frac_of_measured"] = (round(line["token_weight_bytes"] * line["value"] / world / 1e9 / hbm_measured, 4)
                                                      if hbm_measured > 0 else None)
            else:  # the row-split stream failed: the line says so and reports the replicas
                line["row_split"] = tp2
                line["config"]["parallelism"] = f"replicas x{world} (row-split stream failed, see row_split)"
        print(json.dumps(line), flush=True)
    if dist is not None:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
