"""Per-class decode kernel table from a rocprofv3 kernel trace of scripts/decode_prof.py (VERDICT r4
"Next round" #7): one row per class (qkv, attention, attn-out, gate/up, down, logits, advance) with
the exact kernel template name, launches per token and the average duration over the LAST `steps`
tokens (the decode positions; the prompt's tokens before them are skipped), so every
`roofline.classes` fraction of the bench line can be recomputed from algorithmic bytes / avg µs.

  python3 scripts/decode_classes.py {run_results.db | run_kernel_trace.csv} PROMPT STEPS [plan] [out.json] > decode_kernels.md

With out.json the same table is also written as JSON (bench.py embeds the newest profiles/rNN copy).
"""
import json
import csv
import re
import sys
from collections import OrderedDict

# class: (name pattern, algorithmic bytes per launch: the engine's own count, gemma_engine_time's
# algo_bytes, as the bench line's roofline.classes carries them — weights + f32 inputs + outputs)
CLASSES = OrderedDict([
    ("qkv matvec (+norm)", (r"^k_matvec_rr<2, [13], 0,", 2975744)),
    ("decode attention", (r"^k_attn_head|^k_attn_decode", None)),
    ("attn-out matvec (+resid)", (r"^k_matvec_rr<2, [04], 1, 1,", 2383872)),
    ("ffn gate/up matvec (+norm, +gelu*mul)", (r"^k_matvec<2, \d+, 1, 2,", 37830656)),
    ("ffn down matvec (+resid)", (r"^k_matvec_rr<2, 4, 1, (?!1,)\d+,|^k_matvec<2, \d+, 4, 1,", 18909184)),
    ("logits matvec (+argmax)", (r"^k_matvec<2, \d+, 1, 3,", 295952384)),
    ("advance (argmax merge, next token)", (r"^k_advance", None)),
])


def main():
    path, prompt, steps = sys.argv[1], int(sys.argv[2]), int(sys.argv[3])
    plan = sys.argv[4] if len(sys.argv) > 4 else ""
    jpath = sys.argv[5] if len(sys.argv) > 5 else None
    js = {"source": "rocprofv3 --kernel-trace of scripts/decode_prof.py", "prompt": prompt, "steps": steps, "plan": plan,
          "classes": []}
    rows = []
    if path.endswith(".db"):  # rocprofv3's default rocpd SQLite output: the `kernels` view
        import sqlite3
        rows = [(int(a), int(b), n) for a, b, n in sqlite3.connect(path).execute("select start, end, name from kernels")]
    else:  # --output-format csv: *_kernel_trace.csv
        with open(path) as f:
            for r in csv.DictReader(f):
                if r["Kind"] != "KERNEL_DISPATCH":
                    continue
                rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"]))
    # one naming for both outputs: "k_matvec<...>(ghip::mv_args)" (no "void ", no namespaces)
    rows = [(a, b, n.replace("void ", "", 1).replace("ghip::(anonymous namespace)::", "").replace("ghip::", ""))
            for a, b, n in rows]
    rows.sort()
    # one k_advance closes every token: the last `steps` tokens are the dispatches after the
    # (steps+1)-th last k_advance
    adv = [i for i, (_, _, n) in enumerate(rows) if n.startswith("k_advance")]
    if len(adv) < steps + 1:
        sys.exit(f"only {len(adv)} tokens in the trace")
    lo, hi = adv[-steps - 1] + 1, adv[-1] + 1
    win = rows[lo:hi]
    t_tok = (win[-1][1] - rows[adv[-steps - 1]][1]) / steps / 1e3
    print(f"# Decode kernels per class — `scripts/decode_prof.py` (Gemma-2B Q4_0, prompt {prompt}, "
          f"the last {steps} decode tokens), rocprofv3 --kernel-trace\n")
    if plan:
        print(f"Launch plan (k_split, rows_per_wg, image per class): `{plan}`\n")
    print(f"Token wall time in the trace (k_advance to k_advance): {t_tok:.1f} µs\n")
    js["token_wall_us"] = round(t_tok, 3)
    print("| class | kernel (exact template) | launches / token | avg µs | min µs | max µs | algo bytes / launch | GB/s | frac of 8 TB/s |")
    print("|---|---|---|---|---|---|---|---|---|")
    used = set()
    tot = 0.0
    for cls, (pat, algo) in CLASSES.items():
        rx = re.compile(pat)
        hit = [(s, e, n) for (s, e, n) in win if rx.search(n)]
        for n in sorted(set(n for _, _, n in hit)):
            d = [(e - s) / 1e3 for (s, e, nn) in hit if nn == n]
            used.add(n)
            avg = sum(d) / len(d)
            tot += sum(d) / steps
            gbs = f"{algo / avg / 1e3:.1f}" if algo else "—"
            frac = f"{algo / avg / 1e3 / 8000:.3f}" if algo else "—"
            print(f"| {cls} | `{n}` | {len(d) / steps:g} | {avg:.3f} | {min(d):.3f} | {max(d):.3f} | "
                  f"{algo if algo else '—'} | {gbs} | {frac} |")
            js["classes"].append({"class": cls, "kernel": n, "launches_per_token": len(d) / steps, "avg_us": round(avg, 3),
                                  "min_us": round(min(d), 3), "max_us": round(max(d), 3), "algo_bytes": algo,
                                  "GB/s": round(algo / avg / 1e3, 1) if algo else None,
                                  "frac": round(algo / avg / 1e3 / 8000, 4) if algo else None})
    other = [(s, e, n) for (s, e, n) in win if n not in used]
    for n in sorted(set(n for _, _, n in other)):
        d = [(e - s) / 1e3 for (s, e, nn) in other if nn == n]
        tot += sum(d) / steps
        print(f"| other | `{n}` | {len(d) / steps:g} | {sum(d) / len(d):.3f} | {min(d):.3f} | {max(d):.3f} | — | — | — |")
    print(f"\nSum of kernel time per token: {tot:.1f} µs of {t_tok:.1f} µs (the rest: gaps between launches).")
    js["kernel_sum_us_per_token"] = round(tot, 3)
    if jpath:
        with open(jpath, "w") as f:
            json.dump(js, f, indent=1)


if __name__ == "__main__":
    main()
