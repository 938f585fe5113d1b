#!/bin/bash
# rocprofv3 kernel stats of the Q4_K_M decode alone (scripts/run_kqm.py), summary to gpurun_out/kqm/
set -o pipefail
mkdir -p gpurun_out/kqm
export TMPDIR=/tmp
timeout -k 10 200 python -u scripts/run_kqm.py 64 > gpurun_out/kqm/plain.txt 2>&1 || exit 1
cat gpurun_out/kqm/plain.txt
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/kqm/prof -o run -- python3 scripts/run_kqm.py 64 > gpurun_out/kqm/prof.log 2>&1 || { tail -20 gpurun_out/kqm/prof.log; exit 1; }
f=$(find gpurun_out/kqm/prof -name '*kernel_stats.csv' | head -1)
python3 - "$f" <<'PY'
import csv, sys
rows = list(csv.DictReader(open(sys.argv[1])))
tot = sum(float(r["TotalDurationNs"]) for r in rows)
for r in sorted(rows, key=lambda r: -float(r["TotalDurationNs"]))[:16]:
    print(f'{r["Name"][:70]:70s} {int(r["Calls"]):7d} {float(r["AverageNs"])/1e3:9.3f} us {100*float(r["TotalDurationNs"])/tot:5.1f}%')
PY
