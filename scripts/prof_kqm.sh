#!/bin/bash
# rocprofv3 kernel stats of the Q4_K_M decode alone (scripts/run_kqm.py), summary to gpurun_out/kqm/
set -o pipefail
mkdir -p gpurun_out/kqm
export TMPDIR=/tmp
timeout -k 10 200 python -u scripts/run_kqm.py 64 > gpurun_out/kqm/plain.txt 2>&1 || exit 1
cat gpurun_out/kqm/plain.txt
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/kqm/prof$KQM_TAG -o run -- python3 scripts/run_kqm.py 64 > gpurun_out/kqm/prof.log 2>&1 || { tail -20 gpurun_out/kqm/prof.log; exit 1; }
python3 scripts/prof_db_summary.py gpurun_out/kqm/prof$KQM_TAG/run_results.db 84 | head -16
