#!/bin/bash
# rocprofv3 kernel trace of one exact (or fast) Gemma-2B prefill pass; prints per-kernel totals.
# usage: bash scripts/prof_prefill.sh <tag> [T] [exact]
set -o pipefail
TAG=$1; T=${2:-2048}; EX=${3:-1}
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof -o run -- python3 scripts/prof_prefill.py $T $EX 1 > $OUT/prof.log 2>&1 || { tail -20 $OUT/prof.log; exit 1; }
grep "^rep" $OUT/prof.log
python3 scripts/trace_groups.py $OUT/prof
