#!/bin/bash
# round-2 quick GPU pass: selected parity tests, then a decode-only bench (tuned plan) -> gpurun_out/$TAG
set -o pipefail
TAG=${1:-r2}; K=${2:-"round_pipelined or mul_mat_quant or tuned_plan"}
OUT=gpurun_out/$TAG; mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -k "$K" > $OUT/pytest.log 2>&1 || { tail -30 $OUT/pytest.log; exit 1; }
tail -2 $OUT/pytest.log
timeout -k 10 300 python bench.py --no-cpu --prefill 0 --tp-steps 0 --q8-steps 0 > $OUT/bench.json 2> $OUT/bench.err || { tail -20 $OUT/bench.err; exit 1; }
python3 -c "import json; d=json.load(open('$OUT/bench.json')); print(d['value'], d['ms_per_step'], d['launch_plan']); print(json.dumps(d['roofline']['classes'], indent=0))"
