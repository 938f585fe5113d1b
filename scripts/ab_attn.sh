#!/bin/bash
export GHIP_ALLOW_ALT_LIB=1  # the A/B libraries are loaded on purpose (gemma_hip.py refuses GHIP_LIB otherwise)
# attention prefetch-depth experiment: stamps of layer 9 and bench step time for each build
set -o pipefail
mkdir -p gpurun_out/ab
for v in B PF4 PF2; do
  GHIP_LIB=ab_libs/lib$v.so timeout -k 10 200 python tests/stamp_step.py 9 > gpurun_out/ab/st_$v.log 2>&1 || exit 1
  echo "== $v"; grep -A1 "^attention" gpurun_out/ab/st_$v.log
  GHIP_LIB=ab_libs/lib$v.so timeout -k 10 300 python bench.py --no-cpu --prefill 0 --tp-steps 0 > gpurun_out/ab/b_$v.json 2>/dev/null || exit 1
  python3 -c "import json; d=json.load(open('gpurun_out/ab/b_$v.json')); print('$v', d['value'], d['ms_per_step'])"
done
