#!/bin/bash
export GHIP_ALLOW_ALT_LIB=1  # the A/B libraries are loaded on purpose (gemma_hip.py refuses GHIP_LIB otherwise)
# Same-box A/B of two builds of libgemma_hip.so (ab_libs/libA.so vs libB.so): alternating bench
# runs, decode step time + kernel times.  Usage: bash scripts/ab.sh [extra bench args]
set -o pipefail
OUT=gpurun_out/ab
mkdir -p $OUT
for r in 1 2; do
  for v in A B; do
    GHIP_LIB=ab_libs/lib$v.so timeout -k 10 300 python bench.py --no-cpu --prefill 0 --tp-steps 0 "$@" > $OUT/$v$r.json 2> $OUT/$v$r.err || { tail -5 $OUT/$v$r.err; exit 1; }
    python3 -c "import json; d=json.load(open('$OUT/$v$r.json')); print('$v$r', d['value'], d['ms_per_step'], {k[:10]:v for k,v in d['kernels_us'].items()})"
  done
done
