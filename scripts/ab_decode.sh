#!/bin/bash
export GHIP_ALLOW_ALT_LIB=1  # the A/B libraries are loaded on purpose (gemma_hip.py refuses GHIP_LIB otherwise)
# Same-box A/B of decode builds ab_libs/lib<v>.so: alternating bench runs (no CPU/prefill/TP legs),
# decode tok/s + per-kernel µs.  usage: bash scripts/ab_decode.sh v1 v2 ... [-- extra bench args]
set -o pipefail
OUT=gpurun_out/ab
mkdir -p $OUT
for r in 1 2; do
  for v in "$@"; do
    GHIP_LIB=ab_libs/lib$v.so timeout -k 10 300 python bench.py --no-cpu --prefill 0 --tp-steps 0 --q8-steps 0 > $OUT/$v$r.json 2> $OUT/$v$r.err || { tail -5 $OUT/$v$r.err; exit 1; }
    python3 -c "import json; d=json.load(open('$OUT/$v$r.json')); print('$v$r', d['value'], d['ms_per_step'], {k[:10]:v for k,v in d['kernels_us'].items()})"
  done
done
