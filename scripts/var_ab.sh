#!/bin/bash
export GHIP_ALLOW_ALT_LIB=1  # the A/B libraries are loaded on purpose (gemma_hip.py refuses GHIP_LIB otherwise)
# decode bench: in-tree build vs ab_libs/lib<v>.so variants, interleaved (usage: bash scripts/var_ab.sh v1 v2 ...)
set -o pipefail
mkdir -p gpurun_out/varab
export TMPDIR=/tmp
for rep in 1 2; do
  for v in base "$@"; do
    if [ $v = base ]; then unset GHIP_LIB; else export GHIP_LIB=$PWD/ab_libs/lib$v.so; fi
    timeout -k 10 240 python bench.py --no-cpu --prefill 0 --tp-steps 0 --q8-steps 0 --ggml-steps 0 > gpurun_out/varab/$v$rep.json 2> gpurun_out/varab/$v$rep.err || { tail -20 gpurun_out/varab/$v$rep.err; exit 1; }
    python3 -c "import json; d=json.load(open('gpurun_out/varab/$v$rep.json')); c=d['roofline']['classes']; print('$v', d['value'], d['ms_per_step'], [round(x['avg_us'],2) for x in c.values()])"
  done
done
