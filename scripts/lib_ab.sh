#!/bin/bash
export GHIP_ALLOW_ALT_LIB=1  # the A/B libraries are loaded on purpose (gemma_hip.py refuses GHIP_LIB otherwise)
# A/B of two builds on one box: ab_libs/libbase.so (GHIP_LIB) vs the in-tree library, decode bench
# legs, interleaved; optional parity tests of the in-tree build first (TESTS="-k ...")
set -o pipefail
mkdir -p gpurun_out/libab
export TMPDIR=/tmp
if [ -n "$TESTS" ]; then
  timeout -k 10 500 python -u -m pytest -x -q --timeout 200 --timeout-method thread $TESTS > gpurun_out/libab/test.log 2>&1 || { tail -30 gpurun_out/libab/test.log; exit 1; }
  tail -2 gpurun_out/libab/test.log
fi
for rep in 1 2 3; do
  for v in base new; do
    if [ $v = base ]; then export GHIP_LIB=$PWD/ab_libs/libbase.so; else unset GHIP_LIB; fi
    timeout -k 10 240 python bench.py --no-cpu --prefill 0 --tp-steps 0 --q8-steps 0 --ggml-steps 0 ${BENCH_ARGS} > gpurun_out/libab/$v$rep.json 2> gpurun_out/libab/$v$rep.err || { tail -20 gpurun_out/libab/$v$rep.err; exit 1; }
    python3 -c "import json; d=json.load(open('gpurun_out/libab/$v$rep.json')); print('$v', d['value'], d['ms_per_step'], (d.get('q4_k_m_decode') or {}).get('tok_s'))"
  done
done
