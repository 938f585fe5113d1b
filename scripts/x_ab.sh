#!/bin/bash
export GHIP_ALLOW_ALT_LIB=1  # the A/B libraries are loaded on purpose (gemma_hip.py refuses GHIP_LIB otherwise)
# exact Q4_0 prefill GEMM tile variants: parity (exact prefill tests) and T = 2048 prefill time per
# build.  usage: bash scripts/x_ab.sh <tag> <variant...>   (variant "new" = the in-tree library,
# others ab_libs/lib<variant>.so from scripts/build_variant.sh)
set -o pipefail
TAG=$1; shift
O=gpurun_out/$TAG
mkdir -p $O
export TMPDIR=/tmp
for v in "$@"; do
  L=""; [ $v != new ] && L=$PWD/ab_libs/lib$v.so
  GHIP_LIB=$L timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_prefill.py -m gpu -k "exact" > $O/t_$v.log 2>&1 || { echo "$v TESTS FAILED"; tail -20 $O/t_$v.log; exit 1; }
  echo "$v $(tail -1 $O/t_$v.log)"
done
for rep in 1 2; do
  for v in "$@"; do
    L=""; [ $v != new ] && L=$PWD/ab_libs/lib$v.so
    GHIP_LIB=$L timeout -k 10 120 python scripts/prof_prefill.py 2048 1 2 > $O/p_$v$rep.txt 2>&1 || { tail -5 $O/p_$v$rep.txt; exit 1; }
    echo "$v $(tail -1 $O/p_$v$rep.txt)"
  done
done
