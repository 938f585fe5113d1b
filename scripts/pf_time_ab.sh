#!/bin/bash
export GHIP_ALLOW_ALT_LIB=1  # the A/B libraries are loaded on purpose (gemma_hip.py refuses GHIP_LIB otherwise)
# T = 2048 exact prefill time per build (timing only, no parity: for ablation builds).
# usage: bash scripts/pf_time_ab.sh <tag> <variant...>   ("new" = in-tree, else ab_libs/lib<v>.so)
set -o pipefail
TAG=$1; shift
O=gpurun_out/$TAG
mkdir -p $O
export TMPDIR=/tmp
for rep in 1 2; do
  for v in "$@"; do
    L=""; [ $v != new ] && L=$PWD/ab_libs/lib$v.so
    GHIP_LIB=$L timeout -k 10 120 python scripts/prof_prefill.py 2048 1 2 > $O/p_$v$rep.txt 2>&1 || { tail -5 $O/p_$v$rep.txt; exit 1; }
    echo "$v $(tail -1 $O/p_$v$rep.txt)"
  done
done
