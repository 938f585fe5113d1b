#!/bin/bash
export GHIP_ALLOW_ALT_LIB=1  # the A/B libraries are loaded on purpose (gemma_hip.py refuses GHIP_LIB otherwise)
# Q4_K_M decode: in-tree build vs ab_libs/lib<v>.so variants, interleaved (usage: bash scripts/kq_var_ab.sh v1 v2 ...)
set -o pipefail
export TMPDIR=/tmp
for rep in 1 2; do
  echo -n "base "; timeout -k 10 120 python -u scripts/run_kqm.py 64 2>&1 | tail -1 || exit 1
  for v in "$@"; do echo -n "$v "; GHIP_LIB=$PWD/ab_libs/lib$v.so timeout -k 10 120 python -u scripts/run_kqm.py 64 2>&1 | tail -1 || exit 1; done
done
