#!/bin/bash
export GHIP_ALLOW_ALT_LIB=1  # the A/B libraries are loaded on purpose (gemma_hip.py refuses GHIP_LIB otherwise)
# Same-box A/B of exact-prefill builds: ab_libs/lib<v>.so for each v given; per-pass prefill ms.
# usage: bash scripts/ab_prefill.sh v1 v2 ...
set -o pipefail
for r in 1 2; do
  for v in "$@"; do
    echo -n "$v run$r: "
    GHIP_LIB=ab_libs/lib$v.so timeout -k 10 120 python3 scripts/prof_prefill.py 2048 1 2 2>&1 | grep "^rep" | tr '\n' ' ' || exit 1
    echo
  done
done
