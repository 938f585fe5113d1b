#!/bin/bash
export GHIP_ALLOW_ALT_LIB=1  # the A/B libraries are loaded on purpose (gemma_hip.py refuses GHIP_LIB otherwise)
# T=2048 K-quant prefill with each variant library given (ab_libs/lib<name>.so); "base" = the product build
for n in "$@"; do
  if [ "$n" = base ]; then L=""; else L=ab_libs/lib$n.so; fi
  echo "== $n"; GHIP_LIB=$L timeout -k 10 120 python -u scripts/kq_prefill.py 2048 2 2>&1 | tail -1 || exit 1
done
