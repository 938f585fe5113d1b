#!/bin/bash
export GHIP_ALLOW_ALT_LIB=1  # the A/B libraries are loaded on purpose (gemma_hip.py refuses GHIP_LIB otherwise)
# decode step time per build (bench decode leg only), 2 interleaved reps: attention variants differ
# by 18 x their attention time.  usage: bash scripts/attn_ab.sh <tag> <variant...>
# ("new" = in-tree, else ab_libs/lib<v>.so)
set -o pipefail
TAG=$1; shift
O=gpurun_out/$TAG
mkdir -p $O
export TMPDIR=/tmp
for rep in 1 2; do
  for v in "$@"; do
    L=""; [ $v != new ] && L=$PWD/ab_libs/lib$v.so
    GHIP_LIB=$L timeout -k 10 240 python bench.py --no-cpu --prefill 0 --tp-steps 0 --q8-steps 0 --ggml-steps 0 > $O/b_$v$rep.json 2> $O/b_$v$rep.err || { tail -20 $O/b_$v$rep.err; exit 1; }
    python3 -c "import json; d=json.load(open('$O/b_$v$rep.json')); print('$v', d['value'], d['ms_per_step'])"
  done
done
