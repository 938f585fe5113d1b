#!/bin/bash
# decode step time A/B of one environment switch (interleaved, 3 reps): bash scripts/env_ab3.sh <tag> VAR=val [VAR=val2 ...]
set -o pipefail
TAG=$1; shift
O=gpurun_out/$TAG
mkdir -p $O
export TMPDIR=/tmp
for rep in 1 2 3; do
  for kv in "base" "$@"; do
    if [ "$kv" = base ]; then E=""; else E="$kv"; fi
    env $E timeout -k 10 240 python bench.py --no-cpu --prefill 0 --tp-steps 0 --q8-steps 0 --ggml-steps 0 > $O/b_$rep.json 2> $O/b_$rep.err || { tail -20 $O/b_$rep.err; exit 1; }
    python3 -c "import json; d=json.load(open('$O/b_$rep.json')); r=d['roofline']['classes']; print('$kv', d['value'], d['ms_per_step'], 'qkv', r['qkv matvec (+norm)']['avg_us'], 'o', r['attn-out matvec (+resid)']['avg_us'])"
  done
done
