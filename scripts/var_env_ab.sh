#!/bin/bash
export GHIP_ALLOW_ALT_LIB=1  # the A/B libraries are loaded on purpose (gemma_hip.py refuses GHIP_LIB otherwise)
# Interleaved decode-bench A/B over (library, env) variants: VARS="name=lib[:ENV=V,ENV2=V2] ..."
# (lib "new" = the in-tree build, else ab_libs/lib<lib>.so); REPS rounds; per-class µs printed
set -o pipefail
O=gpurun_out/${OUT:-varab}
mkdir -p $O
export TMPDIR=/tmp
for rep in $(seq 1 ${REPS:-2}); do
  for spec in $VARS; do
    name=${spec%%=*}; rest=${spec#*=}; lib=${rest%%:*}; envs=""; [[ $rest == *:* ]] && envs=${rest#*:}
    if [ $lib = new ]; then L=""; else L=$PWD/ab_libs/lib$lib.so; fi
    env GHIP_LIB=$L ${envs//,/ } timeout -k 10 240 python bench.py --no-cpu --prefill 0 --tp-steps 0 --q8-steps 0 --ggml-steps 0 ${BENCH_ARGS} > $O/$name$rep.json 2> $O/$name$rep.err || { tail -20 $O/$name$rep.err; exit 1; }
    python3 -c "
import json; d=json.load(open('$O/$name$rep.json')); c=d['roofline']['classes']
print('$name', d['value'], (d.get('q4_k_m_decode') or {}).get('tok_s'), ' '.join('%s=%.2f' % (k.split()[0], v['avg_us']) for k, v in c.items()))"
  done
done
