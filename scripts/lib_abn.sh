#!/bin/bash
export GHIP_ALLOW_ALT_LIB=1  # the A/B libraries are loaded on purpose (gemma_hip.py refuses GHIP_LIB otherwise)
# A/B/... of several builds on one box: LIBS="base nochk new" (ab_libs/lib<name>.so via GHIP_LIB;
# "new" = the in-tree library), decode bench legs, interleaved, REPS rounds; per-class µs printed
set -o pipefail
O=gpurun_out/${OUT:-libabn}
mkdir -p $O
export TMPDIR=/tmp
for rep in $(seq 1 ${REPS:-3}); do
  for v in ${LIBS:-base new}; do
    if [ $v = new ]; then unset GHIP_LIB; else export GHIP_LIB=$PWD/ab_libs/lib$v.so; fi
    timeout -k 10 240 python bench.py --no-cpu --prefill 0 --tp-steps 0 --q8-steps 0 --ggml-steps 0 ${BENCH_ARGS} > $O/$v$rep.json 2> $O/$v$rep.err || { tail -20 $O/$v$rep.err; exit 1; }
    python3 -c "
import json; d=json.load(open('$O/$v$rep.json')); c=d['roofline']['classes']
print('$v', d['value'], (d.get('q4_k_m_decode') or {}).get('tok_s'), ' '.join('%s=%.2f' % (k.split()[0], v['avg_us']) for k, v in c.items()))"
  done
done
