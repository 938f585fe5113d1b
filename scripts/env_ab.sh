#!/bin/bash
# A/B of an environment switch on one box, interleaved: ENVA / ENVB (e.g. "GHIP_RR_EW=0" / "GHIP_RR_EW=1"),
# decode bench legs (no CPU, prefill, TP, Q8_0, ggml legs unless BENCH_ARGS adds them), REPS rounds
set -o pipefail
O=gpurun_out/${OUT:-envab}
mkdir -p $O
for rep in $(seq 1 ${REPS:-3}); do
  for v in A B; do
    if [ $v = A ]; then E="$ENVA"; else E="$ENVB"; fi
    env $E timeout -k 10 240 python bench.py --no-cpu --prefill 0 --tp-steps 0 --q8-steps 0 --ggml-steps 0 ${BENCH_ARGS} > $O/$v$rep.json 2> $O/$v$rep.err || { tail -20 $O/$v$rep.err; exit 1; }
    python3 -c "
import json; d=json.load(open('$O/$v$rep.json')); c=d['roofline']['classes']
print('$v [$E]', d['value'], d['ms_per_step'], (d.get('q4_k_m_decode') or {}).get('tok_s'), ' '.join('%s=%.2f' % (k.split()[0], v['avg_us']) for k, v in c.items()))"
  done
done
