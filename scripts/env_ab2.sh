#!/bin/bash
# decode A/B of environment variants (one build), optional tests first under the variant env
# usage: VARIANTS="a:X=1 b:X=0" [TESTS="..."] [TESTENV="X=1"] bash scripts/env_ab2.sh tag
set -o pipefail
TAG=${1:-envab2}; OUT=gpurun_out/$TAG; mkdir -p $OUT
export TMPDIR=/tmp
if [ -n "$TESTS" ]; then
  env $TESTENV timeout -k 10 500 python -u -m pytest -x -q --timeout 200 --timeout-method thread $TESTS > $OUT/test.log 2>&1 || { tail -30 $OUT/test.log; exit 1; }
  tail -2 $OUT/test.log
fi
for rep in 1 2 3; do
  for v in $VARIANTS; do
    name=${v%%:*}; envs=${v#*:}
    env ${envs//,/ } timeout -k 10 240 python bench.py --no-cpu --prefill 0 --tp-steps 0 --q8-steps 0 --ggml-steps 0 > $OUT/$name$rep.json 2> $OUT/$name$rep.err || { tail -20 $OUT/$name$rep.err; exit 1; }
    python3 -c "import json; d=json.load(open('$OUT/$name$rep.json')); c=d['roofline']['classes']; print('$name', d['value'], d['ms_per_step'], [round(v['avg_us'],2) for v in c.values()])"
  done
done
