#!/bin/bash
# env-variable A/B (default: HIP runtime launch-path settings) on the decode bench (Q4_0 engine + ggml-API leg).
# usage (GPU box, repo root): [VARIANTS="name:VAR=val ..."] [Q8STEPS=n] bash scripts/env_ab.sh [tag]
set -o pipefail
TAG=${1:-envab}; OUT=gpurun_out/$TAG; mkdir -p $OUT
export TMPDIR=/tmp
run() {  # name, env assignments...
  local name=$1; shift
  env "$@" timeout -k 10 240 python bench.py --no-cpu --prefill 0 --tp-steps 0 --q8-steps ${Q8STEPS:-0} --ggml-steps ${GGSTEPS:-48} \
      > $OUT/$name.json 2> $OUT/$name.err || { tail -20 $OUT/$name.err; return 1; }
  python3 -c "import json,sys; d=json.load(open('$OUT/$name.json')); print('$name', d['value'], d['ms_per_step'], d.get('ggml_path_decode_tok_s'), (d.get('q4_k_m_decode') or {}).get('tok_s'))"
}
VARIANTS=${VARIANTS:-"base:A=0 devkarg:HIP_FORCE_DEV_KERNARG=1 nocapt:DEBUG_CLR_GRAPH_PACKET_CAPTURE=0 capt:DEBUG_CLR_GRAPH_PACKET_CAPTURE=1"}
for rep in 1 2; do
  for v in $VARIANTS; do run ${v%%:*}$rep ${v#*:} || exit 1; done
done
