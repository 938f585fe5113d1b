#!/bin/bash
# HIP runtime launch-path settings A/B on the decode bench (Q4_0 engine + ggml-API leg).
# usage (GPU box, repo root): bash scripts/env_ab.sh [tag]
set -o pipefail
TAG=${1:-envab}; OUT=gpurun_out/$TAG; mkdir -p $OUT
export TMPDIR=/tmp
run() {  # name, env assignments...
  local name=$1; shift
  env "$@" timeout -k 10 240 python bench.py --no-cpu --prefill 0 --tp-steps 0 --q8-steps 0 --ggml-steps 48 \
      > $OUT/$name.json 2> $OUT/$name.err || { tail -20 $OUT/$name.err; return 1; }
  python3 -c "import json,sys; d=json.load(open('$OUT/$name.json')); print('$name', d['value'], d['ms_per_step'], d.get('ggml_path_decode_tok_s'), (d.get('q4_k_m_decode') or {}).get('tok_s'))"
}
for rep in 1 2; do
  run base$rep A=0 || exit 1
  run devkarg$rep HIP_FORCE_DEV_KERNARG=1 || exit 1
  run nocapt$rep DEBUG_CLR_GRAPH_PACKET_CAPTURE=0 || exit 1
  run capt$rep DEBUG_CLR_GRAPH_PACKET_CAPTURE=1 || exit 1
done
