#!/bin/bash
export GHIP_ALLOW_ALT_LIB=1  # the A/B libraries are loaded on purpose (gemma_hip.py refuses GHIP_LIB otherwise)
# Q4_K_M decode A/B over (library, env) variants, interleaved (scripts/run_kqm.py at the bench's
# positions): VARS="name=lib[:ENV=V,ENV2=V2] ..." (lib "new" = in-tree), REPS rounds
set -o pipefail
O=gpurun_out/${OUT:-kqmab}
mkdir -p $O
export TMPDIR=/tmp
for rep in $(seq 1 ${REPS:-2}); do
  for spec in $VARS; do
    name=${spec%%=*}; rest=${spec#*=}; lib=${rest%%:*}; envs=""; [[ $rest == *:* ]] && envs=${rest#*:}
    if [ $lib = new ]; then L=""; else L=$PWD/ab_libs/lib$lib.so; fi
    r=$(env GHIP_LIB=$L ${envs//,/ } timeout -k 10 180 python scripts/run_kqm.py 96 128 2> $O/$name$rep.err) || { tail -20 $O/$name$rep.err; exit 1; }
    echo "$name $r"
  done
done
