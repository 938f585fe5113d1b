#!/bin/bash
# Infinity-Cache warm-up in the attention launch (GHIP_AWARM) A/B + hot/cold kernel times.
# usage (GPU box, repo root): bash scripts/awarm_ab.sh [tag]
set -o pipefail
TAG=${1:-awarm}; OUT=gpurun_out/$TAG; mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 300 python -u scripts/hot_cold.py > $OUT/hot_cold.txt 2>&1 || exit 1
cat $OUT/hot_cold.txt
VARIANTS=${VARIANTS:-"off:GHIP_AWARM=0 gu:GHIP_AWARM=3 gud:GHIP_AWARM=15 guq:GHIP_AWARM=1"} GGSTEPS=0 bash scripts/env_ab.sh $TAG
