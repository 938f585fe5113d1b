#!/bin/bash
# scale-run loads A/B (GHIP_SCL: gate/up, GHIP_RR_SCL: round-pipelined down) after the decode parity tests
set -o pipefail
mkdir -p gpurun_out/scl
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_parity.py -k "gemma2b or tiny or gate_up or tuned" > gpurun_out/scl/test.log 2>&1 || { tail -30 gpurun_out/scl/test.log; exit 1; }
tail -2 gpurun_out/scl/test.log
VARIANTS=${VARIANTS:-"s1:GHIP_SCL=1 s2:GHIP_SCL=2"} GGSTEPS=0 Q8STEPS=0 bash scripts/env_ab.sh scl
for v in 1 2; do GHIP_SCL=$v timeout -k 10 200 python -u scripts/hot_cold.py 2>&1 | tail -2; done
