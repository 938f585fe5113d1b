#!/bin/bash
# ggml-API path: graph tests, then the reference-loop bench with the per-step breakdown, A/B of the
# logits copy form (GHIP_EXT_DIRECT)
set -o pipefail
mkdir -p gpurun_out/gab
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_ggml_graph.py > gpurun_out/gab/test.log 2>&1 || { tail -30 gpurun_out/gab/test.log; exit 1; }
tail -2 gpurun_out/gab/test.log
for d in 0 1 0 1; do
  GHIP_EXT_DIRECT=$d GHIP_GGML_FAST_PROF=1 DRIVER_PROF=1 timeout -k 10 300 python -u scripts/ggml_path_bench.py 48 gpurun_out/gab/d$d > gpurun_out/gab/d$d.log 2>&1 || { tail -20 gpurun_out/gab/d$d.log; exit 1; }
  echo "direct=$d: $(tail -1 gpurun_out/gab/d$d.log)"
  grep "step 4[0-7]:\|ext_decode" gpurun_out/gab/d$d/driver.err | tail -4
done
