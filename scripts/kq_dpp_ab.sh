#!/bin/bash
export GHIP_ALLOW_ALT_LIB=1  # the A/B libraries are loaded on purpose (gemma_hip.py refuses GHIP_LIB otherwise)
# Q8_K quantizer with DPP reductions (ab_libs/libdpp.so) vs the in-tree build: K-quant parity tests
# under the variant, then Q4_K_M decode interleaved
set -o pipefail
mkdir -p gpurun_out/dpp
export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_engine_gguf.py tests/test_gpu_kquants.py tests/test_gpu_ggml_kquant_ops.py tests/test_gpu_ops.py > gpurun_out/dpp/test.log 2>&1 || { tail -30 gpurun_out/dpp/test.log; exit 1; }
tail -1 gpurun_out/dpp/test.log
for rep in 1 2 3; do
  echo -n "base "; GHIP_LIB=$PWD/ab_libs/libbase.so timeout -k 10 120 python -u scripts/run_kqm.py 64 2>&1 | tail -1 || exit 1
  echo -n "new  "; timeout -k 10 120 python -u scripts/run_kqm.py 64 2>&1 | tail -1 || exit 1
done
