#!/bin/bash
# K-quant prefill GEMM check on the GPU box: parity tests, T=2048 prefill timing, kernel profile
set -o pipefail
OUT=${GRAFT_REPO_ROOT:-$(pwd)}/gpurun_out
TAG=${1:-kq}
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu tests/test_gpu_kquants.py tests/test_gpu_engine_gguf.py > $OUT/${TAG}_tests.log 2>&1 || { tail -30 $OUT/${TAG}_tests.log; exit 1; }
tail -1 $OUT/${TAG}_tests.log
timeout -k 10 120 python -u scripts/kq_prefill.py 2048 3 > $OUT/${TAG}_prefill.log 2>&1 || { cat $OUT/${TAG}_prefill.log; exit 1; }
cat $OUT/${TAG}_prefill.log
cd /tmp && export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $OUT/${TAG}prof -o kq -- python3 $GRAFT_REPO_ROOT/scripts/kq_prefill.py 2048 1 > $OUT/${TAG}_prof.log 2>&1 || { tail -20 $OUT/${TAG}_prof.log; exit 1; }
