#!/bin/bash
# Q6_K output head: weight super-blocks in flight per round trip (GHIP_KQ_OPF 2 vs 4), Q4_K_M decode
set -o pipefail
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_kquants.py tests/test_gpu_engine_gguf.py -m gpu > gpurun_out/kqopf_t.log 2>&1 || { tail -20 gpurun_out/kqopf_t.log; exit 1; }
GHIP_KQ_OPF=4 timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_kquants.py tests/test_gpu_engine_gguf.py -m gpu > gpurun_out/kqopf_t4.log 2>&1 || { tail -20 gpurun_out/kqopf_t4.log; exit 1; }
tail -1 gpurun_out/kqopf_t.log; tail -1 gpurun_out/kqopf_t4.log
for rep in 1 2 3; do for v in 2 4; do
  echo "OPF=$v $(GHIP_KQ_OPF=$v timeout -k 10 120 python scripts/run_kqm.py 48 128)" || exit 1
done; done
