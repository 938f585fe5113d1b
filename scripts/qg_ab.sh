#!/bin/bash
# prefill GELU quantizer with the table in LDS (default) vs the per-row form (GHIP_QR_GELU_LDS=0): parity, then T = 2048 time
set -o pipefail
O=gpurun_out/${1:-qg}
mkdir -p $O
export TMPDIR=/tmp
GHIP_QR_GELU_LDS=1 timeout -k 10 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_prefill.py tests/test_gpu_parity.py tests/test_gpu_ggml_graph.py -m gpu -k "prefill or exact" > $O/t.log 2>&1 || { tail -20 $O/t.log; exit 1; }
tail -1 $O/t.log
for rep in 1 2; do for v in 1 0; do
  GHIP_QR_GELU_LDS=$v timeout -k 10 120 python scripts/prof_prefill.py 2048 1 2 > $O/p_$v$rep.txt 2>&1 || { tail -5 $O/p_$v$rep.txt; exit 1; }
  echo "LDS=$v $(tail -1 $O/p_$v$rep.txt)"
done; done
