set -o pipefail
O=gpurun_out/r05u
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_norm_exact.py tests/test_gpu_prefill.py -x -q --timeout 300 --timeout-method thread -m gpu > $O/t.log 2>&1; rc=$?; tail -2 $O/t.log; [ $rc = 0 ] || exit 1
OUT=r05u/q4 LIBS="base shfl new" REPS=4 bash scripts/lib_abn.sh
