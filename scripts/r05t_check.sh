set -o pipefail
O=gpurun_out/r05t
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_ops.py -x -q --timeout 300 --timeout-method thread -m gpu -k "attn or attention" > $O/t.log 2>&1; rc=$?; tail -2 $O/t.log; [ $rc = 0 ] || exit 1
OUT=r05t/q4 LIBS="base r5k new" REPS=4 bash scripts/lib_abn.sh
