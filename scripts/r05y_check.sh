set -o pipefail
O=gpurun_out/r05y
mkdir -p $O
export TMPDIR=/tmp
GHIP_LIB=$PWD/ab_libs/libxfirst.so timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 300 --timeout-method thread -m gpu > $O/t.log 2>&1; rc=$?; tail -2 $O/t.log; [ $rc = 0 ] || exit 1
OUT=r05y/q4 LIBS="new xfirst" REPS=4 bash scripts/lib_abn.sh
