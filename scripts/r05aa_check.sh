set -o pipefail
O=gpurun_out/r05aa
mkdir -p $O
export TMPDIR=/tmp
GHIP_LIB=$PWD/ab_libs/libksx.so timeout -k 10 400 python -u -m pytest tests/test_gpu_kquants.py tests/test_gpu_engine_gguf.py tests/test_gpu_norm_exact.py -x -q --timeout 300 --timeout-method thread -m gpu > $O/t.log 2>&1; rc=$?; tail -2 $O/t.log; [ $rc = 0 ] || exit 1
OUT=r05aa/kq VARS="new=new ksx=ksx" REPS=4 bash scripts/kqm_ab.sh
