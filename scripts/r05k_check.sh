set -o pipefail
O=gpurun_out/r05k
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest tests/test_gpu_norm_exact.py tests/test_gpu_kquants.py -x -q --timeout 300 --timeout-method thread -m gpu > $O/t.log 2>&1; rc=$?; tail -3 $O/t.log; [ $rc = 0 ] || exit 1
OUT=r05k/kq VARS="base=base new=new nochk=nochk" REPS=3 bash scripts/kqm_ab.sh || exit 1
OUT=r05k/q4 LIBS="base nochk new" REPS=3 bash scripts/lib_abn.sh
