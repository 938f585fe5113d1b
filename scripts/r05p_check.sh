set -o pipefail
O=gpurun_out/r05p
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest tests/test_gpu_kquants.py tests/test_gpu_norm_exact.py tests/test_gpu_engine_gguf.py -x -q --timeout 300 --timeout-method thread -m gpu > $O/t.log 2>&1; rc=$?; tail -3 $O/t.log; [ $rc = 0 ] || exit 1
KQ=1 GHIP_LIB=$PWD/ab_libs/libst1.so timeout -k 10 180 python tests/stamp_step.py 9 > $O/st_kq.log 2>&1 || { tail -20 $O/st_kq.log; exit 1; }
grep -A2 "^gate/up" $O/st_kq.log
OUT=r05p/kq VARS="base=base new=new nopipe=new:GHIP_KQ_PIPE=0 e2=e2" REPS=3 bash scripts/kqm_ab.sh
