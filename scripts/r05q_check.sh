set -o pipefail
O=gpurun_out/r05q
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_kquants.py tests/test_gpu_norm_exact.py tests/test_gpu_engine_gguf.py tests/test_gpu_ggml_kquant_ops.py -x -q --timeout 300 --timeout-method thread -m gpu > $O/t.log 2>&1; rc=$?; tail -3 $O/t.log; [ $rc = 0 ] || exit 1
KQ=1 GHIP_LIB=$PWD/ab_libs/libst1.so timeout -k 10 180 python tests/stamp_step.py 9 > $O/st_kq.log 2>&1 || { tail -20 $O/st_kq.log; exit 1; }
grep -A2 "^gate/up" $O/st_kq.log
OUT=r05q/kq VARS="base=base kqold=kqold new=new" REPS=3 bash scripts/kqm_ab.sh
