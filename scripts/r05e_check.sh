set -o pipefail
O=gpurun_out/r05e
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 60 tests/micro/valu_rates > $O/valu.txt 2>&1 || { cat $O/valu.txt; exit 1; }
grep -E "fma_mix|cvt_f32_f16|dot2|fma_f32 " $O/valu.txt
timeout -k 10 600 python -u -m pytest tests/test_gpu_norm_exact.py tests/test_gpu_parity.py tests/test_gpu_ops.py -x -q --timeout 300 --timeout-method thread -m gpu > $O/t.log 2>&1; rc=$?; tail -3 $O/t.log; [ $rc = 0 ] || exit 1
GHIP_LIB=$PWD/ab_libs/libstamps4.so timeout -k 10 180 python tests/stamp_step.py 9 > $O/stamp4.log 2>&1 || { tail -20 $O/stamp4.log; exit 1; }
grep -A2 "^attention" $O/stamp4.log
OUT=r05e/ab LIBS="base nochk trim0 new" REPS=3 bash scripts/lib_abn.sh
