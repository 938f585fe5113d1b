set -o pipefail
O=gpurun_out/r05g
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_ops.py tests/test_gpu_parity.py -x -q --timeout 300 --timeout-method thread -m gpu > $O/t.log 2>&1; rc=$?; tail -3 $O/t.log; [ $rc = 0 ] || exit 1
for v in "st_new:0" "st_k8:0" "st_k8e:0" "st_new:1"; do
  lib=${v%%:*}; x=${v#*:}
  GHIP_ATT_XCD=$x GHIP_LIB=$PWD/ab_libs/lib$lib.so timeout -k 10 180 python tests/stamp_step.py 9 > $O/st_$lib$x.log 2>&1 || { tail -20 $O/st_$lib$x.log; exit 1; }
  echo "== $lib XCD=$x"; grep -A2 "^attention" $O/st_$lib$x.log
done
OUT=r05g/ab VARS="new=new rw0=rw0 k8=k8 k8e=k8e k8t=k8t k6=k6 newx=new:GHIP_ATT_XCD=1 k8x=k8:GHIP_ATT_XCD=1" REPS=2 bash scripts/var_env_ab.sh
