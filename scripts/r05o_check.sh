set -o pipefail
O=gpurun_out/r05o
mkdir -p $O
export TMPDIR=/tmp
KQ=1 GHIP_LIB=$PWD/ab_libs/libst1e2.so timeout -k 10 180 python tests/stamp_step.py 9 > $O/st_kq.log 2>&1 || { tail -20 $O/st_kq.log; exit 1; }
grep -A2 "^gate/up" $O/st_kq.log
OUT=r05o/kq VARS="new=new e0=e0 e2=e2" REPS=3 bash scripts/kqm_ab.sh
