set -o pipefail
O=gpurun_out/r05n
mkdir -p $O
export TMPDIR=/tmp
KQ=1 GHIP_LIB=$PWD/ab_libs/libst1.so timeout -k 10 180 python tests/stamp_step.py 9 > $O/st_kq.log 2>&1 || { tail -20 $O/st_kq.log; exit 1; }
cat $O/st_kq.log
GHIP_LIB=$PWD/ab_libs/libst1.so timeout -k 10 180 python tests/stamp_step.py 9 > $O/st_q4.log 2>&1 || { tail -20 $O/st_q4.log; exit 1; }
cat $O/st_q4.log
