set -o pipefail
O=gpurun_out/r05f
mkdir -p $O
export TMPDIR=/tmp
for v in "stamps4:0" "stamps4k8:0" "stamps4k8:1"; do
  lib=${v%%:*}; vd=${v#*:}
  GHIP_ATT_VDMA=$vd GHIP_LIB=$PWD/ab_libs/lib$lib.so timeout -k 10 180 python tests/stamp_step.py 9 > $O/st_$lib$vd.log 2>&1 || { tail -20 $O/st_$lib$vd.log; exit 1; }
  echo "== $lib VDMA=$vd"; grep -A2 "^attention" $O/st_$lib$vd.log
done
OUT=r05f/ab VARS="new=new k8v0=k8v0 k8v0d=k8v0:GHIP_ATT_VDMA=1 newd=new:GHIP_ATT_VDMA=1 k6v2=k6v2" REPS=3 bash scripts/var_env_ab.sh
