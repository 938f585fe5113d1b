set -o pipefail
O=gpurun_out/r05ab
mkdir -p $O
export TMPDIR=/tmp
OUT=r05ab/q4 LIBS="new up2 up8" REPS=3 bash scripts/lib_abn.sh
