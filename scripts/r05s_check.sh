set -o pipefail
O=gpurun_out/r05s
mkdir -p $O
export TMPDIR=/tmp
OUT=r05s/q4 LIBS="base r5k new" REPS=4 bash scripts/lib_abn.sh
