set -o pipefail
O=gpurun_out/r05r
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests/ -x -q --timeout 400 --timeout-method thread -m gpu > $O/t.log 2>&1; rc=$?; tail -3 $O/t.log; [ $rc = 0 ] || exit 1
OUT=r05r/kq VARS="base=base prev=prev new=new" REPS=3 bash scripts/kqm_ab.sh || exit 1
OUT=r05r/q4 LIBS="base prev new" REPS=2 bash scripts/lib_abn.sh
