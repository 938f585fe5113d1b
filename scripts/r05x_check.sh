set -o pipefail
O=gpurun_out/r05x
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests/ -x -q --timeout 400 --timeout-method thread -m gpu > $O/t.log 2>&1; rc=$?; tail -3 $O/t.log; [ $rc = 0 ] || exit 1
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1; rc=$?; tail -3 $O/smoke.log; [ $rc = 0 ] || exit 1
OUT=r05x/kq VARS="new=new pipe3=new:GHIP_KQ_PIPE=3" REPS=3 bash scripts/kqm_ab.sh
OUT=r05x/ds VARS="ds4=new ds2=new:GHIP_ATT_DSPLIT=2 ds8=new:GHIP_ATT_DSPLIT=8" REPS=2 bash scripts/var_env_ab.sh
