set -o pipefail
O=gpurun_out/r05v
mkdir -p $O
export TMPDIR=/tmp
GHIP_KQ_PIPE=2 timeout -k 10 500 python -u -m pytest tests/test_gpu_kquants.py tests/test_gpu_engine_gguf.py -x -q --timeout 300 --timeout-method thread -m gpu > $O/t.log 2>&1; rc=$?; tail -2 $O/t.log; [ $rc = 0 ] || exit 1
OUT=r05v/kq VARS="new=new pipeo=new:GHIP_KQ_PIPE=2 ogrid=new:GHIP_KQ_OGRID=1" REPS=3 bash scripts/kqm_ab.sh
