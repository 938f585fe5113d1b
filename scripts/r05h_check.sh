set -o pipefail
O=gpurun_out/r05h
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest tests/test_gpu_kquants.py tests/test_gpu_norm_exact.py tests/test_gpu_engine_gguf.py -x -q --timeout 300 --timeout-method thread -m gpu > $O/t.log 2>&1; rc=$?; tail -3 $O/t.log; [ $rc = 0 ] || exit 1
GHIP_KQ_GU2=1 timeout -k 10 500 python -u -m pytest tests/test_gpu_kquants.py tests/test_gpu_engine_gguf.py -x -q --timeout 300 --timeout-method thread -m gpu -k "kq or k_quant or kquant or q4_k or Q4_K" > $O/t2.log 2>&1; rc=$?; tail -3 $O/t2.log; [ $rc = 0 ] || exit 1
OUT=r05h/kq VARS="base=base new=new gu2=new:GHIP_KQ_GU2=1" REPS=3 bash scripts/kqm_ab.sh
