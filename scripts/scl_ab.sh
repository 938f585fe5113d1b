set -o pipefail
mkdir -p gpurun_out/scl
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_parity.py -k "gemma2b or tiny or gate_up or tuned" > gpurun_out/scl/test.log 2>&1 || { tail -30 gpurun_out/scl/test.log; exit 1; }
tail -3 gpurun_out/scl/test.log
VARIANTS="off:GHIP_SCL=0 on:GHIP_SCL=1" GGSTEPS=0 Q8STEPS=32 bash scripts/env_ab.sh scl
for v in 0 1; do GHIP_SCL=$v timeout -k 10 200 python -u scripts/hot_cold.py 2>&1 | tail -2; done
