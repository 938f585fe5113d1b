set -o pipefail
mkdir -p gpurun_out/r05c
export TMPDIR=/tmp
timeout -k 10 700 python -u -m pytest tests/ -x -q --timeout 400 --timeout-method thread -m gpu > gpurun_out/r05c/t.log 2>&1; echo rc=$? >> gpurun_out/r05c/t.log
tail -2 gpurun_out/r05c/t.log
bash scripts/lib_ab.sh > gpurun_out/r05c/ab.txt 2>&1 || exit 1
cat gpurun_out/r05c/ab.txt
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r05c/prof -o run -- python3 scripts/decode_prof.py 48 > gpurun_out/r05c/prof.log 2>&1 || { tail -20 gpurun_out/r05c/prof.log; exit 1; }
python3 scripts/decode_classes.py $(find gpurun_out/r05c/prof -name "run_kernel_trace.csv" | head -1) 128 48 "9,1,0,9,1,0,1,1,0,9,1,1,1,8,0" > gpurun_out/r05c/decode_kernels.md
cat gpurun_out/r05c/decode_kernels.md
