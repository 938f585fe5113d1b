set -o pipefail
mkdir -p gpurun_out/r05c
export TMPDIR=/tmp
timeout -k 10 700 python -u -m pytest tests/ -x -q --timeout 400 --timeout-method thread -m gpu > gpurun_out/r05c/t.log 2>&1; echo rc=$? >> gpurun_out/r05c/t.log
tail -2 gpurun_out/r05c/t.log
OUT=r05c/ew ENVA="GHIP_RR_EW=0" ENVB="GHIP_RR_EW=1" bash scripts/env_ab.sh || exit 1
bash scripts/lib_ab.sh > gpurun_out/r05c/ab.txt 2>&1 || exit 1
cat gpurun_out/r05c/ab.txt
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r05c/prof -o run -- python3 scripts/decode_prof.py 48 > gpurun_out/r05c/prof.log 2>&1 || { tail -20 gpurun_out/r05c/prof.log; exit 1; }
python3 scripts/decode_classes.py $(find gpurun_out/r05c/prof -name "run_kernel_trace.csv" | head -1) 128 48 "9,1,0,9,1,0,1,1,0,9,1,1,1,8,0" > gpurun_out/r05c/decode_kernels.md
cat gpurun_out/r05c/decode_kernels.md
# graph-replay trace of the same decode (gaps between the hipGraph's launches); last, since a
# kernel trace of graph replays crashed the profiler once
GHIP_PROF_GRAPH=1 timeout -k 10 300 rocprofv3 --kernel-trace -d gpurun_out/r05c/profg -o run -- python3 scripts/decode_prof.py 48 > gpurun_out/r05c/profg.log 2>&1 || { tail -20 gpurun_out/r05c/profg.log; exit 1; }
python3 scripts/decode_classes.py $(find gpurun_out/r05c/profg -name "run_kernel_trace.csv" | head -1) 128 48 "9,1,0,9,1,0,1,1,0,9,1,1,1,8,0 (hipGraph replay)" > gpurun_out/r05c/decode_kernels_graph.md
cat gpurun_out/r05c/decode_kernels_graph.md
