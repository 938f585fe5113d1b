# round-5 final artifacts: full GPU suite, the driver-style bench line, rocprofv3 kernel stats of the
# bench (trace pass), FETCH_SIZE / WRITE_SIZE passes (separate runs), the fixed-plan decode profile;
# summaries kept, raw traces deleted on the box (gpurun copies back <= 64 MiB)
set -o pipefail
T=r05final
O=gpurun_out/$T
mkdir -p $O
export TMPDIR=/tmp
bash scripts/gpu_check.sh $T tests || exit 1
cp $O/pytest_gpu.log $O/gpu_tests.txt
bash scripts/gpu_check.sh $T bench > /dev/null || exit 1
python3 -c "
import json; d=json.load(open('$O/bench.json'))
print('decode', d['value'], 'kqm', d['q4_k_m_decode']['tok_s'], 'q8', d['q8_0_decode']['tok_s'], 'prefill', d['prefill'].get('ms'), 'cpu', d['cpu_baseline'].get('value'))"
bash scripts/gpu_check.sh $T prof > /dev/null || exit 1
bash scripts/gpu_check.sh $T pmc > /dev/null || exit 1
python3 scripts/summarize_profiles.py $O r05 > $O/summarize.log 2>&1 || { tail -20 $O/summarize.log; exit 1; }
mkdir -p $O/profiles_r05 && cp profiles/r05/* $O/profiles_r05/ && cp profiles/pmc_traffic.json $O/pmc_traffic_top.json
find $O -name "*kernel_trace.csv" -delete
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/dprof -o run -- python3 scripts/decode_prof.py 48 > $O/dprof.log 2>&1 || { tail -20 $O/dprof.log; exit 1; }
python3 scripts/decode_classes.py $O/dprof/run_results.db 128 48 "9,1,0,9,1,0,1,1,0,9,1,1,1,8,0" > $O/decode_kernels.md
python3 scripts/prof_db_summary.py $O/dprof/run_results.db 48 > $O/decode_kernel_stats.txt
rm -rf $O/dprof
du -sh $O; ls $O $O/profiles_r05
