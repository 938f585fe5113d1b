#!/bin/bash
# One GPU-box pass, in modes (run from the repo root on the GPU box; every GPU step under its own
# time limit, the script stops at the first failure):
#   bash scripts/gpu_check.sh TAG "MODE ..."
#   tests      pytest -m gpu (thread timeouts, so a hang names its test)
#   bench      python bench.py (the driver's line)
#   prof       the bench under rocprofv3 --kernel-trace --stats (csv kernel stats)
#   profgraph  the fixed-plan decode (scripts/decode_prof.py) as hipGraph replays under rocprofv3
#              --kernel-trace --stats -> decode_kernels_graph.md (per-class table of the benched path)
#   pmcprefill the exact T = 2048 prefill under two SQ --pmc passes -> pmc_prefill_q4_0.json
#   pmc        FETCH_SIZE / WRITE_SIZE passes over scripts/pmc_probe.py (decode matvec traffic)
#   stamp / steps  attention / step phase stamps (needs the stamps build in ab_libs/, which
#              .gpurunignore leaves out by default: remove that line for such a run)
set -o pipefail
TAG=${1:-run}
WHAT=${2:-"tests bench prof"}
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
PLAN=${PLAN:-"9,1,0,9,1,1,1,1,0,9,1,1,1,8,0"}  # the plan the round-5 driver bench tuned to (BENCH_r05)
for w in $WHAT; do
  echo "== $w $(date +%T)"
  case $w in
    tests) timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/pytest_gpu.log 2>&1 || { tail -30 $OUT/pytest_gpu.log; exit 1; } ; tail -2 $OUT/pytest_gpu.log ;;
    smoke) timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || { tail -20 $OUT/smoke.log; exit 1; } ; cat $OUT/smoke.log ;;
    bench) timeout -k 10 500 python bench.py > $OUT/bench.json 2> $OUT/bench.err || { tail -20 $OUT/bench.err; exit 1; } ; cat $OUT/bench.json ;;
    prof) timeout -k 10 500 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof -o run -- python3 bench.py --no-cpu --steps 32 > $OUT/prof.log 2>&1 || { tail -20 $OUT/prof.log; exit 1; } ;
          find $OUT/prof -name "*kernel_stats.csv" | head -1 | xargs -I{} cp {} $OUT/kernel_stats.csv ; head -12 $OUT/kernel_stats.csv | cut -c1-200 ;;
    profgraph) TORCH_FIRST=${TORCH_FIRST:-1} PROF_MAPS=$OUT/maps_profg.txt GHIP_PROF_GRAPH=1 PLAN=$PLAN timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/profg -o run -- python3 scripts/decode_prof.py 48 > $OUT/profg.log 2>&1 || { tail -40 $OUT/profg.log; exit 1; } ;
          python3 scripts/decode_classes.py $(find $OUT/profg -name "run_kernel_trace.csv" | head -1) 128 48 "$PLAN (hipGraph replay)" $OUT/decode_kernels_graph.json > $OUT/decode_kernels_graph.md && cat $OUT/decode_kernels_graph.md ;;
    pmcprefill) bash scripts/pmc_prefill.sh $TAG/pmcp 2048 q4_0 > $OUT/pmcp.log 2>&1 || { tail -20 $OUT/pmcp.log; exit 1; } ; tail -20 $OUT/pmcp.log ;;
    pmc) timeout -k 10 400 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/pmc_fetch_size -o run -- python3 scripts/pmc_probe.py > $OUT/pmc1.log 2>&1 || { tail -20 $OUT/pmc1.log; exit 1; } ;
         timeout -k 10 400 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $OUT/pmc_write_size -o run -- python3 scripts/pmc_probe.py > $OUT/pmc2.log 2>&1 || { tail -20 $OUT/pmc2.log; exit 1; } ;
         ls -R $OUT/pmc_fetch_size | head -20 ;;
    stamp) export GHIP_ALLOW_ALT_LIB=1; GHIP_LIB=ab_libs/libstamps.so timeout -k 10 120 python tests/stamp_attn.py 0 > $OUT/stamp.log 2>&1 && GHIP_LIB=ab_libs/libstamps.so timeout -k 10 120 python tests/stamp_attn.py 1 >> $OUT/stamp.log 2>&1 || { cat $OUT/stamp.log; exit 1; } ; cat $OUT/stamp.log ;;
    steps) export GHIP_ALLOW_ALT_LIB=1; GHIP_LIB=ab_libs/libstamps.so timeout -k 10 180 python tests/stamp_step.py 9 > $OUT/stamp_step.log 2>&1 && GHIP_LIB=ab_libs/libstamps.so timeout -k 10 180 python tests/stamp_step.py 17 >> $OUT/stamp_step.log 2>&1 || { cat $OUT/stamp_step.log; exit 1; } ; cat $OUT/stamp_step.log ;;
    k4probe) timeout -k 10 120 tests/micro/mfma_k4 > $OUT/mfma_k4.log 2>&1 || { tail -20 $OUT/mfma_k4.log; exit 1; } ; cat $OUT/mfma_k4.log ;;
    attostamps) GHIP_ALLOW_ALT_LIB=1 GHIP_LIB=ab_libs/libstamps.so timeout -k 10 180 python scripts/attn_o_stamps.py 9 > $OUT/attn_o_stamps.log 2>&1 || { tail -20 $OUT/attn_o_stamps.log; exit 1; } ; cat $OUT/attn_o_stamps.log ;;
    x4ab) timeout -k 10 300 python scripts/gemm_x4_ab.py 3 2048 ${X4MODES:-0,1,2} > $OUT/gemm_x4_ab.log 2>&1 || { tail -20 $OUT/gemm_x4_ab.log; exit 1; } ; cat $OUT/gemm_x4_ab.log ;;
    attoab) timeout -k 10 300 python scripts/att_o_ab.py 3 64 > $OUT/att_o_ab.log 2>&1 || { tail -20 $OUT/att_o_ab.log; exit 1; } ; cat $OUT/att_o_ab.log ;;
    gputest) timeout -k 10 600 python -u -m pytest $TESTS -m gpu -x -v --timeout 300 --timeout-method thread > $OUT/pytest_sel.log 2>&1 || { tail -40 $OUT/pytest_sel.log; exit 1; } ; tail -15 $OUT/pytest_sel.log ;;
    # the graph-replay trace on /opt/rocm's HIP runtime (no torch): the configuration that crashed in
    # rounds 4-6; its mappings are kept so the frames resolve exactly.  LAST in a call: a crash ends it.
    crashrepro) TORCH_FIRST=0 PROF_MAPS=$OUT/maps_crash.txt GHIP_PROF_GRAPH=1 PLAN=$PLAN timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/profc -o run -- python3 scripts/decode_prof.py 48 > $OUT/profc.log 2>&1; echo "crashrepro rc=$?"; tail -40 $OUT/profc.log; exit 0 ;;
    # summaries of the prof / pmc passes into $OUT/summary, then the raw traces removed (gpurun
    # brings back at most 64 MiB of gpurun_out)
    summarize) python3 scripts/summarize_profiles.py $OUT $OUT/summary > $OUT/summarize.log 2>&1 || { tail -20 $OUT/summarize.log; exit 1; } ;
               rm -rf $OUT/prof $OUT/profg $OUT/profc $OUT/pmc_fetch_size $OUT/pmc_write_size ; ls $OUT/summary ;;
    *) echo "unknown mode $w"; exit 2 ;;
  esac
done
