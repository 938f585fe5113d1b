#!/bin/bash
# One GPU-box pass: parity tests, attention phase stamps, bench line, rocprofv3 kernel stats.
# usage (from the repo root, on the GPU box): bash scripts/gpu_check.sh [tag] [what]
# (stamp / steps need the stamps build first, here: bash scripts/build_variant.sh stamps \
#  matvec_ks1.hip,matvec_ks2.hip,matvec_ks4.hip,matvec_ks8.hip,ops.hip,engine.cpp -DGHIP_STAMPS=1)
#   what: any of "tests stamp bench prof" (default: all)
set -o pipefail
TAG=${1:-run}
WHAT=${2:-"tests stamp bench prof"}
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
for w in $WHAT; do
  case $w in
    tests) timeout -k 10 600 python -m pytest tests -m gpu -x -q > $OUT/pytest_gpu.log 2>&1 || { tail -30 $OUT/pytest_gpu.log; exit 1; } ; tail -2 $OUT/pytest_gpu.log ;;
    stamp) GHIP_LIB=ab_libs/libstamps.so timeout -k 10 120 python tests/stamp_attn.py 0 > $OUT/stamp.log 2>&1 && GHIP_LIB=ab_libs/libstamps.so timeout -k 10 120 python tests/stamp_attn.py 1 >> $OUT/stamp.log 2>&1 || { cat $OUT/stamp.log; exit 1; } ; cat $OUT/stamp.log ;;
    steps) GHIP_LIB=ab_libs/libstamps.so timeout -k 10 180 python tests/stamp_step.py 9 > $OUT/stamp_step.log 2>&1 && GHIP_LIB=ab_libs/libstamps.so timeout -k 10 180 python tests/stamp_step.py 17 >> $OUT/stamp_step.log 2>&1 || { cat $OUT/stamp_step.log; exit 1; } ; cat $OUT/stamp_step.log ;;
    bench) timeout -k 10 400 python bench.py > $OUT/bench.json 2> $OUT/bench.err || { tail -20 $OUT/bench.err; exit 1; } ; cat $OUT/bench.json ;;
    prof) timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof -o run -- python3 bench.py --no-cpu --steps 32 > $OUT/prof.log 2>&1 || { tail -20 $OUT/prof.log; exit 1; } ;
          find $OUT/prof -name "*kernel_stats.csv" | head -1 | xargs -I{} cp {} $OUT/kernel_stats.csv ; head -12 $OUT/kernel_stats.csv | cut -c1-200 ;;
    pmc) timeout -k 10 400 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/pmc_fetch_size -o run -- python3 scripts/pmc_probe.py > $OUT/pmc1.log 2>&1 || { tail -20 $OUT/pmc1.log; exit 1; } ;
         timeout -k 10 400 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $OUT/pmc_write_size -o run -- python3 scripts/pmc_probe.py > $OUT/pmc2.log 2>&1 || { tail -20 $OUT/pmc2.log; exit 1; } ;
         ls -R $OUT/pmc_fetch_size | head -20 ;;
  esac
done
