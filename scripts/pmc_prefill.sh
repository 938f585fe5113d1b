#!/bin/bash
# SQ counters of one exact Gemma-2B prefill pass (T=2048), two separate --pmc passes.
# usage: bash scripts/pmc_prefill.sh <tag> [T]
set -o pipefail
TAG=$1; T=${2:-2048}
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
timeout -s KILL 60 rocprofv3 -L > $OUT/counters.txt 2>&1 || true
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS --output-format csv -d $OUT/pmc1 -o run -- python3 scripts/prof_prefill.py $T 1 0 > $OUT/pmc1.log 2>&1 || { tail -5 $OUT/pmc1.log; exit 1; }
timeout -s KILL 120 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_INST_LDS GRBM_GUI_ACTIVE --output-format csv -d $OUT/pmc2 -o run -- python3 scripts/prof_prefill.py $T 1 0 > $OUT/pmc2.log 2>&1 || { tail -5 $OUT/pmc2.log; exit 1; }
python3 scripts/pmc_table.py $OUT k_gemm_x
