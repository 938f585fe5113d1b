#!/bin/bash
# SQ counters of one exact Gemma-2B prefill pass (T=2048), two separate --pmc passes.
# usage: bash scripts/pmc_prefill.sh <tag> [T] [q4_0|kq]   (kq: the Q4_K_M layout, scripts/kq_prefill.py)
set -o pipefail
TAG=$1; T=${2:-2048}; KIND=${3:-q4_0}
if [ "$KIND" = kq ]; then DRV="scripts/kq_prefill.py $T 0"; else DRV="scripts/prof_prefill.py $T 1 0"; fi
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
timeout -s KILL 60 rocprofv3 -L > $OUT/counters.txt 2>&1 || true
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS --output-format csv -d $OUT/pmc1 -o run -- python3 $DRV > $OUT/pmc1.log 2>&1 || { tail -5 $OUT/pmc1.log; exit 1; }
timeout -s KILL 120 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_INST_LDS GRBM_GUI_ACTIVE --output-format csv -d $OUT/pmc2 -o run -- python3 $DRV > $OUT/pmc2.log 2>&1 || { tail -5 $OUT/pmc2.log; exit 1; }
python3 scripts/pmc_table.py $OUT k_gemm
