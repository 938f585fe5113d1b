#!/bin/bash
# Round-4 GPU pass: the new prefill attention and GEMM change (tests, timing, rocprof, PMC), the
# K-quant prologue change (tests + A/B against ab_libs/libnorm0.so), decode phase stamps.
# usage (repo root, GPU box): bash scripts/r04_check.sh <tag> [steps...]   steps: pf kq stamp pmc
set -o pipefail
TAG=${1:-r04}; shift
STEPS=${@:-"pf kq stamp pmc"}
O=gpurun_out/$TAG
mkdir -p $O
export TMPDIR=/tmp
for st in $STEPS; do
  case $st in
    pf)
      timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_prefill.py -m gpu -k "exact or mfma" > $O/pf_tests.log 2>&1 || { tail -30 $O/pf_tests.log; exit 1; }
      tail -1 $O/pf_tests.log
      for mx in 1 0; do GHIP_ATT_MX=$mx timeout -k 10 120 python scripts/prof_prefill.py 2048 1 3 > $O/pf_t_$mx.txt 2>&1 || exit 1; echo "GHIP_ATT_MX=$mx"; cat $O/pf_t_$mx.txt; done
      timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $O/prof_pf -o run -- python3 scripts/prof_prefill.py 2048 1 1 > $O/prof_pf.log 2>&1 || { tail -5 $O/prof_pf.log; exit 1; }
      f=$(find $O/prof_pf -name "*kernel_stats.csv" | head -1); [ -n "$f" ] && cp $f $O/kernel_stats_prefill.csv && head -8 $O/kernel_stats_prefill.csv | cut -c1-160 ;;
    kq)
      timeout -k 10 500 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_kquants.py tests/test_gpu_engine_gguf.py -m gpu > $O/kq_tests.log 2>&1 || { tail -30 $O/kq_tests.log; exit 1; }
      tail -1 $O/kq_tests.log
      for rep in 1 2 3; do
        GHIP_LIB=$PWD/ab_libs/libnorm0.so timeout -k 10 120 python scripts/run_kqm.py 64 2>&1 | sed "s/^/base /" || exit 1
        timeout -k 10 120 python scripts/run_kqm.py 64 2>&1 | sed "s/^/new  /" || exit 1
      done ;;
    stamp)
      GHIP_LIB=$PWD/ab_libs/libstamps.so timeout -k 10 180 python tests/stamp_step.py 9 > $O/stamp_step.log 2>&1 || { tail -20 $O/stamp_step.log; exit 1; }
      cat $O/stamp_step.log ;;
    attn)
      # decode attention without the KQV-phase spills (new) vs the spilling build (base) and K prefetch 8
      timeout -k 10 500 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_parity.py tests/test_gpu_ops.py -m gpu -k "decode or attn or attention" > $O/attn_tests.log 2>&1 || { tail -30 $O/attn_tests.log; exit 1; }
      tail -1 $O/attn_tests.log
      for v in base new akpf8; do
        L=""; [ $v != new ] && L=$PWD/ab_libs/lib$v.so
        GHIP_LIB=$L timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $O/prof_$v -o run -- python3 bench.py --no-cpu --prefill 0 --tp-steps 0 --q8-steps 0 --ggml-steps 0 --steps 32 > $O/prof_$v.json 2> $O/prof_$v.err || { tail -5 $O/prof_$v.err; exit 1; }
        f=$(find $O/prof_$v -name "*kernel_stats.csv" | head -1)
        echo "== $v $(python3 -c "import json; d=json.load(open('$O/prof_$v.json')); print(d['value'], d['ms_per_step'])")"
        grep -E "k_attn_head" $f | cut -d, -f1-8 | cut -c1-200
      done
      for rep in 1 2; do for v in base new akpf8; do
        L=""; [ $v != new ] && L=$PWD/ab_libs/lib$v.so
        GHIP_LIB=$L timeout -k 10 240 python bench.py --no-cpu --prefill 0 --tp-steps 0 --q8-steps 0 --ggml-steps 0 > $O/ab_$v$rep.json 2> $O/ab_$v$rep.err || { tail -20 $O/ab_$v$rep.err; exit 1; }
        python3 -c "import json; d=json.load(open('$O/ab_$v$rep.json')); print('$v', d['value'], d['ms_per_step'], (d.get('q4_k_m_decode') or {}).get('tok_s'))"
      done; done ;;
    vdma)
      # decode attention V rows by LDS-DMA (GHIP_ATT_VDMA=1) vs register/global loads (the default)
      timeout -k 10 500 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_parity.py tests/test_gpu_ops.py tests/test_gpu_persist.py -m gpu > $O/vdma_tests.log 2>&1 || { tail -30 $O/vdma_tests.log; exit 1; }
      tail -1 $O/vdma_tests.log
      for v in 1 0; do GHIP_ATT_VDMA=$v GHIP_LIB=$PWD/ab_libs/libstamps.so timeout -k 10 180 python tests/stamp_step.py 9 > $O/vdma_stamp_$v.log 2>&1 || { tail -20 $O/vdma_stamp_$v.log; exit 1; }; echo "== VDMA=$v"; grep -A2 "^attention" $O/vdma_stamp_$v.log; done
      for rep in 1 2; do for v in 1 0; do
        GHIP_ATT_VDMA=$v timeout -k 10 240 python bench.py --no-cpu --prefill 0 --tp-steps 0 --q8-steps 0 --ggml-steps 0 > $O/vdma_$v$rep.json 2> $O/vdma_$v$rep.err || { tail -20 $O/vdma_$v$rep.err; exit 1; }
        python3 -c "import json; d=json.load(open('$O/vdma_$v$rep.json')); print('VDMA=$v', d['value'], d['ms_per_step'])"
      done; done ;;
    attn2)
      # decode attention round-4 changes (V by LDS-DMA, own-row operand swap, single-exp softmax)
      # against the previous build (ab_libs/libbase.so), and the new build with the DMA off
      timeout -k 10 500 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_parity.py tests/test_gpu_ops.py tests/test_gpu_persist.py tests/test_gpu_ggml_graph.py -m gpu > $O/attn2_tests.log 2>&1 || { tail -30 $O/attn2_tests.log; exit 1; }
      tail -1 $O/attn2_tests.log
      GHIP_LIB=$PWD/ab_libs/libstamps.so timeout -k 10 180 python tests/stamp_step.py 9 > $O/attn2_stamp.log 2>&1 || { tail -20 $O/attn2_stamp.log; exit 1; }; grep -A2 "^attention" $O/attn2_stamp.log
      for rep in 1 2 3; do for v in base new nodma; do
        L=""; E=1; [ $v = base ] && L=$PWD/ab_libs/libbase.so; [ $v = nodma ] && E=0  # new = DMA on
        GHIP_ATT_VDMA=$E GHIP_LIB=$L timeout -k 10 240 python bench.py --no-cpu --prefill 0 --tp-steps 0 --q8-steps 0 --ggml-steps 0 > $O/a2_$v$rep.json 2> $O/a2_$v$rep.err || { tail -20 $O/a2_$v$rep.err; exit 1; }
        python3 -c "import json; d=json.load(open('$O/a2_$v$rep.json')); print('$v', d['value'], d['ms_per_step'])"
      done; done ;;
    pmc)
      bash scripts/pmc_prefill.sh $TAG/pmc 2048 > $O/pmc.log 2>&1 || { tail -20 $O/pmc.log; exit 1; }
      tail -24 $O/pmc.log ;;
  esac
done
