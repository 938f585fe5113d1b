set -o pipefail
O=gpurun_out/r05m
mkdir -p $O
export TMPDIR=/tmp
OUT=r05m/kq VARS="new=new pf3=kqpf3 pf4=kqpf4 gu2=new:GHIP_KQ_GU2=1" REPS=3 bash scripts/kqm_ab.sh
for i in 1 2; do
timeout -k 10 300 python bench.py --no-cpu --prefill 0 --tp-steps 0 --q8-steps 0 --ggml-steps 0 > $O/b$i.json 2> $O/b$i.err || { tail -20 $O/b$i.err; exit 1; }
python3 -c "
import json; d=json.load(open('$O/b$i.json')); print('decode', d['value'], d['launch_plan']['logits'], [(k.split()[0], v['avg_us']) for k, v in d['roofline']['classes'].items()])"
done
KQ=1 GHIP_LIB=$PWD/ab_libs/libst1.so timeout -k 10 180 python tests/stamp_step.py 9 > $O/st_kq.log 2>&1 || { tail -20 $O/st_kq.log; exit 1; }
cat $O/st_kq.log
