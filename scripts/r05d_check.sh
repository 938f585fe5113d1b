set -o pipefail
O=gpurun_out/r05d
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 700 python -u -m pytest tests/ -x -q --timeout 400 --timeout-method thread -m gpu > $O/t.log 2>&1; echo rc=$? >> $O/t.log
tail -3 $O/t.log
bash scripts/lib_ab.sh > $O/ab.txt 2>&1 || exit 1
cat $O/ab.txt
for f in gpurun_out/libab/base1.json gpurun_out/libab/new1.json gpurun_out/libab/base2.json gpurun_out/libab/new2.json; do python3 -c "
import json; d=json.load(open('$f')); c=d['roofline']['classes']
print('$f', d['value'], ' '.join('%s=%.2f' % (k.split()[0], v['avg_us']) for k, v in c.items()))"; done
OUT=r05d/ew ENVA="GHIP_RR_EW=0" ENVB="GHIP_RR_EW=2" REPS=2 bash scripts/env_ab.sh || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof -o run -- python3 scripts/decode_prof.py 48 > $O/prof.log 2>&1 || { tail -20 $O/prof.log; exit 1; }
python3 scripts/decode_classes.py $O/prof/run_results.db 128 48 "9,1,0,9,1,0,1,1,0,9,1,1,1,8,0" > $O/decode_kernels.md
cat $O/decode_kernels.md
