set -o pipefail
O=gpurun_out/r05l
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests/ -x -q --timeout 400 --timeout-method thread -m gpu > $O/t.log 2>&1; rc=$?; tail -3 $O/t.log; [ $rc = 0 ] || exit 1
timeout -k 10 600 python bench.py > $O/bench.json 2> $O/bench.err || { tail -20 $O/bench.err; exit 1; }
python3 -c "
import json; d=json.load(open('$O/bench.json'))
print('decode', d['value'], 'plan', d['launch_plan'])
print('kqm', d['q4_k_m_decode']); print('q8', d['q8_0_decode']); print('prefill', d['prefill'].get('exact', d['prefill']) if isinstance(d['prefill'], dict) else d['prefill'])
print('classes', [(k.split()[0], v['avg_us']) for k, v in d['roofline']['classes'].items()])"
