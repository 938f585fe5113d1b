set -o pipefail
O=gpurun_out/r05z
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests/ -x -q --timeout 400 --timeout-method thread -m gpu > $O/t.log 2>&1; rc=$?; tail -2 $O/t.log; [ $rc = 0 ] || exit 1
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1; rc=$?; tail -2 $O/smoke.log; [ $rc = 0 ] || exit 1
timeout -k 10 600 python bench.py > $O/bench.json 2> $O/bench.err || { tail -20 $O/bench.err; exit 1; }
python3 -c "
import json; d=json.load(open('$O/bench.json'))
print('decode', d['value'], 'kqm', d['q4_k_m_decode']['tok_s'], 'q8', d['q8_0_decode']['tok_s'], 'q6o', d['q4_0_q6k_output_decode']['tok_s'], 'prefill', d['prefill'].get('ms'), 'cpu', d['cpu_baseline'].get('value'), 'gu', d['roofline']['avg_us'])"
