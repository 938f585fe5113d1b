set -o pipefail
O=gpurun_out/r05w
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python bench.py > $O/bench.json 2> $O/bench.err || { tail -20 $O/bench.err; exit 1; }
python3 -c "
import json; d=json.load(open('$O/bench.json'))
print('decode', d['value'], 'kqm', d['q4_k_m_decode']['tok_s'], 'q8', d['q8_0_decode']['tok_s'], 'q6o', d['q4_0_q6k_output_decode']['tok_s'], 'prefill', d['prefill'].get('ms'), 'cpu', d['cpu_baseline'].get('value'))"
