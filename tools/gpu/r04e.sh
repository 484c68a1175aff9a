# Round 4: whole GPU suite, then the default bench (every leg).
set -o pipefail
OUT=gpurun_out/r04e; mkdir -p $OUT
timeout -k 10 900 python -u -m pytest tests -m gpu -v -s --timeout 300 --timeout-method thread > $OUT/gpu_tests.log 2>&1 || { grep -E "s4:|FAILED|Error" $OUT/gpu_tests.log | head -20; tail -30 $OUT/gpu_tests.log; exit 1; }
grep -E "s4:|ids identical|passed|failed" $OUT/gpu_tests.log | tail -8
timeout -k 10 600 python -u bench.py > $OUT/bench.json 2> $OUT/bench.err || { tail -20 $OUT/bench.err; exit 1; }
python3 -c "
import json; d=json.loads(open('$OUT/bench.json').read().strip().splitlines()[-1]); print(d['value'], d['ms_per_step'], d['kernel_ms_per_step']); print('fp64', d['fp64']['value'], 'prop', d['propagation'].get('roofline',{}).get('frac'), 'ate', d['ate'].get('frames_per_s'), 'acc', d.get('accuracy'), d['replicas'])"
