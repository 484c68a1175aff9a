# Quick GPU iteration: a pytest selection, then (optionally) one bench config.
#   bash tools/gpu/quick.sh TAG "k-expression" ["bench args"]
set -o pipefail
OUT=gpurun_out/$1; mkdir -p $OUT
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread -k "$2" > $OUT/t.log 2>&1 || { tail -30 $OUT/t.log; exit 1; }
tail -3 $OUT/t.log
if [ -n "$3" ]; then
  timeout -k 10 400 python -u bench.py $3 > $OUT/b.json 2> $OUT/b.err || { tail -20 $OUT/b.err; exit 1; }
  python3 -c "
import json; d=json.loads(open('$OUT/b.json').read().strip().splitlines()[-1]); print(d['value'], d['ms_per_step'], d.get('kernel_ms_per_step'))"
fi
