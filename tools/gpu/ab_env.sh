# Same-box A/B of an experiment environment variable over one bench config:
#   bash tools/gpu/ab_env.sh TAG VAR "v1 v2 ..." "bench args"
# One bench process per value (each under its own time limit), alternated twice.
set -o pipefail
OUT=gpurun_out/$1; VAR=$2; VALS=$3; ARGS=$4
mkdir -p $OUT
for rep in 1 2; do
  for v in $VALS; do
    env $VAR=$v timeout -k 10 300 python3 -u bench.py $ARGS --no-cpu --no-ate --no-prop --no-fp64 > $OUT/${v}_$rep.json 2> $OUT/${v}_$rep.err \
      || { echo "value $v failed"; tail -20 $OUT/${v}_$rep.err; exit 1; }
    python3 -c "
import json; d=json.loads(open('$OUT/${v}_$rep.json').read().strip().splitlines()[-1]); k=d['kernel_ms_per_step']
print('$VAR=$v rep $rep', d['value'], d['ms_per_step'], 'gate', k.get('gate'), k)"
  done
done
