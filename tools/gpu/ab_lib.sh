# Same-box A/B of the in-tree library against experiment builds on one or more
# bench configs (each run a separate process under its own time limit):
#   bash tools/gpu/ab_lib.sh TAG "exp1 exp2" "cfgname:bench args" ["cfgname:bench args" ...]
set -o pipefail
OUT=gpurun_out/$1; EXPS=$2; shift 2; mkdir -p $OUT
COMMON="--no-cpu --no-ate --no-prop --no-fp64"
for cfg in "$@"; do
  name=${cfg%%:*}; args=${cfg#*:}
  timeout -k 10 400 python3 -u bench.py $args $COMMON > $OUT/${name}_base.json 2> $OUT/${name}_base.err || { tail -20 $OUT/${name}_base.err; exit 1; }
  for e in $EXPS; do
    timeout -k 10 400 python3 -u tools/exp_bench.py tools/exp/libmsckf_$e.so $args $COMMON > $OUT/${name}_$e.json 2> $OUT/${name}_$e.err || { tail -20 $OUT/${name}_$e.err; exit 1; }
  done
done
for f in $OUT/*.json; do
  python3 -c "
import json; d=json.loads(open('$f').read().strip().splitlines()[-1]); k=d['kernel_ms_per_step']
print('$f', d['value'], d['ms_per_step'], {x: k[x] for x in ('kalman_a', 'kalman_c', 'gate', 'compress') if x in k})"
done
