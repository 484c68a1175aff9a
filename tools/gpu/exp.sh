# A/B of experiment builds against the default library on the headline bench
# (fp32 context, no CPU / ATE / propagation / fp64 legs), each a separate process.
#   bash tools/gpu/exp.sh r03x kf8 kf12 ...
set -o pipefail
OUT=gpurun_out/${1:-exp}; shift; mkdir -p $OUT
ARGS="--no-cpu --no-ate --no-prop --no-fp64"
timeout -k 10 300 python -u bench.py $ARGS > $OUT/base.json 2> $OUT/base.err || { tail -20 $OUT/base.err; exit 1; }
for e in "$@"; do
  timeout -k 10 300 python -u tools/exp_bench.py tools/exp/libmsckf_$e.so $ARGS > $OUT/$e.json 2> $OUT/$e.err || { tail -20 $OUT/$e.err; exit 1; }
done
for f in $OUT/*.json; do
  python3 -c "
import json,sys; d=json.loads(open('$f').read().strip().splitlines()[-1]); k=d['kernel_ms_per_step']
print('$f', d['value'], d['ms_per_step'], 'compress', k.get('compress'), 'gate', k.get('gate'), 'kc', k.get('kalman_c'), 'acc', d.get('accuracy',{}).get('state_rel_dev_max'), d.get('accuracy',{}).get('decision_agreement'))"
done
