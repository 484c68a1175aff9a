# A/B with repeats: base and each experiment build alternated R times (noise estimate).
#   bash tools/gpu/exp2.sh r03x 2 seg1 wpb1 ...
#   BENCH_ARGS="--N 50 --F 400 --dtype fp64 ..." bash tools/gpu/exp2.sh ...   (other workloads)
set -o pipefail
OUT=gpurun_out/${1:-exp}; R=${2:-2}; shift 2; mkdir -p $OUT
ARGS=${BENCH_ARGS:-"--no-cpu --no-ate --no-prop --no-fp64"}
for r in $(seq 1 $R); do
  timeout -k 10 300 python -u bench.py $ARGS > $OUT/base_$r.json 2> $OUT/base_$r.err || { tail -20 $OUT/base_$r.err; exit 1; }
  for e in "$@"; do
    timeout -k 10 300 python -u tools/exp_bench.py tools/exp/libmsckf_$e.so $ARGS > $OUT/${e}_$r.json 2> $OUT/${e}_$r.err || { tail -20 $OUT/${e}_$r.err; exit 1; }
  done
done
for f in $OUT/*.json; do
  python3 -c "
import json; d=json.loads(open('$f').read().strip().splitlines()[-1]); k=d['kernel_ms_per_step']
print('$f', d['value'], d['ms_per_step'], 'gate', k.get('gate'), 'feat', k.get('feature_jacobian'), 'tri', k.get('triangulate'))"
done
