# Same-box A/B of the in-tree package against a saved copy (library included):
#   bash tools/gpu/ab_pkg.sh TAG PKG_DIR "bench args"
# One bench process per side (each under its own time limit), alternated twice.
set -o pipefail
OUT=gpurun_out/$1; PKG=$2; ARGS=$3
mkdir -p $OUT
for rep in 1 2; do
  for side in base new; do
    if [ $side = base ]; then CMD="python3 -u tools/exp/run_pkg.py $PKG bench.py"; else CMD="python3 -u bench.py"; fi
    timeout -k 10 300 $CMD $ARGS --no-cpu --no-ate --no-prop --no-fp64 > $OUT/${side}_$rep.json 2> $OUT/${side}_$rep.err \
      || { echo "side $side failed"; tail -20 $OUT/${side}_$rep.err; exit 1; }
    python3 -c "
import json; d=json.loads(open('$OUT/${side}_$rep.json').read().strip().splitlines()[-1]); k=d['kernel_ms_per_step']
print('$side rep $rep', d['value'], d['ms_per_step'], {n: round(v, 4) for n, v in k.items() if n.startswith('kalman')})"
  done
done
