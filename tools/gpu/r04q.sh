# Timing diagnostics: bench steps 20 / 50 vs the bare K = 1 loop at 20 / 50 steps.
set -o pipefail
OUT=gpurun_out/r04q; mkdir -p $OUT
A="--no-cpu --no-ate --no-prop --no-fp64"
timeout -k 10 300 python -u bench.py $A --steps 20 > $OUT/b20.json 2> $OUT/b20.err || { tail -20 $OUT/b20.err; exit 1; }
timeout -k 10 300 python -u bench.py $A --steps 50 > $OUT/b50.json 2> $OUT/b50.err || { tail -20 $OUT/b50.err; exit 1; }
timeout -k 10 300 python -u tools/exp_two_ctx.py --k 1 --steps 50 > $OUT/k50.json 2> $OUT/k50.err || { tail -20 $OUT/k50.err; exit 1; }
timeout -k 10 300 python -u tools/exp_two_ctx.py --k 1 --steps 20 > $OUT/k20.json 2> $OUT/k20.err || { tail -20 $OUT/k20.err; exit 1; }
for f in $OUT/b20.json $OUT/b50.json; do python3 -c "import json; d=json.loads(open('$f').read().strip().splitlines()[-1]); print('$f', d['value'], d['ms_per_step'], d['roofline']['ms_per_step'], d['kernel_ms_per_step']['gate'])"; done
cat $OUT/k50.json $OUT/k20.json
