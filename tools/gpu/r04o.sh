# Multi-context overlap experiment (2048 filters over K contexts / streams).
set -o pipefail
OUT=gpurun_out/r04o; mkdir -p $OUT
timeout -k 10 400 python -u tools/exp_two_ctx.py --k 1 2 4 1 2 > $OUT/k.json 2> $OUT/k.err || { tail -20 $OUT/k.err; exit 1; }
cat $OUT/k.json
