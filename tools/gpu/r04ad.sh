# Kalman B phase 1: column-major round-robin tile deal (default) vs 3x3 blocks with interleaved columns (kbil)
set -o pipefail
OUT=gpurun_out/r04ad; mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 200 --timeout-method thread -k "update or batched or cholesky or sequence" > $OUT/t.log 2>&1 || { tail -30 $OUT/t.log; exit 1; }
tail -2 $OUT/t.log
bash tools/gpu/exp.sh r04ad/ab1 kbil || exit 1
bash tools/gpu/exp.sh r04ad/ab2 kbil || exit 1
for f in $OUT/ab*/*.json; do python3 -c "import json; d=json.loads(open('$f').read().strip().splitlines()[-1]); print('$f', d['kernel_ms_per_step']['kalman_b'])"; done
