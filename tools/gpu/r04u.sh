# Kalman B: interleaved tile columns in phase 1 (balanced chunks).
set -o pipefail
OUT=gpurun_out/r04u; mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 200 --timeout-method thread -k "update or batched or cholesky or sequence_s1" > $OUT/t.log 2>&1 || { tail -30 $OUT/t.log; exit 1; }
tail -2 $OUT/t.log
bash tools/gpu/exp.sh r04u/ab1 kbc || exit 1
bash tools/gpu/exp.sh r04u/ab2 kbc || exit 1
for f in $OUT/ab1/*.json $OUT/ab2/*.json; do python3 -c "import json; d=json.loads(open('$f').read().strip().splitlines()[-1]); print('$f', d['kernel_ms_per_step']['kalman_b'])"; done
