# Kalman C2: double-buffered block-row staging (one barrier per step) and 4 accumulators.
set -o pipefail
OUT=gpurun_out/r04s; mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 200 --timeout-method thread -k "update or batched or cholesky or sequence_s1" > $OUT/t.log 2>&1 || { tail -30 $OUT/t.log; exit 1; }
tail -2 $OUT/t.log
bash tools/gpu/exp.sh r04s/ab1 db0 acc4 || exit 1
bash tools/gpu/exp.sh r04s/ab2 db0 acc4 || exit 1
