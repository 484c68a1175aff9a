# Quick: fp32 parity tests of the batched update + default fp32 bench (no CPU / fp64 / ATE / propagation legs).
set -o pipefail
OUT=gpurun_out/${1:-r02q}
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q -k "batched or gate or sequence" --timeout 300 --timeout-method thread > $OUT/t.log 2>&1 &&
timeout -k 10 300 python -u bench.py --no-cpu --no-ate --no-fp64 --no-prop > $OUT/b32.json 2> $OUT/b32.err
