# GPU parity suite, then the fp32 bench with the propagation leg.
set -o pipefail
OUT=gpurun_out/${1:-r02k}
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $OUT/t.log 2>&1 &&
timeout -k 10 300 python -u bench.py --no-cpu --no-ate --no-fp64 > $OUT/b32.json 2> $OUT/b32.err
