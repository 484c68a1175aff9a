# GPU parity suite, then the default bench line.
set -o pipefail
OUT=gpurun_out/${1:-r02b}
mkdir -p $OUT
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $OUT/t.log 2>&1 &&
timeout -k 10 300 python -u bench.py --no-cpu > $OUT/b32.json 2> $OUT/b32.err
