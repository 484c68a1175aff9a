# Full GPU parity suite + the bench line without the CPU leg (fp32 headline and fp64 leg).
set -o pipefail
OUT=gpurun_out/${1:-r02c}
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/t.log 2>&1 &&
timeout -k 10 300 python -u bench.py --no-cpu --no-ate > $OUT/b.json 2> $OUT/b.err
