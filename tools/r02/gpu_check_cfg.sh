# GPU parity suite, the default bench line (no CPU leg) and the SURVEY config-3 shape (50 x 400, fp32).
set -o pipefail
OUT=gpurun_out/${1:-r02cc}
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/t.log 2>&1 &&
timeout -k 10 300 python -u bench.py --no-cpu --no-ate > $OUT/b.json 2> $OUT/b.err &&
timeout -k 10 300 python -u bench.py --N 50 --F 400 --batch 512 --no-fp64 --no-ate --no-prop --no-cpu > $OUT/b50.json 2> $OUT/b50.err
