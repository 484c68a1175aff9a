# GPU parity suite + the bench line (no CPU leg unless $2 = cpu).  Output under gpurun_out/<tag>.
#   bash tools/gpu/check.sh r03a [cpu]
set -o pipefail
OUT=gpurun_out/${1:-check}
mkdir -p $OUT
CPU="--no-cpu --no-ate"; [ "$2" = cpu ] && CPU=""
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $OUT/t.log 2>&1 &&
timeout -k 10 600 python -u bench.py $CPU > $OUT/b.json 2> $OUT/b.err
