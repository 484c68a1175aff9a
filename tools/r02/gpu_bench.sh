# Default bench line (all legs) on one GPU.
set -o pipefail
OUT=gpurun_out/${1:-r02c}
mkdir -p $OUT
timeout -k 10 400 python -u bench.py > $OUT/bench.json 2> $OUT/bench.err
