# Kernel-trace stats of the fp64-context bench (per-class gating times).
set -o pipefail
OUT=gpurun_out/${1:-r02p64}
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/stats -o run --output-format csv -- \
    python3 bench.py --dtype fp64 --steps 3 --warmup 1 --no-cpu --no-ate --no-prop --no-fp64 > $OUT/bench.log 2>&1
