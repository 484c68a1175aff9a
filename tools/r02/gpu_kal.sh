# GPU parity suite, the fp32 bench, and a kernel-trace --stats profile of the bench.
set -o pipefail
OUT=gpurun_out/${1:-r02h}
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $OUT/t.log 2>&1 &&
timeout -k 10 300 python -u bench.py --no-cpu --no-ate --no-fp64 --no-prop > $OUT/b32.json 2> $OUT/b32.err || exit 1
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/stats -o run --output-format csv -- \
    python3 bench.py --steps 3 --warmup 1 --no-cpu --no-ate --no-prop --no-fp64 > $OUT/stats.log 2>&1
