# rocprofv3 kernel-trace statistics of a short bench run (fp32 headline + fp64 leg).
#   bash tools/gpu/stats.sh r03t [bench args]
set -o pipefail
OUT=gpurun_out/${1:-stats}; shift
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/stats -o run --output-format csv -- \
    python3 bench.py --steps 3 --warmup 1 --no-cpu --no-ate --no-prop "$@" > $OUT/stats.log 2>&1
