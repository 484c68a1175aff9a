# Propagation: the filters x samples sweep, then kernel-trace stats of one
# 2048 x 10 launch (scalar kernel and matrix kernel separately).
#   bash tools/gpu/prop.sh r03p
set -o pipefail
OUT=gpurun_out/${1:-prop}; mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 300 python -u tools/prop_sweep.py > $OUT/sweep.json 2> $OUT/sweep.err || { tail -20 $OUT/sweep.err; exit 1; }
PROP_ONE=2048,10 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/stats -o run --output-format csv -- \
    python3 tools/prop_sweep.py > $OUT/stats.log 2>&1 || { tail -20 $OUT/stats.log; exit 1; }
cat $OUT/sweep.json
find $OUT/stats -name "*kernel_stats.csv" -exec cut -c1-160 {} \; | grep -i "prop"
