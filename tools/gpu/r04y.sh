# kernel stats of the per-frame path, split off / on
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
OUT=gpurun_out/r04y; mkdir -p $OUT
for sp in 0 1; do
  MSCKF_KAL_SPLIT=$sp timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/s$sp -o run --output-format csv -- python3 tools/profile_frame.py --frames 120 > $OUT/s$sp.log 2>&1 || { tail -20 $OUT/s$sp.log; exit 1; }
done
find $OUT -name "*kernel_stats.csv"
