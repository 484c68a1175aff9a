# rocprofv3 kernel stats of one bench config per value of an experiment variable:
#   bash tools/gpu/stats_env.sh TAG VAR "v1 v2 ..." "bench args"
set -o pipefail
OUT=gpurun_out/$1; VAR=$2; VALS=$3; ARGS=$4
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
for v in $VALS; do
  export $VAR=$v
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/s_$v -o run --output-format csv -- \
      python3 bench.py --steps 2 --warmup 0 --no-cpu --no-ate --no-prop --no-fp64 $ARGS > $OUT/s_$v.log 2>&1 \
      || { echo "value $v failed"; tail -20 $OUT/s_$v.log; exit 1; }
  python3 - $OUT/s_$v/run_kernel_stats.csv $v <<'PY'
import csv, sys
rows = [r for r in csv.DictReader(open(sys.argv[1])) if "k_gate" in r["Name"]]
print("value", sys.argv[2])
for r in sorted(rows, key=lambda r: -float(r["TotalDurationNs"])):
    n = r["Name"].replace("msckf::", "").replace("(anonymous namespace)::", "").replace("void ", "").split("(")[0]
    print("  %-36s calls %4s avg %9.1f us" % (n, r["Calls"], float(r["AverageNs"]) / 1e3))
PY
done
