# A/B of one repo script across experiment builds (tools/exp/libmsckf_<name>.so)
# and the working tree ("base"), alternated R times.
#   bash tools/gpu/exp_script.sh TAG R "script.py args" name [name ...]
set -o pipefail
OUT=gpurun_out/$1; R=$2; SCRIPT=$3; shift 3; mkdir -p $OUT
for r in $(seq 1 $R); do
  for e in base "$@"; do
    if [ $e = base ]; then
      timeout -k 10 300 python -u $SCRIPT > $OUT/${e}_$r.out 2> $OUT/${e}_$r.err || { tail -20 $OUT/${e}_$r.err; exit 1; }
    else
      timeout -k 10 300 python -u tools/exp_run.py tools/exp/libmsckf_$e.so $SCRIPT > $OUT/${e}_$r.out 2> $OUT/${e}_$r.err || { tail -20 $OUT/${e}_$r.err; exit 1; }
    fi
  done
done
