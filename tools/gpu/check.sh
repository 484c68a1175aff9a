# GPU parity suite, the bench line, the per-frame drop-in path and (with
# "full") the fp64 legs at configs 3 and 5.  Output under gpurun_out/<tag>.
#   bash tools/gpu/check.sh r03i [cpu] [full]
set -o pipefail
OUT=gpurun_out/${1:-check}
mkdir -p $OUT
CPU="--no-cpu --no-ate"; [ "$2" = cpu ] && CPU=""
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $OUT/t.log 2>&1 || { tail -40 $OUT/t.log; exit 1; }
tail -3 $OUT/t.log
timeout -k 10 600 python -u bench.py $CPU > $OUT/b.json 2> $OUT/b.err || { tail -20 $OUT/b.err; exit 1; }
timeout -k 10 300 python -u tools/profile_frame.py > $OUT/frame.json 2> $OUT/frame.err || { tail -20 $OUT/frame.err; exit 1; }
if [ "$3" = full ]; then
  timeout -k 10 600 python -u bench.py --N 50 --F 400 --dtype fp64 --no-cpu --no-ate --no-prop > $OUT/b_50x400_fp64.json 2> $OUT/b_50x400_fp64.err || exit 1
  timeout -k 10 600 python -u bench.py --N 80 --F 1000 --dtype fp64 --batch 512 --no-cpu --no-ate --no-prop > $OUT/b_80x1000_fp64.json 2> $OUT/b_80x1000_fp64.err || exit 1
  timeout -k 10 600 python -u tools/bench_sequences.py --seqs 11 > $OUT/seq.json 2> $OUT/seq.err || exit 1
fi
cat $OUT/frame.json
