# One round checkpoint (profiles/<tag>): the GPU suite, the bench line with
# every leg, kernel-trace stats, FETCH / WRITE passes, SQ counters of the hot
# kernels, the fp64 configs 3 / 5 and the config-4 scheduler run.
#   bash tools/gpu/round.sh r03
set -o pipefail
TAG=${1:-r03}; OUT=gpurun_out/$TAG; mkdir -p $OUT
timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread > $OUT/gpu_tests.log 2>&1 || { tail -40 $OUT/gpu_tests.log; exit 1; }
tail -2 $OUT/gpu_tests.log
timeout -k 10 600 python -u bench.py > $OUT/bench.json 2> $OUT/bench.err || { tail -20 $OUT/bench.err; exit 1; }
bash tools/profile_round.sh $TAG 3 || exit 1
bash tools/gpu/sq.sh $TAG/sqp "k_gate|k_info|k_kal|k_feature" || exit 1
timeout -k 10 600 python -u bench.py --N 50 --F 400 --dtype fp64 --no-cpu --no-ate --no-prop > $OUT/bench_50x400_fp64.json 2> $OUT/b50.err || exit 1
timeout -k 10 600 python -u bench.py --N 80 --F 1000 --dtype fp64 --batch 512 --no-cpu --no-ate --no-prop > $OUT/bench_80x1000_fp64.json 2> $OUT/b80.err || exit 1
timeout -k 10 600 python -u tools/bench_sequences.py --seqs 11 > $OUT/sequences.json 2> $OUT/seq.err || exit 1
timeout -k 10 300 python -u tools/profile_frame.py > $OUT/frame.json 2> $OUT/frame.err || exit 1
tail -c 600 $OUT/bench.json
