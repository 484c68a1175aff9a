# SURVEY configs 3 / 5 bench lines (with CPU baselines), the 11-sequence scheduler run, front-end throughput.
set -o pipefail
OUT=gpurun_out/${1:-r02cfg}
mkdir -p $OUT
timeout -k 10 400 python -u bench.py --N 50 --F 400 --batch 512 --no-fp64 --no-ate --no-prop --cpu-seconds 20 > $OUT/b50.json 2> $OUT/b50.err &&
timeout -k 10 400 python -u bench.py --N 80 --F 1000 --batch 128 --no-fp64 --no-ate --no-prop --cpu-seconds 20 > $OUT/b80.json 2> $OUT/b80.err &&
timeout -k 10 400 python -u tools/bench_sequences.py --seqs 11 > $OUT/seq.json 2> $OUT/seq.err &&
timeout -k 10 300 python -u tools/bench_frontend.py > $OUT/fe.json 2> $OUT/fe.err
