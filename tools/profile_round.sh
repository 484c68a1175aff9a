#!/bin/bash
# Profiles committed under profiles/<tag>/ (run on the GPU box from the repo root):
#   kernel-trace stats of the default bench, separate FETCH_SIZE / WRITE_SIZE
#   passes over every msckf kernel, and the per-stage PMC summary.
#   bash tools/profile_round.sh r01 [steps [bench args ...]]   (e.g. --N 50 --F 400 --no-fp64)
set -e
TAG=${1:-r01}; STEPS=${2:-3}; shift 2 || true
OUT=gpurun_out/prof_$TAG
mkdir -p $OUT/stats $OUT/fetch $OUT/write
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/stats -o run --output-format csv -- \
    python3 bench.py --steps $STEPS --warmup 1 --no-cpu --no-ate --no-prop "$@" > $OUT/stats/bench.log 2>&1
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --kernel-include-regex "msckf" -d $OUT/fetch -o run --output-format csv -- \
    python3 bench.py --steps 1 --warmup 0 --no-cpu --no-ate --no-prop "$@" > $OUT/fetch/bench.log 2>&1
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --kernel-include-regex "msckf" -d $OUT/write -o run --output-format csv -- \
    python3 bench.py --steps 1 --warmup 0 --no-cpu --no-ate --no-prop "$@" > $OUT/write/bench.log 2>&1
# the per-stage summary, labelled with the workload and dtype of the passes' own bench line
python3 tools/pmc_summary.py $OUT/fetch/run_counter_collection.csv $OUT/write/run_counter_collection.csv \
    --bench-log $OUT/fetch/bench.log --source "$TAG: rocprofv3 FETCH_SIZE / WRITE_SIZE passes" \
    -o $OUT/pmc_summary.json > $OUT/pmc_summary.txt
