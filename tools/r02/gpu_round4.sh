# Round-2 final checkpoint: GPU parity suite, default bench line (all legs), the
# kernel-trace / FETCH_SIZE / WRITE_SIZE profile passes, SQ counters of the update
# kernels, and the propagation kernel's trace + SQ counters (2048 filters x 10 samples).
set -o pipefail
TAG=${1:-r02v4}
OUT=gpurun_out/$TAG
mkdir -p $OUT
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $OUT/t.log 2>&1 &&
timeout -k 10 600 python -u bench.py > $OUT/bench.json 2> $OUT/bench.err &&
timeout -k 10 900 bash tools/profile_round.sh $TAG 3 || exit 1
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
CTR="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_MFMA SQ_LDS_BANK_CONFLICT"
timeout -s KILL 90 rocprofv3 --pmc $CTR --kernel-include-regex "k_gate|k_info|k_kal|k_feature" -d $OUT/sq -o run --output-format csv -- \
    python3 bench.py --steps 1 --warmup 0 --no-cpu --no-ate --no-prop --no-fp64 > $OUT/sq.log 2>&1 || exit 1
export PROP_ONE=2048,10
timeout -k 10 120 rocprofv3 --kernel-trace --stats --kernel-include-regex k_propagate -d $OUT/prop -o run --output-format csv -- \
    python3 tools/prop_sweep.py > $OUT/prop.log 2>&1 || exit 1
timeout -s KILL 90 rocprofv3 --pmc $CTR --kernel-include-regex k_propagate -d $OUT/propsq -o run --output-format csv -- \
    python3 tools/prop_sweep.py > $OUT/propsq.log 2>&1
