# Round-2 checkpoint: GPU parity suite, default bench line (all legs), the
# kernel-trace / FETCH_SIZE / WRITE_SIZE profile passes, and the gate's SQ counters.
set -o pipefail
TAG=${1:-r02v2}
OUT=gpurun_out/$TAG
mkdir -p $OUT
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $OUT/t.log 2>&1 &&
timeout -k 10 600 python -u bench.py > $OUT/bench.json 2> $OUT/bench.err &&
timeout -k 10 900 bash tools/profile_round.sh $TAG 3 || exit 1
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
CTR="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_MFMA SQ_LDS_BANK_CONFLICT"
timeout -s KILL 90 rocprofv3 --pmc $CTR --kernel-include-regex "k_gate|k_info|k_kal|k_feature" -d $OUT/sq -o run --output-format csv -- \
    python3 bench.py --steps 1 --warmup 0 --no-cpu --no-ate --no-prop --no-fp64 > $OUT/sq.log 2>&1
