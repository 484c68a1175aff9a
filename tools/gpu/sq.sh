# SQ counter pass (per-wave instruction mix / waits) over the kernels matching $2
# in one fp32 bench step; summarise with tools/pmc_sq.py.
#   bash tools/gpu/sq.sh r03s "k_gate|k_info|k_kal|k_feature" [bench args]
set -o pipefail
OUT=gpurun_out/${1:-sq}; RE=${2:-msckf}; shift 2
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
CTR="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_MFMA SQ_LDS_BANK_CONFLICT"
timeout -s KILL 90 rocprofv3 --pmc $CTR --kernel-include-regex "$RE" -d $OUT/sq -o run --output-format csv -- \
    python3 bench.py --steps 1 --warmup 0 --no-cpu --no-ate --no-prop --no-fp64 "$@" > $OUT/sq.log 2>&1
