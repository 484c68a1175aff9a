# Counter passes over one 2048 x 10 propagation launch (tools/prop_sweep.py,
# PROP_ONE): SQ instruction mix / waits, then FETCH_SIZE and WRITE_SIZE, each
# pass a run of its own.
#   bash tools/gpu/prop_pmc.sh TAG
set -o pipefail
OUT=gpurun_out/${1:-prop_pmc}; mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
CTR="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_MFMA SQ_LDS_BANK_CONFLICT"
PROP_ONE=2048,10 timeout -s KILL 90 rocprofv3 --pmc $CTR --kernel-include-regex "k_propagate" -d $OUT/sq -o run --output-format csv -- \
    python3 tools/prop_sweep.py > $OUT/sq.log 2>&1 || { tail -20 $OUT/sq.log; exit 1; }
PROP_ONE=2048,10 timeout -s KILL 90 rocprofv3 --pmc FETCH_SIZE --kernel-include-regex "k_propagate" -d $OUT/fetch -o run --output-format csv -- \
    python3 tools/prop_sweep.py > $OUT/fetch.log 2>&1 || { tail -20 $OUT/fetch.log; exit 1; }
PROP_ONE=2048,10 timeout -s KILL 90 rocprofv3 --pmc WRITE_SIZE --kernel-include-regex "k_propagate" -d $OUT/write -o run --output-format csv -- \
    python3 tools/prop_sweep.py > $OUT/write.log 2>&1 || { tail -20 $OUT/write.log; exit 1; }
