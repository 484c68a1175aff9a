# SQ counters of k_propagate on one 2048-filter x 10-sample launch (tools/prop_sweep.py
# PROP_ONE mode), one rocprofv3 pass per counter set; summarise with tools/pmc_sq.py.
set -o pipefail
OUT=gpurun_out/pmc_prop_${1:-x}
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
export PROP_ONE=2048,10
SETS=("SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS"
      "SQ_WAVES SQ_INSTS_VMEM_RD SQ_INSTS_SALU SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INSTS_BRANCH SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT")
i=0
for ctr in "${SETS[@]}"; do
  i=$((i+1))
  timeout -s KILL 90 rocprofv3 --pmc $ctr --kernel-include-regex k_propagate -d $OUT/p_$i -o run --output-format csv -- \
      python3 tools/prop_sweep.py ${2:-} > $OUT/p_$i.log 2>&1 || exit 1
done
