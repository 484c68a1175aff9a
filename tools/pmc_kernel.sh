# SQ counters of one kernel family (regex $1) over the default bench, one
# rocprofv3 pass per counter set; summarise with tools/pmc_gate_sum.py <dir> <regex>.
set -o pipefail
RE=${1:-k_info}; OUT=gpurun_out/pmc_$2
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
SETS=("SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS"
      "SQ_INSTS_VMEM_RD SQ_INSTS_SALU SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INST_CYCLES_VMEM_RD SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_MFMA SQ_LDS_BANK_CONFLICT")
i=0
for ctr in "${SETS[@]}"; do
  i=$((i+1))
  timeout -s KILL 90 rocprofv3 --pmc $ctr --kernel-include-regex "$RE" -d $OUT/ph7_$i -o run --output-format csv -- \
      python3 bench.py --steps 1 --warmup 0 --no-cpu --no-ate --no-prop > $OUT/ph7_$i.log 2>&1 || exit 1
done
