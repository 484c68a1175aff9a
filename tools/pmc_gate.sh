# SQ counters of the fp32 gating kernel (k_gate_mfma), whole and by phase
# (MSCKF_GATE_PHASES: 1 = Y blocks only, 4 = elimination only).  One rocprofv3
# pass per counter set and phase; summarise with tools/pmc_gate_sum.py.
set -o pipefail
mkdir -p gpurun_out/pmc
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
SETS=("SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS"
      "SQ_INSTS_VMEM_RD SQ_INSTS_SALU SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INST_CYCLES_VMEM_RD SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_MFMA SQ_LDS_BANK_CONFLICT")
for ph in 7 1 4; do
  i=0
  for ctr in "${SETS[@]}"; do
    i=$((i+1))
    MSCKF_GATE_PHASES=$ph timeout -s KILL 90 rocprofv3 --pmc $ctr --kernel-include-regex "k_gate" -d gpurun_out/pmc/ph${ph}_$i -o run --output-format csv -- \
        python3 bench.py --steps 1 --warmup 0 --no-cpu --no-ate --no-prop > gpurun_out/pmc/ph${ph}_$i.log 2>&1 || exit 1
  done
done
