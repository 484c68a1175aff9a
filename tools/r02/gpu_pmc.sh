# SQ counter passes over the kernels matching $2 (default: everything msckf) of the fp32 bench.
set -o pipefail
OUT=gpurun_out/${1:-r02i}; RE=${2:-msckf}
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
SETS=("SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_MFMA"
      "SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_TRANS_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_SALU SQ_ACTIVE_INST_VALU SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_VMEM_RD")
i=0
for ctr in "${SETS[@]}"; do
  i=$((i+1))
  timeout -s KILL 90 rocprofv3 --pmc $ctr --kernel-include-regex "$RE" -d $OUT/p$i -o run --output-format csv -- \
      python3 bench.py --steps 1 --warmup 0 --no-cpu --no-ate --no-prop --no-fp64 > $OUT/p$i.log 2>&1 || exit 1
done
