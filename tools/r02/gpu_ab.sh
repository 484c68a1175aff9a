# GPU parity suite, the fp32 bench with and without the filter-resident gate,
# and one SQ counter pass of the gating kernels for each.
set -o pipefail
OUT=gpurun_out/${1:-r02d}
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $OUT/t.log 2>&1 &&
timeout -k 10 300 python -u bench.py --no-cpu --no-ate --no-fp64 --no-prop > $OUT/b32.json 2> $OUT/b32.err &&
MSCKF_GATE_RES=0 timeout -k 10 300 python -u bench.py --no-cpu --no-ate --no-fp64 --no-prop > $OUT/b32_old.json 2> $OUT/b32_old.err || exit 1
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
CTR="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_MFMA SQ_LDS_BANK_CONFLICT"
for r in 1 0; do
  MSCKF_GATE_RES=$r timeout -s KILL 90 rocprofv3 --pmc $CTR --kernel-include-regex "k_gate" -d $OUT/pmc_res$r -o run --output-format csv -- \
      python3 bench.py --steps 1 --warmup 0 --no-cpu --no-ate --no-prop --no-fp64 > $OUT/pmc_res$r.log 2>&1 || exit 1
done
