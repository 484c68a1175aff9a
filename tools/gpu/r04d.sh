# Round 4: fused-assembly A/B + SQ counters of both assembly kernels, the s4 test, RCCL / front-end tests.
set -o pipefail
OUT=gpurun_out/r04d; mkdir -p $OUT
bash tools/gpu/exp.sh r04d/ab f0 rec || exit 1
bash tools/gpu/sq.sh r04d/sq_fused "k_info|k_feature" || exit 1
timeout -k 10 120 python3 tools/pmc_sq.py gpurun_out/r04d/sq_fused/sq/run_counter_collection.csv > $OUT/sq_fused.txt 2>&1; cat $OUT/sq_fused.txt
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
CTR="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_MFMA SQ_LDS_BANK_CONFLICT"
timeout -s KILL 90 rocprofv3 --pmc $CTR --kernel-include-regex "k_info|k_feature" -d $OUT/sq_rec/sq -o run --output-format csv -- \
    python3 tools/exp_bench.py tools/exp/libmsckf_rec.so --steps 1 --warmup 0 --no-cpu --no-ate --no-prop --no-fp64 > $OUT/sq_rec.log 2>&1 || exit 1
timeout -k 10 120 python3 tools/pmc_sq.py $OUT/sq_rec/sq/run_counter_collection.csv > $OUT/sq_rec.txt 2>&1; cat $OUT/sq_rec.txt
timeout -k 10 500 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_replicas.py tests/test_gpu_frontend.py -m gpu -v -s --timeout 200 --timeout-method thread -k "s4 or rccl or replica or reference" > $OUT/t.log 2>&1 || { grep -E "s4:|Error|assert" $OUT/t.log | head; tail -30 $OUT/t.log; exit 1; }
grep -E "s4:|ids identical|passed|failed" $OUT/t.log | tail -8
