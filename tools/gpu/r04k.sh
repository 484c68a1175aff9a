# Gate: parity + A/B vs the previous commit's gate + SQ counters.
set -o pipefail
OUT=gpurun_out/r04k; mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 200 --timeout-method thread  > $OUT/t.log 2>&1 || { tail -30 $OUT/t.log; exit 1; }
tail -2 $OUT/t.log
bash tools/gpu/exp.sh r04k/ab1 old || exit 1
bash tools/gpu/exp.sh r04k/ab2 old || exit 1
bash tools/gpu/sq.sh r04k/sq "k_gate" || exit 1
python3 tools/pmc_sq.py gpurun_out/r04k/sq/sq/run_counter_collection.csv > gpurun_out/r04k/sq.txt 2>&1
cat gpurun_out/r04k/sq.txt
