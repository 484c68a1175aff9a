# Round-4: fused information assembly -- update parity tests, then A/B against the record path.
set -o pipefail
OUT=gpurun_out/r04b; mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -v -s --timeout 200 --timeout-method thread -k "update or batched or sequence or gate or restore or corrupted" > $OUT/t.log 2>&1 || { grep -E "s4:|FAIL|Error|assert" $OUT/t.log | head -30; tail -30 $OUT/t.log; exit 1; }
grep -E "s4:|passed|failed" $OUT/t.log | tail -5
bash tools/gpu/exp.sh r04b/ab rec
