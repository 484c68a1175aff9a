# Round-4 first check: the whole GPU suite (with the s4 print), then the default bench.
set -o pipefail
OUT=gpurun_out/r04a; mkdir -p $OUT
timeout -k 10 900 python -u -m pytest tests -m gpu -v -s --timeout 300 --timeout-method thread > $OUT/gpu_tests.log 2>&1 || { grep -E "s4:|FAIL|Error|assert" $OUT/gpu_tests.log | head -40; tail -40 $OUT/gpu_tests.log; exit 1; }
grep -E "s4:|passed|failed" $OUT/gpu_tests.log | tail -5
timeout -k 10 600 python -u bench.py > $OUT/bench.json 2> $OUT/bench.err || { tail -20 $OUT/bench.err; exit 1; }
tail -c 1500 $OUT/bench.json
