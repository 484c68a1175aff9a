# gate-focused tests first (fast fail), then the full GPU suite, then the fp32 bench
set -o pipefail
OUT=gpurun_out/r03e; mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -v --timeout 120 --timeout-method thread -k "gate or batched_fp32" > $OUT/t_gate.log 2>&1
timeout -k 10 300 python -u bench.py --no-cpu --no-ate --no-fp64 > $OUT/b.json 2> $OUT/b.err
timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread > $OUT/t.log 2>&1
tail -3 $OUT/t_gate.log; tail -3 $OUT/t.log
