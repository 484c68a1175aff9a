# Gate staging budget A/B (GATE_SINGLE_KB 44 / 52 / 60), gate tests.
set -o pipefail
OUT=gpurun_out/r04n; mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 200 --timeout-method thread -k "gate or update or batched" > $OUT/t.log 2>&1 || { tail -30 $OUT/t.log; exit 1; }
tail -2 $OUT/t.log
bash tools/gpu/exp.sh r04n/ab1 kb52 kb60 aearly || exit 1
bash tools/gpu/exp.sh r04n/ab2 kb52 kb60 aearly || exit 1
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 200 --timeout-method thread -k "cholesky_paths or sequence_s1" > $OUT/t2.log 2>&1 || { tail -30 $OUT/t2.log; exit 1; }
tail -2 $OUT/t2.log
timeout -k 10 300 python -u tools/probes/gate_phases.py > $OUT/gate_phases.json 2> $OUT/gp.err || { tail -20 $OUT/gp.err; exit 1; }
cat $OUT/gate_phases.json
