set -o pipefail
OUT=gpurun_out/r04i; mkdir -p $OUT
timeout -k 10 300 python -u tools/probes/info_phases.py > $OUT/info_phases.json 2> $OUT/err.log || { tail -20 $OUT/err.log; exit 1; }
cat $OUT/info_phases.json
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 200 --timeout-method thread -k "batched or update_golden or sequence or degenerate" > $OUT/t.log 2>&1 || { tail -30 $OUT/t.log; exit 1; }
tail -2 $OUT/t.log
bash tools/gpu/exp.sh r04i/ab f1 || exit 1
