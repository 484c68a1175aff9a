# Gate P-block loads with uniform row bases (saddr): parity, A/B vs the previous gate.
set -o pipefail
OUT=gpurun_out/r04r; mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 200 --timeout-method thread -k "gate or update or batched" > $OUT/t.log 2>&1 || { tail -30 $OUT/t.log; exit 1; }
tail -2 $OUT/t.log
bash tools/gpu/exp.sh r04r/ab1 old || exit 1
bash tools/gpu/exp.sh r04r/ab2 old || exit 1
