# Kalman A / C1 on fp64 MFMA (k_kal_mchol): parity, A/B against the register tiles and NW = 16.
set -o pipefail
OUT=gpurun_out/r04l; mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 200 --timeout-method thread > $OUT/t.log 2>&1 || { tail -30 $OUT/t.log; exit 1; }
tail -2 $OUT/t.log
bash tools/gpu/exp.sh r04l/ab1 rchol || exit 1
bash tools/gpu/exp.sh r04l/ab2 rchol || exit 1
bash tools/gpu/sq.sh r04l/sq "k_kal" || exit 1
python3 tools/pmc_sq.py gpurun_out/r04l/sq/sq/run_counter_collection.csv > gpurun_out/r04l/sq.txt 2>&1
cat gpurun_out/r04l/sq.txt
