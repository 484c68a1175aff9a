set -o pipefail
OUT=gpurun_out/r04c; mkdir -p $OUT
timeout -k 10 300 python -u tools/debug/s4_frame3.py > $OUT/s4.log 2>&1; rc=$?; tail -60 $OUT/s4.log; [ $rc -eq 0 ] || exit $rc
bash tools/gpu/exp.sh r04c/ab rec || exit 1
timeout -k 10 400 python -u -m pytest tests/test_gpu_replicas.py tests/test_gpu_frontend.py -m gpu -v -s --timeout 200 --timeout-method thread > $OUT/t.log 2>&1 || { tail -40 $OUT/t.log; exit 1; }
grep -E "ids identical|passed|failed" $OUT/t.log | tail -6
