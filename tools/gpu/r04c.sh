set -o pipefail
OUT=gpurun_out/r04c; mkdir -p $OUT
timeout -k 10 300 python -u tools/debug/s4_frame3.py > $OUT/s4.log 2>&1; rc=$?; tail -80 $OUT/s4.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u -m pytest tests/test_gpu_replicas.py -m gpu -x -v --timeout 200 --timeout-method thread > $OUT/t.log 2>&1 || { tail -40 $OUT/t.log; exit 1; }
tail -3 $OUT/t.log
