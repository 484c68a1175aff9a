# small-batch split of Kalman B / C2 / E: parity, then per-frame A/B (env switch, same library)
set -o pipefail
OUT=gpurun_out/r04x; mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 200 --timeout-method thread -k "update or batched or cholesky or sequence" > $OUT/t.log 2>&1 || { tail -30 $OUT/t.log; exit 1; }
tail -2 $OUT/t.log
for i in 1 2; do
  for sp in 0 1; do
    MSCKF_KAL_SPLIT=$sp timeout -k 10 300 python -u tools/profile_frame.py > $OUT/frame_s${sp}_$i.json 2> $OUT/frame_s${sp}_$i.err || { tail -20 $OUT/frame_s${sp}_$i.err; exit 1; }
    echo "split=$sp run $i: $(tail -c 400 $OUT/frame_s${sp}_$i.json)"
  done
done
