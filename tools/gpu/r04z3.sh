# gather kernel + single propagate upload + resident identity lists: GPU suite, then per-frame A/B vs the
# build before the gather change (old), 4 alternations, 400 frames
set -o pipefail
OUT=gpurun_out/r04z3; mkdir -p $OUT
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > $OUT/t.log 2>&1 || { tail -30 $OUT/t.log; exit 1; }
tail -2 $OUT/t.log
for i in 1 2 3 4; do
  timeout -k 10 300 python -u tools/exp_frame.py tools/exp/libmsckf_old.so --frames 400 > $OUT/old_$i.json 2> $OUT/old_$i.err || { tail -20 $OUT/old_$i.err; exit 1; }
  timeout -k 10 300 python -u tools/profile_frame.py --frames 400 > $OUT/new_$i.json 2> $OUT/new_$i.err || { tail -20 $OUT/new_$i.err; exit 1; }
done
for f in $OUT/new_*.json $OUT/old_*.json; do python3 -c "import json; d=json.loads(open('$f').read().strip().splitlines()[-1]); print('$f', d['frames_per_s'], d['device_requests_ms_per_frame']['states'], d['host_ms_per_frame'])"; done
