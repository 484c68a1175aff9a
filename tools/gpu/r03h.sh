# Kalman stages A / C1 on MFMA: parity tests first, then the bench and kernel stats
set -o pipefail
OUT=gpurun_out/r03h; mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -x -v --timeout 200 --timeout-method thread -k "batched or update or sequence or degenerate" > $OUT/t_kal.log 2>&1 || { tail -30 $OUT/t_kal.log; exit 1; }
timeout -k 10 300 python -u bench.py --no-cpu --no-ate > $OUT/b.json 2> $OUT/b.err
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/stats -o run --output-format csv -- python3 bench.py --steps 3 --warmup 1 --no-cpu --no-ate --no-prop > $OUT/stats.log 2>&1
tail -3 $OUT/t_kal.log
