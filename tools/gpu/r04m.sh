# Propagation split (k_propagate serial chain + k_prop_cross streaming): parity, sweep, stats, bench leg.
set -o pipefail
OUT=gpurun_out/r04m; mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 200 --timeout-method thread -k "propagat or sequence or augment or config4" > $OUT/t.log 2>&1 || { tail -30 $OUT/t.log; exit 1; }
tail -2 $OUT/t.log
bash tools/gpu/prop.sh r04m/prop || exit 1
timeout -k 10 300 python -u bench.py --no-cpu --no-ate --no-fp64 > $OUT/bench.json 2> $OUT/bench.err || { tail -20 $OUT/bench.err; exit 1; }
python3 -c "import json; d=json.loads(open('$OUT/bench.json').read().strip().splitlines()[-1]); print(d['value'], d['ms_per_step'], json.dumps(d['propagation']))"
timeout -k 10 300 python -u tools/profile_frame.py > $OUT/frame.json 2> $OUT/frame.err || { tail -20 $OUT/frame.err; exit 1; }
cat $OUT/frame.json
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/fstats -o run --output-format csv -- python3 tools/profile_frame.py --frames 100 > $OUT/fstats.log 2>&1 || { tail -20 $OUT/fstats.log; exit 1; }
