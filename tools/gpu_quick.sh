# GPU parity tests + two default bench runs (gate time of the current build)
set -o pipefail
mkdir -p gpurun_out/q
B="python -u bench.py --no-cpu --no-ate --no-prop"
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/t.log 2>&1 &&
timeout -k 10 300 $B > gpurun_out/q/a.json 2> gpurun_out/q/b.err &&
timeout -k 10 300 $B > gpurun_out/q/b.json 2>> gpurun_out/q/b.err &&
timeout -k 10 200 python -u bench.py --N 80 --F 1000 --batch 128 --no-cpu --no-ate --no-prop > gpurun_out/q/b80.json 2>> gpurun_out/q/b.err
