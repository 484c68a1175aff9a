# Round-2 baseline: GPU parity tests, default fp32 bench, fp64 bench at 30x200.
set -o pipefail
mkdir -p gpurun_out/r02a
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/r02a/t.log 2>&1 &&
timeout -k 10 300 python -u bench.py --no-cpu > gpurun_out/r02a/b32.json 2> gpurun_out/r02a/b32.err &&
timeout -k 10 300 python -u bench.py --no-cpu --no-ate --dtype fp64 > gpurun_out/r02a/b64.json 2> gpurun_out/r02a/b64.err
