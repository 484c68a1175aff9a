# GPU round check: parity tests, then the default bench line.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/t.log 2>&1 &&
timeout -k 10 300 python -u bench.py > gpurun_out/b.json 2> gpurun_out/b.err
