# Round-end check: parity tests, smoke, the default bench line
set -o pipefail
mkdir -p gpurun_out/final
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/final/t.log 2>&1 &&
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/final/smoke.log 2>&1 &&
timeout -k 10 300 python -u bench.py > gpurun_out/final/bench.json 2> gpurun_out/final/bench.err
