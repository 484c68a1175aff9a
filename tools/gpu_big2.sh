# GPU parity tests, then SURVEY configs 3 and 5
set -o pipefail
mkdir -p gpurun_out/big
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/t.log 2>&1 &&
timeout -k 10 200 python -u bench.py --N 50 --F 400 --batch 512 --no-cpu --no-ate --no-prop > gpurun_out/big/b50.json 2> gpurun_out/big/b.err &&
timeout -k 10 200 python -u bench.py --N 80 --F 1000 --batch 128 --no-cpu --no-ate --no-prop > gpurun_out/big/b80.json 2>> gpurun_out/big/b.err
