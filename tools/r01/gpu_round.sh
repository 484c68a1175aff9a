set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/t1.log 2>&1 &&
timeout -k 10 200 python -u bench.py > gpurun_out/b1.json 2> gpurun_out/b1.err &&
timeout -k 10 200 python -u bench.py --N 50 --F 400 --batch 512 --no-cpu > gpurun_out/b1_50.json 2>> gpurun_out/b1.err &&
bash tools/profile_round.sh r01v6 3
