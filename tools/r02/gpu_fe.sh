# GPU front-end tests only.
set -o pipefail
OUT=gpurun_out/${1:-r02fe}
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests/test_gpu_frontend.py -m gpu -v --timeout 300 --timeout-method thread > $OUT/t.log 2>&1
