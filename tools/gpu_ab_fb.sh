# A/B of k_info's staged features per batch (MSCKF_INFO_FB)
set -o pipefail
mkdir -p gpurun_out/ab
B="python -u bench.py --no-cpu --no-ate --no-prop"
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/t.log 2>&1 || exit 1
for v in 4 5 6 4 5 6; do
  MSCKF_INFO_FB=$v timeout -k 10 300 $B > gpurun_out/ab/fb$v.json 2>> gpurun_out/b.err || exit 1
  python -c "import json; d=json.load(open('gpurun_out/ab/fb$v.json')); print($v, d['value'], d['kernel_ms_per_step']['compress'])" >> gpurun_out/ab/fb.txt
done
