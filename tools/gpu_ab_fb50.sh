# A/B of k_info's staged features per batch at SURVEY config 3 (MSCKF_INFO_FB)
set -o pipefail
mkdir -p gpurun_out/ab
B="python -u bench.py --N 50 --F 400 --batch 512 --no-cpu --no-ate --no-prop"
for v in 2 3 4 2 3 4; do
  MSCKF_INFO_FB=$v timeout -k 10 300 $B > gpurun_out/ab/fb50_$v.json 2>> gpurun_out/b.err || exit 1
  python -c "import json; d=json.load(open('gpurun_out/ab/fb50_$v.json')); print($v, d['value'], d['kernel_ms_per_step']['compress'])" >> gpurun_out/ab/fb50.txt
done
