# A/B of the gating Y-staging budget (MSCKF_GATE_SPKB: multi-pass below it)
set -o pipefail
mkdir -p gpurun_out/ab
B="python -u bench.py --no-cpu --no-ate --no-prop"
for v in ${SPKB_LIST:-28 20 12 28 20 12}; do
  MSCKF_GATE_SPKB=$v timeout -k 10 300 $B > gpurun_out/ab/s$v.json 2>> gpurun_out/b.err || exit 1
  python -c "import json; d=json.load(open('gpurun_out/ab/s$v.json')); print($v, d['value'], d['kernel_ms_per_step']['gate'])" >> gpurun_out/ab/spkb.txt
done
