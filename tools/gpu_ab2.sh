# GPU check + in-call A/B of a runtime switch ($1=VAR, $2=value for the B leg)
set -o pipefail
mkdir -p gpurun_out/ab
B="python -u bench.py --no-cpu --no-ate --no-prop"
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/t.log 2>&1 &&
timeout -k 10 300 $B > gpurun_out/ab/a1.json 2> gpurun_out/b.err &&
env $1=$2 timeout -k 10 300 $B > gpurun_out/ab/b1.json 2>> gpurun_out/b.err &&
timeout -k 10 300 $B > gpurun_out/ab/a2.json 2>> gpurun_out/b.err &&
env $1=$2 timeout -k 10 300 $B > gpurun_out/ab/b2.json 2>> gpurun_out/b.err
