# GPU check + A/B: parity tests, the default bench, the gating phases alone
# (MSCKF_GATE_PHASES), and a kernel-trace profile of the default bench.
set -o pipefail
mkdir -p gpurun_out/ab
B="python -u bench.py --no-cpu --no-ate --no-prop"
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/t.log 2>&1 &&
timeout -k 10 300 python -u bench.py --no-cpu --no-ate > gpurun_out/b.json 2> gpurun_out/b.err &&
MSCKF_GATE_PHASES=1 timeout -k 10 300 $B > gpurun_out/ab/y.json 2>> gpurun_out/b.err &&
MSCKF_GATE_PHASES=4 timeout -k 10 300 $B > gpurun_out/ab/elim.json 2>> gpurun_out/b.err &&
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/ab/prof -o run --output-format csv -- \
    python3 bench.py --steps 3 --warmup 1 --no-cpu --no-ate --no-prop > gpurun_out/ab/prof.log 2>&1
