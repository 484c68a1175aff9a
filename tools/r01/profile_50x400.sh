set -o pipefail
mkdir -p gpurun_out/p50
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/p50 -o run --output-format csv -- python3 bench.py --N 50 --F 400 --batch 512 --steps 2 --warmup 1 --no-cpu --no-ate --no-prop > gpurun_out/p50/log 2>&1
