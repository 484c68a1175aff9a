# Round profile: default bench line (CPU baseline, ATE, propagation legs), the
# SURVEY config 3 / 5 bench lines, kernel-trace stats and FETCH/WRITE passes.
set -o pipefail
mkdir -p gpurun_out/v11
timeout -k 10 300 python -u bench.py > gpurun_out/v11/bench.json 2> gpurun_out/v11/bench.err &&
timeout -k 10 200 python -u bench.py --N 50 --F 400 --batch 512 --no-cpu --no-ate --no-prop > gpurun_out/v11/bench_50x400.json 2>> gpurun_out/v11/bench.err &&
timeout -k 10 200 python -u bench.py --N 80 --F 1000 --batch 128 --no-cpu --no-ate --no-prop > gpurun_out/v11/bench_80x1000.json 2>> gpurun_out/v11/bench.err &&
bash tools/profile_round.sh r01v11 3 &&
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/v11/smoke.log 2>&1 &&
bash tools/pmc_gate.sh
