# s4 debug dump, gate phase probe after the chi2 prefetch, fp32 bench (no CPU/ATE legs)
set -o pipefail
OUT=gpurun_out/r03d; mkdir -p $OUT
timeout -k 10 120 python -u tools/debug/dump_s4.py > $OUT/dump.log 2>&1
timeout -k 10 120 python -u tools/probes/gate_phases.py > $OUT/phases32.json 2>&1 &&
timeout -k 10 300 python -u bench.py --no-cpu --no-ate --no-fp64 > $OUT/b.json 2> $OUT/b.err
