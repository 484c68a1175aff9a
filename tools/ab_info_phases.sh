mkdir -p gpurun_out/ab
B="python -u bench.py --no-cpu --no-ate --no-prop --steps 5"
for ph in 0 1 2 3; do MSCKF_INFO_PHASES=$ph timeout -k 10 200 $B > gpurun_out/ab/info$ph.json 2>/dev/null || exit 1; done
