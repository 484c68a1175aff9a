# Kalman E: 8 waves x 12 tiles at 4 waves / SIMD (two filters per CU) vs 16 x 6 (one)
set -o pipefail
bash tools/gpu/exp.sh r04aa/ab1 ke8 || exit 1
bash tools/gpu/exp.sh r04aa/ab2 ke8 || exit 1
for f in gpurun_out/r04aa/ab*/*.json; do python3 -c "import json; d=json.loads(open('$f').read().strip().splitlines()[-1]); print('$f', d['kernel_ms_per_step']['kalman_e'])"; done
