# Kalman stage A inline on the main stream (serial) vs on the side stream beside k_feature
set -o pipefail
bash tools/gpu/exp.sh r04ac/ab1 ainl || exit 1
bash tools/gpu/exp.sh r04ac/ab2 ainl || exit 1
for f in gpurun_out/r04ac/ab*/*.json; do python3 -c "import json; d=json.loads(open('$f').read().strip().splitlines()[-1]); k=d['kernel_ms_per_step']; print('$f', d['ms_per_step'], k['feature_jacobian'], k['kalman_a'], k['compress'])"; done
