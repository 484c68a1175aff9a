# Kalman stage A forked after the gate (beside select + compress) vs before k_feature
set -o pipefail
bash tools/gpu/exp.sh r04ab/ab1 alate || exit 1
bash tools/gpu/exp.sh r04ab/ab2 alate || exit 1
for f in gpurun_out/r04ab/ab*/*.json; do python3 -c "import json; d=json.loads(open('$f').read().strip().splitlines()[-1]); k=d['kernel_ms_per_step']; print('$f', d['ms_per_step'], k['feature_jacobian'], k['kalman_a'], k['compress'])"; done
