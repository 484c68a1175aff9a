# Stage A as a persistent grid (256 / 512 workgroups) beside k_feature / the gate.
set -o pipefail
OUT=gpurun_out/r04p; mkdir -p $OUT
bash tools/gpu/exp.sh r04p/ab1 ag256 ag512 || exit 1
bash tools/gpu/exp.sh r04p/ab2 ag256 ag512 || exit 1
