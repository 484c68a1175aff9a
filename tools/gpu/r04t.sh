# Gate: fp32 NB = 5 class streamed at four waves per SIMD (experiment).
set -o pipefail
OUT=gpurun_out/r04t; mkdir -p $OUT
bash tools/gpu/exp.sh r04t/ab1 st5 || exit 1
bash tools/gpu/exp.sh r04t/ab2 st5 || exit 1
timeout -k 10 600 python -u tools/exp_bench.py tools/exp/libmsckf_st5.so --no-cpu --no-ate --no-prop --no-fp64 --steps 2 > /dev/null 2>&1 || true
