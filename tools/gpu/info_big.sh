set -o pipefail
OUT=gpurun_out/r06/ib; mkdir -p $OUT
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread -k "50x400 or 80x1000 or batched_fp64 or kalman or stage_c or 34 or config4" > $OUT/t.log 2>&1 || { tail -30 $OUT/t.log; exit 1; }; tail -1 $OUT/t.log
bash tools/gpu/ab_env.sh r06/ib/ab50 MSCKF_EXP_OLDINFO_X "0" "--N 50 --F 400 --steps 10" || exit 1
MSCKF_EXP_OLDINFO=1 bash tools/gpu/ab_env.sh r06/ib/ab50_old MSCKF_EXP_OLDINFO_X "0" "--N 50 --F 400 --steps 10" || exit 1
bash tools/gpu/ab_env.sh r06/ib/ab80 MSCKF_EXP_OLDINFO_X "0" "--N 80 --F 1000 --batch 512 --steps 10" || exit 1
