set -o pipefail
mkdir -p gpurun_out/dbg2
timeout -k 10 120 python -u tools/debug/degen.py > gpurun_out/dbg2/fused.log 2>&1; echo "== fused"; cat gpurun_out/dbg2/fused.log
timeout -k 10 120 python -u tools/debug/degen.py tools/exp/libmsckf_rec.so > gpurun_out/dbg2/rec.log 2>&1; echo "== records"; cat gpurun_out/dbg2/rec.log
