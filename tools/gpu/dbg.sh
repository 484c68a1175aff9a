set -o pipefail
mkdir -p gpurun_out/dbg
timeout -k 10 300 python -u "$@" > gpurun_out/dbg/out.log 2>&1; rc=$?; tail -60 gpurun_out/dbg/out.log; exit $rc
