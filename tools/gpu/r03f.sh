# resident-gate phase probe, GPU suite (async C-ABI), per-frame profile + its kernel trace
set -o pipefail
OUT=gpurun_out/r03f; mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 120 python -u tools/probes/gate_phases.py > $OUT/phases32.json 2>&1
timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread > $OUT/t.log 2>&1
timeout -k 10 120 python -u tools/profile_frame.py > $OUT/frame.json 2>&1
timeout -k 10 120 python -u tools/profile_frame.py --cprofile > $OUT/frame_cprof.txt 2>&1
timeout -k 10 180 rocprofv3 --kernel-trace --stats -d $OUT/frame_trace -o run --output-format csv -- python3 tools/profile_frame.py > $OUT/frame_trace.log 2>&1
tail -3 $OUT/t.log; cat $OUT/frame.json
