set -o pipefail
OUT=gpurun_out/r04h; mkdir -p $OUT
timeout -k 10 300 python -u tools/probes/info_phases.py > $OUT/info_phases.json 2> $OUT/err.log || { tail -20 $OUT/err.log; exit 1; }
cat $OUT/info_phases.json
