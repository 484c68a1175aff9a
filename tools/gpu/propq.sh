# Propagation check: parity tests, the sweep + kernel stats, the SQ / traffic passes
#   bash tools/gpu/propq.sh TAG
set -o pipefail
TAG=${1:-prop}; OUT=gpurun_out/$TAG; mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread -k "propagate or sequence or augment" > $OUT/t.log 2>&1 || { tail -30 $OUT/t.log; exit 1; }
tail -1 $OUT/t.log
bash tools/gpu/prop.sh $TAG/prop > $OUT/prop.txt || { cat $OUT/prop.txt; exit 1; }
tail -4 $OUT/prop.txt
bash tools/gpu/prop_pmc.sh $TAG/pmc || exit 1
python3 tools/pmc_sq.py $OUT/pmc/sq/run_counter_collection.csv
