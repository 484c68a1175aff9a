# counter names, resident-gate probe with the raw fetch latency, SQ pass over k_gate_res
set -o pipefail
OUT=gpurun_out/r03g; mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 60 rocprofv3 -L > $OUT/counters.txt 2>&1
grep -i -E "icache|sqc|ifetch|inst|utcl|tlb" $OUT/counters.txt > $OUT/counters_sel.txt
timeout -k 10 120 python -u tools/probes/gate_phases.py > $OUT/phases32.json 2>&1
CTR="SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS"
timeout -s KILL 90 rocprofv3 --pmc $CTR --kernel-include-regex "k_gate" -d $OUT/sq -o run --output-format csv -- \
    python3 bench.py --steps 1 --warmup 0 --no-cpu --no-ate --no-prop --no-fp64 > $OUT/sq.log 2>&1
python3 tools/pmc_sq.py $OUT/sq/run_counter_collection.csv > $OUT/sq.txt 2>&1
cat $OUT/sq.txt
