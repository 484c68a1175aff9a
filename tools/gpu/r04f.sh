# Round-4 profiles: kernel-trace stats, FETCH / WRITE passes (pmc summary), SQ counters.
set -o pipefail
bash tools/profile_round.sh r04 3 || exit 1
bash tools/gpu/sq.sh r04f/sq "k_gate|k_info|k_kal|k_feature" || exit 1
python3 tools/pmc_sq.py gpurun_out/r04f/sq/sq/run_counter_collection.csv > gpurun_out/r04f/sq.txt 2>&1
python3 tools/pmc_summary.py gpurun_out/prof_r04/fetch/run_counter_collection.csv gpurun_out/prof_r04/write/run_counter_collection.csv --dtype fp32 --source "profiles/r04 v2 passes" -o gpurun_out/r04f/pmc_summary.json > gpurun_out/r04f/pmc.log 2>&1
tail -5 gpurun_out/r04f/pmc.log; cat gpurun_out/r04f/sq.txt
