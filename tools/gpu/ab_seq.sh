# Same-box A/B of the multi-sequence scheduler (tools/bench_sequences.py, 11
# lanes x 200 frames, fp64) across package builds: each tools/exp/pkg_<name>
# (a copy of the package with its own libmsckf_hip.so, e.g. an earlier
# round's) and the working tree ("head"), alternated R times.
#   bash tools/gpu/ab_seq.sh TAG R name [name ...]
set -o pipefail
OUT=gpurun_out/$1; R=$2; shift 2; mkdir -p $OUT
for rep in $(seq 1 $R); do
  for name in head "$@"; do
    if [ $name = head ]; then
      timeout -k 10 300 python -u tools/bench_sequences.py --seqs 11 > $OUT/${name}_$rep.json 2> $OUT/${name}_$rep.err || { tail -20 $OUT/${name}_$rep.err; exit 1; }
    else
      timeout -k 10 300 python -u tools/exp/run_pkg.py tools/exp/pkg_$name tools/bench_sequences.py --seqs 11 \
        > $OUT/${name}_$rep.json 2> $OUT/${name}_$rep.err || { tail -20 $OUT/${name}_$rep.err; exit 1; }
    fi
    python3 -c "import json; d=json.loads(open('$OUT/${name}_$rep.json').read().strip().splitlines()[-1]); print('$name', $rep, d['batched_frames_per_s'], d['single_frames_per_s'], d['speedup'])"
  done
done
