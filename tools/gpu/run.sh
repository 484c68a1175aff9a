# One parameterised GPU session (run on the box from the repo root through
# gpurun).  Every step runs under its own time limit; the first failing step
# ends the session (no GPU work after a fault, abort or time-out).
#   bash tools/gpu/run.sh TAG step [step ...]
# steps:
#   tests          the whole -m gpu suite
#   tests:EXPR     the -m gpu tests matching -k EXPR
#   smoke          __graft_entry__.smoke()
#   bench          the default bench line (every leg)
#   quick          the headline leg only (no CPU / ATE / propagation / fp64)
#   b50 / b80      configs 3 / 5 (fp32), b50d / b80d the same in fp64
#   stats          rocprofv3 kernel-trace stats of a short fp32 bench
#   sq             SQ counters of the hot kernels (one fp32 step)
#   pmc            FETCH_SIZE / WRITE_SIZE passes (tools/profile_round.sh)
#   pmc50 / pmc50d / pmc80   the same (+ kernel stats) at 50x400 fp32 / fp64, 80x1000 fp32
#   seq            the 11-lane scheduler vs single filters (tools/bench_sequences.py)
#   frame          the drop-in per-frame path (tools/profile_frame.py)
#   prop           the propagation sweep + kernel stats (tools/gpu/prop.sh)
set -o pipefail
TAG=$1; shift
OUT=gpurun_out/$TAG; mkdir -p $OUT
NB="--no-cpu --no-ate --no-prop"
run() {   # run NAME SECONDS cmd...  (stdout -> NAME.out, stderr -> NAME.err)
  local name=$1 secs=$2; shift 2
  timeout -k 10 $secs "$@" > $OUT/$name.out 2> $OUT/$name.err
  local rc=$?
  if [ $rc -ne 0 ]; then echo "step $name failed rc=$rc"; tail -30 $OUT/$name.out; tail -30 $OUT/$name.err; exit $rc; fi
}
line() { python3 -c "
import json,sys; d=json.loads(open('$OUT/$1.out').read().strip().splitlines()[-1])
print('$1', d['value'], d['ms_per_step'], 'frac', d['roofline']['frac'], d.get('kernel_ms_per_step'))"; }
for step in "$@"; do
  case $step in
    tests) run tests 900 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread; tail -2 $OUT/tests.out ;;
    tests:*) run tests_k 600 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread -k "${step#tests:}"; tail -2 $OUT/tests_k.out ;;
    smoke) run smoke 300 python -u -c "import __graft_entry__ as g; g.smoke()"; tail -1 $OUT/smoke.out ;;
    bench) run bench 600 python -u bench.py; line bench ;;
    quick) run quick 300 python -u bench.py $NB --no-fp64; line quick ;;
    b50) run b50 600 python -u bench.py --N 50 --F 400 $NB --no-fp64; line b50 ;;
    b80) run b80 600 python -u bench.py --N 80 --F 1000 --batch 512 $NB --no-fp64; line b80 ;;
    b50d) run b50d 600 python -u bench.py --N 50 --F 400 --dtype fp64 $NB; line b50d ;;
    b80d) run b80d 600 python -u bench.py --N 80 --F 1000 --dtype fp64 --batch 512 $NB; line b80d ;;
    stats) bash tools/gpu/stats.sh $TAG/st --no-fp64 || exit 1 ;;
    sq) bash tools/gpu/sq.sh $TAG/sq "k_gate|k_info|k_kal|k_feature|k_prop|k_triang" || exit 1 ;;
    pmc) bash tools/profile_round.sh $TAG 3 || exit 1 ;;
    pmc50) bash tools/profile_round.sh ${TAG}_50x400 2 --N 50 --F 400 --no-fp64 || exit 1 ;;
    pmc50d) bash tools/profile_round.sh ${TAG}_50x400_fp64 2 --N 50 --F 400 --dtype fp64 || exit 1 ;;
    pmc80) bash tools/profile_round.sh ${TAG}_80x1000 2 --N 80 --F 1000 --batch 512 --no-fp64 || exit 1 ;;
    seq) run seq 600 python -u tools/bench_sequences.py --seqs 11; tail -c 400 $OUT/seq.out ;;
    frame) run frame 300 python -u tools/profile_frame.py; tail -c 300 $OUT/frame.out ;;
    prop) bash tools/gpu/prop.sh $TAG/prop || exit 1 ;;
    *) echo "unknown step $step"; exit 2 ;;
  esac
done
