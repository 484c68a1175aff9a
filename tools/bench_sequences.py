"""SURVEY config 4 ("all 11 EuRoC sequences batched"), on synthetic streams of
the same shape (EuRoC is not reachable here): S stereo+IMU sequences replayed
through ONE device context by the multi-sequence scheduler
(msckf_amd.scheduler.MultiMSCKF), against the same S sequences replayed one
after another through the single-filter drop-in class.  Prints one JSON line:
frames/s of both, the batched launch counts, and ATE vs ground truth.  The
replayed messages (the front-end's output) are built before both timed
regions.

    python tools/bench_sequences.py [--seqs 11] [--frames 200] [--fp32]
    python -m torch.distributed.run --nproc-per-node N --master-addr 127.0.0.1 \
        tools/bench_sequences.py --seqs 11      # sequences dealt round-robin over N GPUs

On N GPUs every rank replays its share of the sequences (replicas.shard) on
its own device; the replicas' host TCP hub (msckf_amd.replicas, no RCCL:
no data crosses GPUs) carries only the barriers, the max of the elapsed time
and the sum of the frame counts (SURVEY config 4: no cross-GPU state).
"""
import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import msckf_pkg  # noqa: E402,F401
import msckf_amd  # noqa: E402
from msckf_amd import synth, replicas  # noqa: E402
from msckf_amd.replay import FeatureStream, replay  # noqa: E402
from msckf_amd.scheduler import MultiMSCKF  # noqa: E402
from msckf_amd.trajectory import ate  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--seqs", type=int, default=11)
    ap.add_argument("--frames", type=int, default=200)
    ap.add_argument("--fp32", action="store_true")
    ap.add_argument("--no-single", action="store_true")
    a = ap.parse_args()
    dtype = np.float32 if a.fp32 else np.float64
    grp = replicas.init()
    mine = replicas.shard(list(range(a.seqs)), grp.rank, grp.world)
    streams = [FeatureStream.from_synthetic(synth.make_sequence(a.frames, 100 + i)) for i in mine]
    n_frames = sum(s.n_frames for s in streams)
    multi = MultiMSCKF(len(streams), dtype=dtype, device=grp.local_rank) if streams else None
    # the messages are the front-end's output: built before either timed
    # region (as the bench's ATE leg does), fresh objects for each run
    msgs = [s.messages() for s in streams]
    grp.barrier()
    t0 = time.perf_counter()
    trajs = multi.run_streams(streams, messages=msgs) if multi else []
    el_b = grp.max_over_ranks(time.perf_counter() - t0)
    total_frames = grp.sum_over_ranks(n_frames)
    launches = dict(multi.launches) if multi else {}
    if multi:
        multi.close()
    out = {"config": "SURVEY config 4 shape: %d synthetic stereo+IMU sequences x %d frames, %s, %d GPU(s)"
                     % (a.seqs, a.frames, "fp32" if a.fp32 else "fp64", grp.world),
           "batched_frames_per_s": round(total_frames / el_b, 1), "batched_s": round(el_b, 2),
           "batched_launches_rank0": launches,
           "ate_vs_gt_m_rank0": [round(ate(t, s.gt), 5) for t, s in zip(trajs, streams)]}
    if not a.no_single and grp.world == 1:
        evs = [s.events() for s in streams]
        t0 = time.perf_counter()
        for s, ev in zip(streams, evs):
            flt = msckf_amd.MSCKF(dtype=dtype)
            replay(flt, s, events=ev)
            flt.close()
        el_s = time.perf_counter() - t0
        out["single_frames_per_s"] = round(n_frames / el_s, 1)
        out["single_s"] = round(el_s, 2)
        out["speedup"] = round(el_s / el_b, 2)
    if grp.rank != 0:
        grp.close()
        return
    print(json.dumps(out), flush=True)
    grp.close()


if __name__ == "__main__":
    main()
