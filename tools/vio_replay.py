"""Replay a recorded feature stream through the GPU filter and report ATE.

    python tools/vio_replay.py STREAM [--euroc DIR] [--fp32] [--out traj.csv]

STREAM is a replay .npz (msckf_amd.replay.FeatureStream.save) or a directory
holding imu.csv + features.csv.  Ground truth comes from the stream itself or
from an EuRoC sequence directory (--euroc, mav0/state_groundtruth_estimate0).
A synthetic stream can be written with --make-synthetic N_FRAMES SEED.
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
from msckf_amd import synth  # noqa: E402
from msckf_amd.replay import FeatureStream, replay  # noqa: E402
from msckf_amd.trajectory import ate  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("stream")
    ap.add_argument("--euroc", default=None)
    ap.add_argument("--fp32", action="store_true")
    ap.add_argument("--out", default=None)
    ap.add_argument("--make-synthetic", nargs=2, type=int, metavar=("N_FRAMES", "SEED"))
    a = ap.parse_args()
    if a.make_synthetic:
        st = FeatureStream.from_synthetic(synth.make_sequence(*a.make_synthetic),
                                          meta={"synthetic": list(a.make_synthetic)})
        st.save(a.stream)
        print("wrote", a.stream)
        return
    st = FeatureStream.load_csv(a.stream) if os.path.isdir(a.stream) else FeatureStream.load(a.stream)
    gt = st.gt
    if a.euroc:
        from msckf_amd.euroc import EuRoC
        gt = EuRoC(a.euroc).groundtruth()
    import msckf_amd
    flt = msckf_amd.MSCKF(dtype=np.float32 if a.fp32 else np.float64)
    t0 = time.perf_counter()
    traj = replay(flt, st)
    el = time.perf_counter() - t0
    flt.close()
    out = {"frames": len(traj), "seconds": round(el, 3), "frames_per_s": round(len(traj) / max(el, 1e-9), 1)}
    if gt is not None and len(traj) >= 3:
        out["ate_vs_gt_m"] = ate(traj, gt)
    if a.out:
        np.savetxt(a.out, np.column_stack([traj.t, traj.p]), delimiter=",", header="t,x,y,z", comments="")
    print(json.dumps(out))


if __name__ == "__main__":
    main()
