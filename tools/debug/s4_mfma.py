"""Golden stream s4 through the drop-in class with the Kalman stages A / C1
forced onto one implementation (MSCKF_KALMAN_CHOL=mfma|tiles): prints the
frame at which an update fails (if any) and the per-frame state deviation
from the reference's recorded run.  GPU; runs against another package copy
with tools/exp/run_pkg.py.

    python tools/debug/s4_mfma.py [mfma|tiles]
"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
os.environ["MSCKF_KALMAN_CHOL"] = sys.argv[1] if len(sys.argv) > 1 else "mfma"
import numpy as np  # noqa: E402
import msckf_pkg  # noqa: E402,F401
import msckf_amd  # noqa: E402
from msckf_amd import synth  # noqa: E402
from helpers import sequence_config  # noqa: E402


def golden(name):
    return dict(np.load(os.path.join(ROOT, "tests", "golden", name + ".npz"), allow_pickle=False))


g = golden("sequence_s4")
seq = synth.make_sequence(int(g["n_frames"]), int(g["seed"]))
flt = msckf_amd.MSCKF(sequence_config(g))
ref = g["rec"]
k = 0
try:
    for kind, m in seq.events():
        if kind == 0:
            flt.imu_callback(m)
            continue
        res = flt.feature_callback(m)
        if res is None:
            continue
        s = flt.imu_state()
        x = np.concatenate([s["q"], s["p"], s["v"], s["bg"], s["ba"], s["R_imu_cam0"].ravel(), s["t_cam0_imu"]])
        dev = np.linalg.norm(x - ref[k, 1:29]) / np.linalg.norm(ref[k, 1:29])
        if k < 8 or k % 20 == 0:
            print("frame %3d  state deviation %.3e  D %d" % (k, dev, flt.state_cov().shape[0]), flush=True)
        k += 1
    print("s4 (%s): ran all %d frames" % (os.environ["MSCKF_KALMAN_CHOL"], k))
except msckf_amd.MsckfError as e:
    print("s4 (%s): frame %d failed: %s" % (os.environ["MSCKF_KALMAN_CHOL"], k, e))
    sys.exit(3)
