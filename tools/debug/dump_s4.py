"""Debug: the update requests of golden sequence s4's first frames on the GPU
(drop-in class, fp64) with the device's gamma / accept / positions, saved to
gpurun_out/dump_s4.npz for a CPU comparison with the oracle."""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
import msckf_pkg  # noqa: E402,F401
import msckf_amd  # noqa: E402
from conftest import golden  # noqa: E402
from helpers import sequence_config  # noqa: E402
from msckf_amd import synth  # noqa: E402

g = golden("sequence_s4")
seq = synth.make_sequence(int(g["n_frames"]), int(g["seed"]))
flt = msckf_amd.MSCKF(sequence_config(g))
serve = flt._serve
rec = {}
k = [0]


def hook(req):
    r = serve(req)
    if req[0] in ("update", "triangulate") and flt._n_published <= 7:
        i = k[0]
        k[0] += 1
        for j, a in enumerate(req[1:]):
            if isinstance(a, np.ndarray):
                rec["%d_%s_in%d" % (i, req[0], j)] = a
        for j, a in enumerate(r if isinstance(r, tuple) else (r,)):
            if isinstance(a, np.ndarray):
                rec["%d_%s_out%d" % (i, req[0], j)] = a
        rec["%d_frame" % i] = np.array(flt._n_published)
        imu, cams, P = flt.ctx.get_state(flt.slot)
        rec["%d_P" % i] = P
        rec["%d_cams" % i] = cams
        rec["%d_imu" % i] = imu
    return r


flt._serve = hook
for kind, m in seq.events():
    if kind == 0:
        flt.imu_callback(m)
        continue
    flt.feature_callback(m)
    if flt._n_published > 7:
        break
os.makedirs(os.path.join(ROOT, "gpurun_out"), exist_ok=True)
np.savez(os.path.join(ROOT, "gpurun_out", "dump_s4.npz"), **rec)
print("gate log", flt.gate_log[:8])
