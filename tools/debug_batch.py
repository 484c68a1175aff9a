"""Debug helper: run the bench's synthetic problems through the batched path
and report per-filter status against the fp64 oracle."""
import os, sys
import numpy as np
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT); sys.path.insert(0, os.path.join(ROOT, "tests"))
import msckf_pkg  # noqa
from msckf_amd import synth, CHI2_05
from msckf_amd._lib import MsckfError
from helpers import problem_to_dict, oracle_update
from test_gpu_parity import _batched

dtype = np.float32 if (len(sys.argv) < 2 or sys.argv[1] == "fp32") else np.float64
seeds = range(int(sys.argv[2]) if len(sys.argv) > 2 else 32)
probs = [synth.make_update_problem(30, 200, seed=s) for s in seeds]
try:
    ctx, ds, feat_off, acc, gam, pw, valid, rows = _batched(probs, dtype)
    print("batch ok")
except MsckfError as e:
    print("batch error:", e)
    ctx = None
for s, p in zip(seeds, probs):
    try:
        c1, d1, fo, a1, g1, pw1, v1, r1 = _batched([p], dtype)
        imu, cams, P = c1.get_state(0)
        st, acc_o, tri_p, tri_ok, gam_o = oracle_update(problem_to_dict(p))
        err = np.linalg.norm(P - st.P) / np.linalg.norm(st.P)
        print("seed %2d ok rows=%d agree=%.3f relP=%.2e nan=%s" % (s, r1[0], (a1 == acc_o).mean(), err, np.isnan(P).any()))
    except MsckfError as e:
        print("seed %2d FAIL %s" % (s, e))
