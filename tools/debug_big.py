"""Large-batch check: B filters tiled from the bench problems, compare a few
filters against the fp64 oracle after one batched update."""
import os, sys
import numpy as np
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT); sys.path.insert(0, os.path.join(ROOT, "tests"))
import msckf_pkg  # noqa
from msckf_amd import synth
from msckf_amd._lib import MsckfError
from helpers import problem_to_dict, oracle_update
from test_gpu_parity import _batched
B = int(sys.argv[1]) if len(sys.argv) > 1 else 2048
uniq = [synth.make_update_problem(30, 200, seed=s) for s in range(16)]
probs = [uniq[b % 16] for b in range(B)]
try:
    ctx, ds, feat_off, acc, gam, pw, valid, rows = _batched(probs, np.float32)
    print("batch ok, rows mean", rows.mean())
except MsckfError as e:
    print("batch error:", e); sys.exit(1)
for b in [0, 1, B // 2, B - 1]:
    st, acc_o, *_ = oracle_update(problem_to_dict(probs[b]))
    P = ctx.get_state(b)[2]
    print(b, "relP %.2e" % (np.linalg.norm(P - st.P) / np.linalg.norm(st.P)))
