"""Large-batch check mirroring bench.py's setup, with knobs to bisect:
  debug_big.py B UNIQUE CAP(0 = N+2) RESTORE(0/1)"""
import os, sys
import numpy as np
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT); sys.path.insert(0, os.path.join(ROOT, "tests"))
import msckf_pkg  # noqa
from msckf_amd import synth, FilterConfig, CHI2_05
from msckf_amd._lib import MsckfError, Context, pack_imu, pack_cams
from helpers import problem_to_dict, oracle_update
B, U, CAP, RESTORE = [int(x) for x in (sys.argv[1:] + ["2048", "32", "0", "1"][len(sys.argv) - 1:])]
uniq = [synth.make_update_problem(30, 200, seed=s) for s in range(U)]
probs = [uniq[b % U] for b in range(B)]
ctx = Context(FilterConfig(), n_filters=B, n_cam_capacity=CAP or 32, dtype=np.float32)
feat_off, obs_off, cams, zs, chi = [0], [0], [], [], []
for b, p in enumerate(probs):
    imu = pack_imu(q=p.imu["q"], p=p.imu["p"], v=p.imu["v"], bg=p.imu["bg"], ba=p.imu["ba"], q_null=p.imu["q_null"],
                   p_null=p.imu["p_null"], v_null=p.imu["v_null"], R_imu_cam0=p.imu["R_imu_cam0"],
                   t_cam0_imu=p.imu["t_cam0_imu"], gravity=p.gravity, alias=True)
    ctx.set_state(b, imu, pack_cams(p.cam_q, p.cam_p, p.cam_q_null), p.P)
    feat_off.append(feat_off[-1] + p.F)
    obs_off.extend(list(obs_off[-1] + p.obs_off[1:]))
    cams.append(p.obs_cam); zs.append(p.obs_z)
    chi.extend(CHI2_05[m - 2] for m in p.track_lengths())
ctx.batch_load(np.array(feat_off), np.array(obs_off), np.concatenate(cams), np.concatenate(zs), None, np.array(chi))
if RESTORE:
    ctx.snapshot(); ctx.restore()
ctx.batch_update(row_cap=0, triangulate=True)
try:
    acc, gam, pw, valid, rows = ctx.batch_results()
    print("B=%d U=%d CAP=%d RESTORE=%d ok rows %.1f" % (B, U, CAP, RESTORE, rows.mean()))
except MsckfError as e:
    print("B=%d U=%d CAP=%d RESTORE=%d FAIL %s" % (B, U, CAP, RESTORE, e))
    sys.exit(0)
for b in [0, 1, B - 1]:
    st, acc_o, *_ = oracle_update(problem_to_dict(probs[b]))
    P = ctx.get_state(b)[2]
    print("  filter", b, "relP %.2e" % (np.linalg.norm(P - st.P) / np.linalg.norm(st.P)))
