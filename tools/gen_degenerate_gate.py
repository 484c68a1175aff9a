"""Fixture tests/golden/degenerate_gate.npz: a numerically degenerate gating
case met on golden sequence s4 (frame 3, the first update): a landmark
triangulated 0.86 mm in front of the camera, so the measurement Jacobian's
entries reach ~1e9 and the reference's S = H P H^T + s2 I (msckf.py:606-609)
has condition number ~5e18 -- singular in fp64.  The reference's gamma
(SVD nullspace basis, LU solve) is rounding noise there: an equally valid
rotated nullspace basis changes it by 5x or makes S exactly singular.

Inputs: the filter state and update request captured from the GPU run of s4
(tools/debug/dump_s4.py -> gpurun_out/dump_s4.npz).  Expected: gamma of each
feature from the saddle-point form [[Y, H_f, r], [H_f^T, 0, 0]] (the same
value as r0^T S^-1 r0 in exact arithmetic) solved with 50 significant digits
(mpmath), plus the fp64 numpy values of the reference formula for contrast.

    python tools/gen_degenerate_gate.py [gpurun_out/dump_s4.npz]
"""
import os
import sys
from collections import OrderedDict

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import msckf_pkg  # noqa: E402,F401
from msckf_amd import FilterConfig, _lib  # noqa: E402
import oracle.msckf_oracle as O  # noqa: E402
import mpmath  # noqa: E402


def main():
    src = sys.argv[1] if len(sys.argv) > 1 else os.path.join(ROOT, "gpurun_out", "dump_s4.npz")
    d = np.load(src)
    imu_rec, cams, P = d["0_imu"], d["0_cams"], d["0_P"]
    off, cam, z, pw = d["1_update_in0"], d["1_update_in1"], d["1_update_in2"], d["1_update_in3"]
    imu = _lib.unpack_imu(imu_rec)
    n = (P.shape[0] - 21) // 6
    T = np.asarray(FilterConfig().T_cn_cnm1)
    Qc = np.diag([0.005 ** 2] * 3 + [0.001 ** 2] * 3 + [0.05 ** 2] * 3 + [0.01 ** 2] * 3)
    oi = O.ImuState(q=imu["q"], p=imu["p"], v=imu["v"], bg=imu["bg"], ba=imu["ba"], q_null=imu["q_null"],
                    R_imu_cam0=imu["R_imu_cam0"], t_cam0_imu=imu["t_cam0_imu"])
    oc = OrderedDict((i, O.CamState(i, float(i), cams[i, 0:4].copy(), cams[i, 4:7].copy(), cams[i, 7:11].copy()))
                     for i in range(n))
    st = O.FilterState(oi, oc, P.copy(), imu["gravity"].copy(), T[:3, :3], T[:3, 3], Qc, 0.035 ** 2)
    mpmath.mp.dps = 50
    exact, ref64, cond = [], [], []
    for f in range(len(off) - 1):
        obs = [(int(cam[i]), z[i]) for i in range(off[f], off[f + 1])]
        H, r = O.feature_jacobian(st, pw[f], obs)
        ref64.append(O.gating_gamma(st, H, r))
        S = H @ st.P @ H.T + st.sigma2 * np.eye(len(H))
        cond.append(np.linalg.cond(S))
        keys = list(st.cams.keys())
        rows = 4 * len(obs)
        Hx = np.zeros((rows, 21 + 6 * n))
        Hf = np.zeros((rows, 3))
        rr = np.zeros(rows)
        for i, (cid, zz) in enumerate(obs):
            a, b, c = O.measurement_jacobian(st, st.cams[cid], pw[f], zz)
            k = keys.index(cid)
            Hx[4 * i:4 * i + 4, 21 + 6 * k:27 + 6 * k] = a
            Hf[4 * i:4 * i + 4] = b
            rr[4 * i:4 * i + 4] = c
        Hm, Pm, Fm = mpmath.matrix(Hx.tolist()), mpmath.matrix(st.P.tolist()), mpmath.matrix(Hf.tolist())
        Ym = Hm * Pm * Hm.T + mpmath.mpf(st.sigma2) * mpmath.eye(rows)
        Km = mpmath.zeros(rows + 3, rows + 3)
        for i in range(rows):
            for j in range(rows):
                Km[i, j] = Ym[i, j]
            for j in range(3):
                Km[i, rows + j] = Fm[i, j]
                Km[rows + j, i] = Fm[i, j]
        bv = mpmath.matrix(rows + 3, 1)
        for i in range(rows):
            bv[i] = rr[i]
        x = mpmath.lu_solve(Km, bv)
        exact.append(float(sum(mpmath.mpf(rr[i]) * x[i] for i in range(rows))))
    out = os.path.join(ROOT, "tests", "golden", "degenerate_gate.npz")
    np.savez_compressed(out, imu=imu_rec, cams=cams, P=P, obs_off=off, obs_cam=cam, obs_z=z, p_w=pw,
                        chi2=d["1_update_in4"], gamma_exact=np.array(exact), gamma_ref_fp64=np.array(ref64),
                        cond_S=np.array(cond))
    print("gamma exact", exact, "reference formula fp64", ref64, "cond(S)", cond)


if __name__ == "__main__":
    main()
