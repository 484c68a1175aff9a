"""Shared test helpers: build oracle states from golden/synthetic problems."""
from collections import OrderedDict

import numpy as np

from oracle import msckf_oracle as O


def oracle_state_from_arrays(d, sigma2=0.035 ** 2, Qc=None):
    """``d`` holds the keys written by tools/gen_golden.py:problem_arrays (or
    an UpdateProblem converted with ``problem_to_dict``)."""
    imu = O.ImuState(q=d["imu_q"].copy(), p=d["imu_p"].copy(), v=d["imu_v"].copy(),
                     bg=d["imu_bg"].copy(), ba=d["imu_ba"].copy(), q_null=d["imu_q_null"].copy(),
                     R_imu_cam0=d["imu_R_imu_cam0"].copy(), t_cam0_imu=d["imu_t_cam0_imu"].copy())
    cams = OrderedDict()
    for i in range(int(d["N"])):
        cams[i] = O.CamState(i, float(i), d["cam_q"][i].copy(), d["cam_p"][i].copy(),
                             d["cam_q_null"][i].copy())
    if Qc is None:
        Qc = np.diag([0.005 ** 2] * 3 + [0.001 ** 2] * 3 + [0.05 ** 2] * 3 + [0.01 ** 2] * 3)
    return O.FilterState(imu, cams, d["P"].copy(), d["gravity"].copy(), d["R_cam0_cam1"],
                         d["t_cam0_cam1"], Qc, sigma2)


def problem_to_dict(pr):
    d = dict(N=pr.N, F=pr.F, cam_q=pr.cam_q, cam_p=pr.cam_p, cam_q_null=pr.cam_q_null,
             P=pr.P, gravity=pr.gravity, R_cam0_cam1=pr.R_cam0_cam1, t_cam0_cam1=pr.t_cam0_cam1,
             obs_off=pr.obs_off, obs_cam=pr.obs_cam, obs_z=pr.obs_z)
    for k, v in pr.imu.items():
        d["imu_" + k] = v
    return d


def feature_obs(d, f):
    a, b = int(d["obs_off"][f]), int(d["obs_off"][f + 1])
    return [(int(c), d["obs_z"][r]) for r, c in zip(range(a, b), d["obs_cam"][a:b])]


def oracle_update(d, row_cap=None, triangulate=True, accept=None, tri=None, sigma2=0.035 ** 2):
    """Oracle restatement of the synthetic update: triangulate, jacobian,
    gate (dof = M-1, the lost-feature path), stack, EKF update.
    ``tri = (p, ok)`` replaces the triangulation and ``accept`` (bool per
    feature) the chi2 decisions -- to rerun the update on another path's own
    decisions (the fp32 parity tests).
    Returns (state, accept flags, tri positions, tri ok, gammas)."""
    st = oracle_state_from_arrays(d, sigma2=sigma2)
    F = int(d["F"])
    tri_p = np.zeros((F, 3))
    tri_ok = np.zeros(F, bool)
    gam = np.full(F, np.nan)
    acc = np.zeros(F, bool)
    Hs, rs = [], []
    count = 0
    from msckf_amd import chi2_threshold
    for f in range(F):
        obs = feature_obs(d, f)
        if tri is not None:
            p, ok = np.asarray(tri[0][f], float), bool(tri[1][f])
        elif triangulate:
            p, ok, _ = O.triangulate(OrderedDict(obs), st.cams, st.R_cam0_cam1, st.t_cam0_cam1)
        else:
            p, ok = d["tri_p"][f], bool(d["tri_ok"][f])
        tri_p[f], tri_ok[f] = p, ok
        if not ok:
            continue
        H, r = O.feature_jacobian(st, p, obs)
        if accept is not None:      # forced decisions: no gating
            take = bool(accept[f])
        else:
            gam[f] = O.gating_gamma(st, H, r)
            take = gam[f] < chi2_threshold(len(obs) - 1)
        if take:
            acc[f] = True
            Hs.append(H)
            rs.append(r)
            count += H.shape[0]
        if row_cap is not None and count > row_cap:
            break
    if Hs:
        O.measurement_update(st, np.vstack(Hs), np.concatenate(rs))
    return st, acc, tri_p, tri_ok, gam


def rounded(d, dtype=np.float32):
    """The problem as a context of scalar type ``dtype`` holds it: every
    floating-point array rounded to ``dtype`` (and back to float64)."""
    out = {}
    for k, v in d.items():
        a = np.asarray(v)
        out[k] = a.astype(dtype).astype(np.float64) if a.dtype.kind == "f" else v
    return out


def sequence_config(g):
    """FilterConfig with the config edits a sequence fixture was made with
    (tools/gen_golden.py:gen_sequence)."""
    from msckf_amd import FilterConfig
    cfg = FilterConfig()
    if "translation_threshold" in g:
        cfg.optimization.translation_threshold = float(g["translation_threshold"])
    if "position_std_threshold" in g:
        cfg.position_std_threshold = float(g["position_std_threshold"])
    return cfg


def oracle_state_from_device(imu_rec, cams, P, sigma2=0.035 ** 2):
    """Oracle FilterState of one device filter slot (ctx.get_state output):
    cam states keyed by slot, the EuRoC extrinsics and noise of FilterConfig."""
    from msckf_amd import FilterConfig, _lib
    imu = _lib.unpack_imu(imu_rec)
    T = np.asarray(FilterConfig().T_cn_cnm1)
    Qc = np.diag([0.005 ** 2] * 3 + [0.001 ** 2] * 3 + [0.05 ** 2] * 3 + [0.01 ** 2] * 3)
    oi = O.ImuState(q=imu["q"], p=imu["p"], v=imu["v"], bg=imu["bg"], ba=imu["ba"], q_null=imu["q_null"],
                    R_imu_cam0=imu["R_imu_cam0"], t_cam0_imu=imu["t_cam0_imu"])
    oc = OrderedDict((i, O.CamState(i, float(i), cams[i, 0:4].copy(), cams[i, 4:7].copy(), cams[i, 7:11].copy()))
                     for i in range(len(cams)))
    return O.FilterState(oi, oc, P.copy(), imu["gravity"].copy(), T[:3, :3], T[:3, 3], Qc, sigma2)


def gamma_basis_spread(st, p_w, obs, n_bases=8, seed=0):
    """The reference's gamma (msckf.py:606-614: SVD left-nullspace basis,
    msckf.py:535-539, LU solve) of one feature, and its largest relative change
    when the nullspace basis is replaced by other orthonormal bases of the same
    space (H -> Q H, r -> Q r, Q random orthogonal).  In exact arithmetic gamma
    does not depend on the basis (quirk Q4); a spread far above rounding marks a
    numerically degenerate feature whose reference decision is rounding noise.
    A basis in which S is singular counts as an unbounded change."""
    H, r = O.feature_jacobian(st, p_w, obs)
    g0 = O.gating_gamma(st, H, r)
    rng = np.random.default_rng(seed)
    spread = 0.0
    for _ in range(n_bases):
        Q, _ = np.linalg.qr(rng.standard_normal((len(r), len(r))))
        try:
            g = O.gating_gamma(st, Q @ H, Q @ r)
        except np.linalg.LinAlgError:
            return g0, np.inf
        spread = max(spread, abs(g / g0 - 1) if g0 != 0 else np.inf)
    return g0, spread
