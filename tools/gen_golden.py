"""Generate the golden fixtures under tests/golden/ by running the REFERENCE
filter (NonStopEagle137/Visual-Inertial-Odometry-MSCKF-Stereo, read-only at
/root/reference/MSCKF) in the build container.

The reference has no tests or fixtures of its own, so
every parity pin is produced here and committed as data (inputs + expected
outputs).  The reference cannot travel to the GPU box; these .npz files do.

Usage:  python tools/gen_golden.py            (about a minute on 8 cores)
"""
import os
import sys
from collections import OrderedDict

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
sys.path.insert(0, ROOT)
sys.path.insert(0, HERE)

import msckf_pkg  # noqa: E402,F401
from msckf_amd import synth, CHI2_05  # noqa: E402
from refload import load_reference, fresh_filter  # noqa: E402

OUT = os.path.join(ROOT, "tests", "golden")
ref = load_reference()
U = ref.utils


def save(name, **arrs):
    path = os.path.join(OUT, name + ".npz")
    np.savez_compressed(path, **arrs)
    print("%-28s %7.1f KB" % (name, os.path.getsize(path) / 1024))


def rand_quat(rng, scale=1.0):
    q = rng.standard_normal(4) * np.array([scale, scale, scale, 1.0])
    q[3] = abs(q[3]) + 0.5
    return q / np.linalg.norm(q)


def install_problem(R, pr: synth.UpdateProblem, with_features=True):
    """Load an UpdateProblem into a reference MSCKF instance."""
    ss = R.state_server
    imu = ss._vio_imu_state__
    imu.orientation = pr.imu["q"].copy()
    imu._vio_position__ = pr.imu["p"].copy()
    imu.velocity = pr.imu["v"].copy()
    imu._vio_gyro_bias__ = pr.imu["bg"].copy()
    imu.acc_bias = pr.imu["ba"].copy()
    imu.orientation_null = pr.imu["q_null"].copy()
    imu.R_imu_cam0 = pr.imu["R_imu_cam0"].copy()
    imu.t_cam0_imu = pr.imu["t_cam0_imu"].copy()
    ref.msckf.IMUState._vio_gravity__ = pr.gravity.copy()
    ss._vio_cam_states__ = OrderedDict()
    for i in range(pr.N):
        c = ref.msckf.CAMState(i)
        c.timestamp = float(i)
        c.orientation = pr.cam_q[i].copy()
        c._vio_position__ = pr.cam_p[i].copy()
        c.orientation_null = pr.cam_q_null[i].copy()
        c.position_null = c._vio_position__          # alias, as msckf.py:400
        ss._vio_cam_states__[i] = c
    ss._vio_state_cov__ = pr.P.copy()
    R.map_server = OrderedDict()
    if with_features:
        for f in range(pr.F):
            feat = ref.feature.Feature(f, R.optimization_config)
            for r in range(pr.obs_off[f], pr.obs_off[f + 1]):
                feat.observations[int(pr.obs_cam[r])] = pr.obs_z[r].copy()
            R.map_server[f] = feat


def problem_arrays(pr: synth.UpdateProblem):
    d = dict(N=pr.N, F=pr.F, cam_q=pr.cam_q, cam_p=pr.cam_p, cam_q_null=pr.cam_q_null,
             P=pr.P, gravity=pr.gravity, R_cam0_cam1=pr.R_cam0_cam1, t_cam0_cam1=pr.t_cam0_cam1,
             obs_off=pr.obs_off, obs_cam=pr.obs_cam, obs_z=pr.obs_z)
    for k, v in pr.imu.items():
        d["imu_" + k] = v
    return d


def gen_math():
    rng = np.random.default_rng(100)
    qs = np.stack([rand_quat(rng) for _ in range(64)])
    qs2 = np.stack([rand_quat(rng) for _ in range(64)])
    Rs = np.stack([U.to_rotation(q) for q in qs])
    qR = np.stack([U.to_quaternion(R) for R in Rs])
    qm = np.stack([U.quaternion_multiplication(a, b) for a, b in zip(qs, qs2)])
    dth = rng.standard_normal((64, 3)) * np.r_[np.full(48, 0.1), np.full(16, 3.0)][:, None]
    sa = np.stack([U.small_angle_quaternion(d) for d in dth])
    v0 = rng.standard_normal((64, 3))
    v1 = rng.standard_normal((64, 3))
    v1[0] = v0[0] * 2.0
    v1[1] = -v0[1]
    ftv = np.stack([U.from_two_vectors(a, b) for a, b in zip(v0, v1)])
    save("math", qs=qs, qs2=qs2, to_rotation=Rs, to_quaternion=qR, quat_mult=qm,
         dtheta=dth, small_angle=sa, v0=v0, v1=v1, from_two_vectors=ftv,
         chi2=np.array(CHI2_05))


def gen_process_model():
    """Fixture (i): 20 IMU steps of msckf.py:291-368 on a window of 5 cams."""
    rng = np.random.default_rng(1)
    R, _ = fresh_filter(ref)
    pr = synth.make_update_problem(5, 4, seed=11)
    install_problem(R, pr, with_features=False)
    imu = R.state_server._vio_imu_state__
    imu.timestamp = 10.0
    imu.velocity = np.array([0.3, -0.2, 0.1])
    imu._vio_position__ = np.array([1.0, 2.0, -0.5])
    # after a previous process_model the null velocity/position alias the live
    # arrays (Q5); the null orientation is the pre-update estimate
    imu.velocity_null = imu.velocity
    imu.position_null = imu._vio_position__
    imu.orientation_null = U.quaternion_multiplication(
        U.small_angle_quaternion(np.array([1e-3, -2e-3, 5e-4])), imu.orientation)
    g = np.array([0.0, 0.0, -9.806])
    ref.msckf.IMUState._vio_gravity__ = g
    init = dict(q=imu.orientation.copy(), v=imu.velocity.copy(), p=imu._vio_position__.copy(),
                bg=imu._vio_gyro_bias__.copy(), ba=imu.acc_bias.copy(),
                q_null=imu.orientation_null.copy(), P=R.state_server._vio_state_cov__.copy())
    ts = 10.0 + 0.005 * np.arange(1, 21)
    gyro = 0.3 * rng.standard_normal((20, 3))
    acc = np.array([0.0, 0.0, 9.806]) + 0.5 * rng.standard_normal((20, 3))
    gyro[5] = 1e-7 * rng.standard_normal(3)           # the small-rotation branch
    qs, vs, ps, Phis = [], [], [], []
    for k in range(20):
        R.process_model(ts[k], gyro[k], acc[k])
        R.state_server._vio_imu_state__.timestamp = ts[k]
        im = R.state_server._vio_imu_state__
        qs.append(im.orientation.copy())
        vs.append(im.velocity.copy())
        ps.append(im._vio_position__.copy())
    F, G, _, _, _, Phi0 = ref.jit_utils._process_model(gyro[0] - init["bg"],
                                                       U.to_rotation(init["q"]), acc[0] - init["ba"], 0.005)
    save("process_model", t0=10.0, ts=ts, gyro=gyro, acc=acc, gravity=g, Qc=R.state_server._vio_continuous_noise_cov__,
         cam_q=pr.cam_q, cam_p=pr.cam_p, cam_q_null=pr.cam_q_null,
         R_imu_cam0=pr.imu["R_imu_cam0"], t_cam0_imu=pr.imu["t_cam0_imu"],
         **{"init_" + k: v for k, v in init.items()},
         q=np.stack(qs), v=np.stack(vs), p=np.stack(ps), P=R.state_server._vio_state_cov__,
         F0=F, G0=G, Phi0_unedited=Phi0)


def gen_augment():
    """Fixture (ii): msckf.py:385-407 on a window of 7 cams."""
    R, _ = fresh_filter(ref)
    pr = synth.make_update_problem(7, 4, seed=12)
    install_problem(R, pr, with_features=False)
    imu = R.state_server._vio_imu_state__
    imu.id = 99
    R.state_augmentation(55.5)
    c = R.state_server._vio_cam_states__[99]
    save("augment", **problem_arrays(pr), new_q=c.orientation, new_p=c._vio_position__,
         P_out=R.state_server._vio_state_cov__)


def gen_update(name, N, F, seed, full=False, n_inv=24):
    """Fixtures (iii)-(vii): triangulation, jacobians, invariants, gating and
    the EKF update on one synthetic problem."""
    R, _ = fresh_filter(ref)
    pr = synth.make_update_problem(N, F, seed=seed, full_tracks=full)
    install_problem(R, pr)
    tri_p, tri_ok = [], []
    for f in range(F):
        feat = R.map_server[f]
        ok = feat.initialize_position(R.state_server._vio_cam_states__)
        tri_p.append(feat._vio_position__.copy())
        tri_ok.append(bool(ok))
    tri_p = np.array(tri_p)
    # raw measurement Jacobian blocks for the first observation of each feature
    mj_Hx, mj_Hf, mj_r = [], [], []
    for f in range(F):
        cid = int(pr.obs_cam[pr.obs_off[f]])
        Hx, Hf, r = R.measurement_jacobian(cid, f)
        mj_Hx.append(Hx)
        mj_Hf.append(Hf)
        mj_r.append(r)
    HtH, Htr, rtr, gam, acc, k = [], [], [], [], [], []
    Hs, rs = [], []
    for f in range(F):
        cids = [int(c) for c in pr.obs_cam[pr.obs_off[f]:pr.obs_off[f + 1]]]
        H, r = R.feature_jacobian(f, cids)
        S = H @ R.state_server._vio_state_cov__ @ H.T + R.config._vio_observation_noise__ * np.identity(len(H))
        g = r @ ref.jit_utils._fastSolve(S, r)
        a = bool(R.gating_test(H, r, len(cids) - 1))
        Hc = H[:, 21:]
        HtH.append(Hc.T @ Hc)
        Htr.append(Hc.T @ r)
        rtr.append(r @ r)
        gam.append(g)
        acc.append(a)
        k.append(H.shape[0])
        if a and tri_ok[f]:
            Hs.append(H)
            rs.append(r)
    C = 6 * N
    HtH_full = np.zeros((C, C))
    for f in range(F):
        if acc[f] and tri_ok[f]:
            HtH_full += HtH[f]
    H = np.vstack(Hs)
    r = np.concatenate(rs)
    imu = R.state_server._vio_imu_state__
    R.measurement_update(H, r)
    cams = R.state_server._vio_cam_states__
    # per-feature invariants are stored for the first n_inv features only (size)
    nk = min(F, n_inv)
    save(name, **problem_arrays(pr), tri_p=tri_p, tri_ok=np.array(tri_ok),
         mj_Hx=np.array(mj_Hx), mj_Hf=np.array(mj_Hf), mj_r=np.array(mj_r),
         HtH=np.concatenate([h.ravel() for h in HtH[:nk]]),
         HtH_sizes=np.array([h.shape[0] for h in HtH[:nk]]),
         Htr=np.concatenate(Htr[:nk]), rtr=np.array(rtr), gamma=np.array(gam), accept=np.array(acc),
         rows=np.array(k), stacked_rows=H.shape[0], HtH_total=HtH_full,
         P_out=R.state_server._vio_state_cov__,
         imu_q_out=imu.orientation, imu_p_out=imu._vio_position__, imu_v_out=imu.velocity,
         imu_bg_out=imu._vio_gyro_bias__, imu_ba_out=imu.acc_bias,
         R_imu_cam0_out=imu.R_imu_cam0, t_cam0_imu_out=imu.t_cam0_imu,
         cam_q_out=np.stack([c.orientation for c in cams.values()]),
         cam_p_out=np.stack([c._vio_position__ for c in cams.values()]))


def gen_prune():
    """Fixture (viii): P compaction msckf.py:803-818 + keyframe choice 691-727."""
    R, _ = fresh_filter(ref)
    pr = synth.make_update_problem(9, 4, seed=13)
    install_problem(R, pr, with_features=False)
    out = {}
    for tr in (0.3, 0.9):
        R.tracking_rate = tr
        out["rm_%d" % int(tr * 10)] = np.array(R.find_redundant_cam_states())
    rm = [2, 5]
    R.state_server._vio_state_cov__ = pr.P.copy()
    for cid in rm:
        idx = list(R.state_server._vio_cam_states__.keys()).index(cid)
        s, e = 21 + 6 * idx, 27 + 6 * idx
        P = R.state_server._vio_state_cov__.copy()
        if e < P.shape[0]:
            P[s:-6, :] = P[e:, :]
            P[:, s:-6] = P[:, e:]
        R.state_server._vio_state_cov__ = P[:-6, :-6]
        del R.state_server._vio_cam_states__[cid]
    save("prune", **problem_arrays(pr), rm=np.array(rm), P_out=R.state_server._vio_state_cov__, **out)


def gen_check_motion():
    """Fixture (x): Feature.check_motion feature.py:124-165 on random cam
    windows and observations, at the config.py:10 thresholds -1 / 0.2 and
    config.py:68's 0.4."""
    rng = np.random.default_rng(21)
    n_cams, n_feat = 12, 64
    cq = np.stack([rand_quat(rng, 0.3) for _ in range(n_cams)])
    cp = rng.standard_normal((n_cams, 3)) * 0.35
    cams = OrderedDict()
    for i in range(n_cams):
        c = ref.msckf.CAMState(i)
        c.orientation = cq[i].copy()
        c._vio_position__ = cp[i].copy()
        cams[i] = c
    first = rng.integers(0, n_cams - 2, n_feat)
    last = np.minimum(first + rng.integers(2, 8, n_feat), n_cams - 1)
    z = rng.uniform(-0.6, 0.6, (n_feat, 4))
    out = {}
    for thr in (-1.0, 0.2, 0.4):
        oc = ref.config.OptimizationConfigEuRoC()
        oc._vio_translation_threshold__ = thr
        res = []
        for j in range(n_feat):
            f = ref.feature.Feature(j, oc)
            for c in range(first[j], last[j] + 1):
                f.observations[c] = z[j] + 0.01 * (c - first[j])
            res.append(bool(f.check_motion(cams)))
        out["ok_%s" % ("m1" if thr < 0 else str(int(thr * 10)))] = np.array(res)
    save("check_motion", cam_q=cq, cam_p=cp, first=first, last=last, z=z, **out)


def gen_sequence(name, n_frames, seed, translation_threshold=None, position_std_threshold=None):
    """Fixture (ix): the full reference filter on a synthetic stereo+IMU stream,
    fed in strict time order.  Per frame: state, covariance norms, the gating
    decision sequence and the stacked-H shapes.  Optional config edits: the
    feature translation threshold (check_motion, feature.py:124-165) and the
    position std threshold of online_reset (msckf.py:859-886)."""
    R, _ = fresh_filter(ref)
    if translation_threshold is not None:
        R.optimization_config._vio_translation_threshold__ = translation_threshold
    if position_std_threshold is not None:
        R.config._vio_position_std_threshold__ = position_std_threshold
    resets = []
    orig_reset = R.reset_state_cov

    def reset():
        resets.append(len(recs))
        return orig_reset()
    seq = synth.make_sequence(n_frames, seed)
    gates, shapes = [], []
    orig_gate, orig_upd = R.gating_test, R.measurement_update

    def gate(H, r, dof):
        ok = orig_gate(H, r, dof)
        gates.append((len(recs), dof, H.shape[0], int(bool(ok))))
        return ok

    def upd(H, r):
        shapes.append((len(recs), H.shape[0], H.shape[1] if H.ndim == 2 else 0))
        return orig_upd(H, r)

    R.gating_test, R.measurement_update = gate, upd
    recs = []
    R.reset_state_cov = reset
    for kind, m in seq.events():
        if kind == 0:
            R.imu_callback(m)
            continue
        res = R.feature_callback(m)
        if res is None:
            continue
        imu = R.state_server._vio_imu_state__
        P = R.state_server._vio_state_cov__
        recs.append(np.concatenate([
            [m.timestamp], imu.orientation, imu._vio_position__, imu.velocity,
            imu._vio_gyro_bias__, imu.acc_bias, imu.R_imu_cam0.ravel(), imu.t_cam0_imu,
            [np.linalg.norm(P), np.trace(P), P.shape[0], len(R.state_server._vio_cam_states__),
             len(R.map_server)], res.cam0_pose._vio_R__.ravel(), res.cam0_pose._vio_t__]))
    P = R.state_server._vio_state_cov__
    extra = {}
    if translation_threshold is not None:
        extra["translation_threshold"] = translation_threshold
    if position_std_threshold is not None:
        extra["position_std_threshold"] = position_std_threshold
    save(name, seed=seed, n_frames=n_frames, rec=np.array(recs),
         gates=np.array(gates, dtype=np.int64), shapes=np.array(shapes, dtype=np.int64),
         P_final=P, gravity=ref.msckf.IMUState._vio_gravity__, resets=np.array(resets, dtype=np.int64), **extra)


JOBS = {
    "math": gen_math,
    "process_model": gen_process_model,
    "augment": gen_augment,
    "update_n10_f40": lambda: gen_update("update_n10_f40", 10, 40, seed=3),
    "update_n20_f100": lambda: gen_update("update_n20_f100", 20, 100, seed=4, n_inv=6),
    "prune": gen_prune,
    "check_motion": gen_check_motion,
    "sequence_s1": lambda: gen_sequence("sequence_s1", 200, 1),
    # check_motion on: threshold 0.2, the value config.py:10 comments out
    "sequence_s2": lambda: gen_sequence("sequence_s2", 120, 2, translation_threshold=0.2),
    # online_reset firing: position std threshold 0.11 m instead of 8 m (config.py:64)
    "sequence_s3": lambda: gen_sequence("sequence_s3", 100, 2, position_std_threshold=0.11),
    # the reference's non-Joseph update leaves P_cc indefinite at rounding level
    # (min eigenvalue ~ -2e-12 from frame 2 on); a Cholesky of P_cc without a
    # pivot floor fails at frame 19 (found by the 11-lane config-4 test)
    "sequence_s4": lambda: gen_sequence("sequence_s4", 180, 307),
}

if __name__ == "__main__":
    # python tools/gen_golden.py [fixture ...]   (default: all)
    os.makedirs(OUT, exist_ok=True)
    for name in (sys.argv[1:] or list(JOBS)):
        JOBS[name]()
