"""CPU ORACLE -- TEST INFRASTRUCTURE ONLY.

This module is a plain-numpy restatement of the reference MSCKF hot path
(NonStopEagle137/Visual-Inertial-Odometry-MSCKF-Stereo, MSCKF/*.py).  It is the
checker for the HIP path: only ``tests/``, ``__graft_entry__.smoke()`` and
``bench.py``'s ``cpu_baseline`` leg may import it.  The product package
(``visual-inertial-odometry-msckf-stereo_amd/``) never imports it and has no
CPU fallback.

Parity pin: every function below is checked against golden vectors produced by
running the reference itself in the build container (``tools/gen_golden.py``,
fixtures under ``tests/golden/``; ``tests/test_oracle_golden.py``).

Arithmetic follows the reference op for op (same numpy expressions, same
evaluation order, fp64) including its quirks:

* Q1  RK4 rotation reuse in ``predict_new_state``     (jit_utils.py:81-104)
* Q2  LM ``is_cost_reduced`` never reset               (feature.py:224-275)
* Q3  observability projection of H_x                 (msckf.py:483-490)
* Q4  SVD left-nullspace                              (msckf.py:533-539)
* Q5  ``*_null`` aliasing of position/velocity        (msckf.py:366-368, 399-400)
* Q6  chi2 at the 5 % lower quantile                  (msckf.py:121-123)
* Q7  class-level globals become per-instance fields here.
"""
from __future__ import annotations

from collections import OrderedDict
from dataclasses import dataclass, field
from typing import Dict, List, Optional, Sequence, Tuple

import numpy as np

I3 = np.identity(3)
I4 = np.identity(4)

# --------------------------------------------------------------------------
# SO(3) / JPL quaternion helpers                               (utils.py:1-152)
# Quaternions are JPL, stored [x, y, z, w]; to_rotation(q) maps world->body.
# --------------------------------------------------------------------------


def skew(w):
    """utils.py:4-12"""
    x, y, z = w
    return np.array([[0, -z, y], [z, 0, -x], [-y, x, 0]])


def to_rotation(q):
    """utils.py:14-27 (Trawny & Roumeliotis eq. 78)."""
    q = q / np.linalg.norm(q)
    v, w = q[:3], q[3]
    return (2 * w * w - 1) * I3 - 2 * w * skew(v) + 2 * v[:, None] * v


def to_quaternion(R):
    """utils.py:29-53 (branch order kept, result normalised)."""
    if R[2, 2] < 0:
        if R[0, 0] > R[1, 1]:
            t = 1 + R[0, 0] - R[1, 1] - R[2, 2]
            q = [t, R[0, 1] + R[1, 0], R[2, 0] + R[0, 2], R[1, 2] - R[2, 1]]
        else:
            t = 1 - R[0, 0] + R[1, 1] - R[2, 2]
            q = [R[0, 1] + R[1, 0], t, R[2, 1] + R[1, 2], R[2, 0] - R[0, 2]]
    else:
        if R[0, 0] < -R[1, 1]:
            t = 1 - R[0, 0] - R[1, 1] + R[2, 2]
            q = [R[0, 2] + R[2, 0], R[2, 1] + R[1, 2], t, R[0, 1] - R[1, 0]]
        else:
            t = 1 + R[0, 0] + R[1, 1] + R[2, 2]
            q = [R[1, 2] - R[2, 1], R[2, 0] - R[0, 2], R[0, 1] - R[1, 0], t]
    q = np.array(q)
    return q / np.linalg.norm(q)


def quaternion_conjugate(q):
    """utils.py:61-65"""
    return np.array([*-q[:3], q[3]])


def quaternion_multiplication(q1, q2):
    """utils.py:67-82: q1 (x) q2, both normalised first."""
    q1 = q1 / np.linalg.norm(q1)
    q2 = q2 / np.linalg.norm(q2)
    L = np.array([
        [q1[3], q1[2], -q1[1], q1[0]],
        [-q1[2], q1[3], q1[0], q1[1]],
        [q1[1], -q1[0], q1[3], q1[2]],
        [-q1[0], -q1[1], -q1[2], q1[3]]])
    q = L @ q2
    return q / np.linalg.norm(q)


def small_angle_quaternion(dtheta):
    """utils.py:85-101"""
    dq = dtheta / 2.
    n2 = dq @ dq
    if n2 <= 1:
        q = np.array([*dq, np.sqrt(1 - n2)])
    else:
        q = np.array([*dq, 1.])
        q /= np.sqrt(1 + n2)
    return q


def from_two_vectors(v0, v1):
    """utils.py:104-128 (Hamilton result conjugated to JPL)."""
    v0 = v0 / np.linalg.norm(v0)
    v1 = v1 / np.linalg.norm(v1)
    d = v0 @ v1
    if d < -0.999999:
        axis = np.cross([1, 0, 0], v0)
        if np.linalg.norm(axis) < 0.000001:
            axis = np.cross([0, 1, 0], v0)
        q = np.array([*axis, 0.])
    elif d > 0.999999:
        q = np.array([0., 0., 0., 1.])
    else:
        s = np.sqrt((1 + d) * 2)
        axis = np.cross(v0, v1)
        q = np.array([*(axis / s), 0.5 * s])
    q = q / np.linalg.norm(q)
    return quaternion_conjugate(q)


class Iso:
    """Rigid transform (R, t) -- utils.py:132-152."""

    def __init__(self, R, t):
        self.R, self.t = R, t

    def inverse(self):
        return Iso(self.R.T, -self.R.T @ self.t)

    def __mul__(self, o):
        return Iso(self.R @ o.R, self.R @ o.t + self.t)


# --------------------------------------------------------------------------
# State                                  (msckf.py:16-100, with Q5/Q7 explicit)
# --------------------------------------------------------------------------


@dataclass
class ImuState:
    q: np.ndarray = field(default_factory=lambda: np.array([0., 0., 0., 1.]))
    p: np.ndarray = field(default_factory=lambda: np.zeros(3))
    v: np.ndarray = field(default_factory=lambda: np.zeros(3))
    bg: np.ndarray = field(default_factory=lambda: np.zeros(3))
    ba: np.ndarray = field(default_factory=lambda: np.zeros(3))
    q_null: np.ndarray = field(default_factory=lambda: np.array([0., 0., 0., 1.]))
    p_null: np.ndarray = field(default_factory=lambda: np.zeros(3))
    v_null: np.ndarray = field(default_factory=lambda: np.zeros(3))
    # Q5: after the first process_model, p_null/v_null ARE p/v (aliases), so
    # EKF corrections move them too.  Before it they are independent zeros.
    nulls_alias: bool = False
    R_imu_cam0: np.ndarray = field(default_factory=lambda: np.identity(3))
    t_cam0_imu: np.ndarray = field(default_factory=lambda: np.zeros(3))
    timestamp: Optional[float] = None
    id: Optional[int] = None

    def copy(self):
        c = ImuState(**{k: (v.copy() if isinstance(v, np.ndarray) else v)
                        for k, v in self.__dict__.items()})
        return c


@dataclass
class CamState:
    id: int
    timestamp: float
    q: np.ndarray
    p: np.ndarray           # Q5: position_null aliases p (msckf.py:400)
    q_null: np.ndarray      # augmentation-time orientation (msckf.py:399)

    def copy(self):
        return CamState(self.id, self.timestamp, self.q.copy(), self.p.copy(),
                        self.q_null.copy())


@dataclass
class FilterState:
    imu: ImuState
    cams: "OrderedDict[int, CamState]"
    P: np.ndarray
    gravity: np.ndarray
    R_cam0_cam1: np.ndarray
    t_cam0_cam1: np.ndarray
    Qc: np.ndarray
    sigma2: float           # observation noise variance

    def copy(self):
        return FilterState(self.imu.copy(),
                           OrderedDict((k, c.copy()) for k, c in self.cams.items()),
                           self.P.copy(), self.gravity.copy(), self.R_cam0_cam1,
                           self.t_cam0_cam1, self.Qc, self.sigma2)


# --------------------------------------------------------------------------
# IMU propagation                    (msckf.py:291-380, jit_utils.py:6-135)
# --------------------------------------------------------------------------


def process_model_matrices(gyro, R_w_i, acc, dt):
    """jit_utils.py:6-43 -> (F, G, Phi)."""
    F = np.zeros((21, 21))
    G = np.zeros((21, 12))
    F[:3, :3] = -skew(gyro)
    F[:3, 3:6] = -I3
    F[6:9, :3] = -R_w_i.T @ skew(acc)
    F[6:9, 9:12] = -R_w_i.T
    F[12:15, 6:9] = I3
    G[:3, :3] = -I3
    G[3:6, 3:6] = I3
    G[6:9, 6:9] = -R_w_i.T
    G[9:12, 9:12] = I3
    Fdt = F * dt
    Fdt2 = Fdt @ Fdt
    Fdt3 = Fdt2 @ Fdt
    Phi = np.identity(21) + Fdt + Fdt2 / 2. + Fdt3 / 6.
    return F, G, Phi


def predict_new_state(dt, gyro, acc, q, v, p, g):
    """jit_utils.py:46-128 -- RK4 with the reference's mixed rotations (Q1):
    the skew of the normalised dq_dt vector is reused for dR_dt2 and for the
    k1 rotation."""
    gnorm = np.linalg.norm(gyro)
    Om = np.zeros((4, 4))
    Om[:3, :3] = -skew(gyro)
    Om[:3, 3] = gyro
    Om[3, :3] = -gyro
    if gnorm > 1e-5:
        dq = (np.cos(gnorm * dt * 0.5) * I4 + np.sin(gnorm * dt * 0.5) / gnorm * Om) @ q
        dq2 = (np.cos(gnorm * dt * 0.25) * I4 + np.sin(gnorm * dt * 0.25) / gnorm * Om) @ q
    else:
        dq = np.cos(gnorm * dt * 0.5) * (I4 + Om * dt * 0.5) @ q
        dq2 = np.cos(gnorm * dt * 0.25) * (I4 + Om * dt * 0.25) @ q
    dq = dq / np.linalg.norm(dq)
    vec, w = dq[:3], dq[3]
    S1 = skew(vec)                                   # reused below (Q1)
    dR_T = ((2 * w * w - 1) * I3 - 2 * w * S1 + 2 * vec[:, None] * vec).T
    dq2 = dq2 / np.linalg.norm(dq2)
    vec, w = dq2[:3], dq2[3]
    dR2_T = ((2 * w * w - 1) * I3 - 2 * w * S1 + 2 * vec[:, None] * vec).T
    k1_p = v
    qn = q / np.linalg.norm(q)
    vec, w = qn[:3], qn[3]
    R = (2 * w * w - 1) * I3 - 2 * w * S1 + 2 * vec[:, None] * vec
    k1_v = R.T @ acc + g
    v1 = v + k1_v * dt / 2.
    k2_p = v1
    k2_v = dR2_T @ acc + g
    v2 = v + k2_v * dt / 2
    k3_p = v2
    k3_v = dR2_T @ acc + g
    v3 = v + k3_v * dt
    k4_p = v3
    k4_v = dR_T @ acc + g
    q_new = dq / np.linalg.norm(dq)
    v_new = v + (k1_v + 2 * k2_v + 2 * k3_v + k4_v) * dt / 6.
    p_new = p + (k1_p + 2 * k2_p + 2 * k3_p + k4_p) * dt / 6.
    return q_new, v_new, p_new


def process_model(st: FilterState, t, m_gyro, m_acc):
    """msckf.py:291-368 (one IMU sample).  Returns the edited Phi (for tests)."""
    imu = st.imu
    dt = t - imu.timestamp
    gyro = m_gyro - imu.bg
    acc = m_acc - imu.ba
    R_w_i = to_rotation(imu.q)
    _, G, Phi = process_model_matrices(gyro, R_w_i, acc, dt)
    # Q5: the null velocity/position are the values at entry once aliased.
    v_null = imu.v.copy() if imu.nulls_alias else imu.v_null
    p_null = imu.p.copy() if imu.nulls_alias else imu.p_null
    imu.q, imu.v, imu.p = predict_new_state(dt, gyro, acc, imu.q, imu.v, imu.p, st.gravity)
    g = st.gravity
    R_kk_1 = to_rotation(imu.q_null)
    Phi[:3, :3] = to_rotation(imu.q) @ R_kk_1.T
    u = R_kk_1 @ g
    s = u / (u @ u)
    A1 = Phi[6:9, :3]
    w1 = skew(v_null - imu.v) @ g
    Phi[6:9, :3] = A1 - (A1 @ u - w1)[:, None] * s
    A2 = Phi[12:15, :3]
    w2 = skew(dt * v_null + p_null - imu.p) @ g
    Phi[12:15, :3] = A2 - (A2 @ u - w2)[:, None] * s
    # jit_utils.py:130-135 then msckf.py:355-363
    P = st.P
    Q = Phi @ G @ st.Qc @ G.T @ Phi.T * dt
    P[:21, :21] = Phi @ P[:21, :21] @ Phi.T + Q
    if len(st.cams) > 0:
        P[:21, 21:] = Phi @ P[:21, 21:]
        P[21:, :21] = P[21:, :21] @ Phi.T
    st.P = (P + P.T) / 2.
    imu.q_null = imu.q
    imu.nulls_alias = True
    imu.v_null = imu.v
    imu.p_null = imu.p
    return Phi


def batch_imu_processing(st: FilterState, buffer: list, time_bound: float,
                         next_id: int) -> Tuple[list, int]:
    """msckf.py:262-287.  ``buffer`` holds (t, gyro, acc); returns the trimmed
    buffer and the next state id."""
    used = 0
    for (t, w, a) in buffer:
        if t < st.imu.timestamp:
            used += 1
            continue
        if t > time_bound:
            break
        process_model(st, t, w, a)
        used += 1
        st.imu.timestamp = t
    st.imu.id = next_id
    return buffer[used:], next_id + 1


# --------------------------------------------------------------------------
# State augmentation                    (msckf.py:385-407, jit_utils.py:137-167)
# --------------------------------------------------------------------------


def state_augmentation(st: FilterState, t: float, cam_id: int):
    imu = st.imu
    R_i_c = imu.R_imu_cam0
    t_c_i = imu.t_cam0_imu
    R_w_i = to_rotation(imu.q)
    R_w_c = R_i_c @ R_w_i
    t_c_w = imu.p + R_w_i.T @ t_c_i
    q = to_quaternion(R_w_c)
    st.cams[cam_id] = CamState(cam_id, t, q, t_c_w, q)
    J = np.zeros((6, 21))
    J[:3, :3] = R_i_c
    J[:3, 15:18] = I3
    J[3:6, :3] = skew(R_w_i.T @ t_c_i)
    J[3:6, 12:15] = I3
    J[3:6, 18:21] = I3
    n = st.P.shape[0]
    Pn = np.zeros((n + 6, n + 6))
    Pn[:n, :n] = st.P
    Pn[n:, :n] = J @ Pn[:21, :n]
    Pn[:n, n:] = Pn[n:, :n].T
    Pn[n:, n:] = J @ Pn[:21, :21] @ J.T
    st.P = (Pn + Pn.T) / 2.


# --------------------------------------------------------------------------
# Triangulation                                         (feature.py:33-295)
# --------------------------------------------------------------------------


@dataclass
class LMConfig:
    huber_epsilon: float = 0.01
    estimation_precision: float = 5e-7
    initial_damping: float = 1e-3
    outer_loop_max_iteration: int = 5
    inner_loop_max_iteration: int = 5
    translation_threshold: float = -1.0


def _lm_cost(T, x, z):
    """feature.py:33-55"""
    h = T.R @ np.array([x[0], x[1], 1.0]) + x[2] * T.t
    zh = h[:2] / h[2]
    return ((zh - z) ** 2).sum()


def _lm_jacobian(T, x, z, eps):
    """feature.py:57-97"""
    h = T.R @ np.array([x[0], x[1], 1.0]) + x[2] * T.t
    h1, h2, h3 = h
    W = np.zeros((3, 3))
    W[:, :2] = T.R[:, :2]
    W[:, 2] = T.t
    J = np.zeros((2, 3))
    J[0] = W[0] / h3 - W[2] * h1 / (h3 * h3)
    J[1] = W[1] / h3 - W[2] * h2 / (h3 * h3)
    r = np.array([h1 / h3, h2 / h3]) - z
    e = np.linalg.norm(r)
    w = 1.0 if e <= eps else eps / (2 * e)
    return J, r, w


def triangulate(obs: "OrderedDict[int, np.ndarray]", cams: Dict[int, CamState],
                R_cam0_cam1, t_cam0_cam1, cfg: LMConfig = LMConfig()):
    """feature.py:167-295.  ``obs`` maps cam id -> (u0, v0, u1, v1) in
    insertion order.  Returns (p_w, valid, n_solves)."""
    T_c1_c0 = Iso(R_cam0_cam1, t_cam0_cam1).inverse()
    poses, meas = [], []
    for cid, m in obs.items():
        if cid not in cams:
            continue
        meas.append(m[:2])
        meas.append(m[2:])
        c = cams[cid]
        T0 = Iso(to_rotation(c.q).T, c.p)
        poses.append(T0)
        poses.append(T0 * T_c1_c0)
    T_c0_w = poses[0]
    poses = [P.inverse() * T_c0_w for P in poses]
    # initial guess (feature.py:99-122): first meas vs the LAST cam0 view
    T12, z1, z2 = poses[-2], meas[0], meas[-2]
    m = T12.R @ np.array([*z1, 1.0])
    a = m[:2] - z2 * m[2]
    b = z2 * T12.t[2] - T12.t[:2]
    depth = a @ b / (a @ a)
    p0 = np.array([*z1, 1.0]) * depth
    x = np.array([*p0[:2], 1.0]) / p0[2]
    lam = cfg.initial_damping
    inner = outer = 0
    reduced = False            # Q2: never reset per outer iteration
    dnorm = float('inf')
    n_solves = 0
    cost = 0.0
    for T, z in zip(poses, meas):
        cost += _lm_cost(T, x, z)
    while outer < cfg.outer_loop_max_iteration and dnorm > cfg.estimation_precision:
        A = np.zeros((3, 3))
        bb = np.zeros(3)
        for T, z in zip(poses, meas):
            J, r, w = _lm_jacobian(T, x, z, cfg.huber_epsilon)
            if w == 1.0:
                A += J.T @ J
                bb += J.T @ r
            else:
                A += w * w * J.T @ J
                bb += w * w * J.T @ r
        while inner < cfg.inner_loop_max_iteration and not reduced:
            delta = np.linalg.solve(A + lam * I3, bb)
            n_solves += 1
            xn = x - delta
            dnorm = np.linalg.norm(delta)
            nc = 0.0
            for T, z in zip(poses, meas):
                nc += _lm_cost(T, xn, z)
            if nc < cost:
                reduced = True
                x = xn
                cost = nc
                lam = max(lam / 10., 1e-10)
            else:
                reduced = False
                lam = min(lam * 10., 1e12)
            inner += 1
        inner = 0
        outer += 1
    pf = np.array([*x[:2], 1.0]) / x[2]
    valid = True
    for T in poses:
        if (T.R @ pf + T.t)[2] <= 0:
            valid = False
            break
    p_w = T_c0_w.R @ pf + T_c0_w.t
    return p_w, valid, n_solves


# --------------------------------------------------------------------------
# Measurement Jacobian, nullspace, gating         (msckf.py:429-541, 606-614)
# --------------------------------------------------------------------------


def measurement_jacobian(st: FilterState, cam: CamState, p_w, z):
    """msckf.py:429-498 -> (H_x 4x6, H_f 4x3, r 4)."""
    R_w_c0 = to_rotation(cam.q)
    t_c0_w = cam.p
    R_w_c1 = st.R_cam0_cam1 @ R_w_c0
    t_c1_w = t_c0_w - R_w_c1.T @ st.t_cam0_cam1
    p_c0 = R_w_c0 @ (p_w - t_c0_w)
    p_c1 = R_w_c1 @ (p_w - t_c1_w)
    dz0 = np.zeros((4, 3))
    dz0[0, 0] = 1 / p_c0[2]
    dz0[1, 1] = 1 / p_c0[2]
    dz0[0, 2] = -p_c0[0] / (p_c0[2] * p_c0[2])
    dz0[1, 2] = -p_c0[1] / (p_c0[2] * p_c0[2])
    dz1 = np.zeros((4, 3))
    dz1[2, 0] = 1 / p_c1[2]
    dz1[3, 1] = 1 / p_c1[2]
    dz1[2, 2] = -p_c1[0] / (p_c1[2] * p_c1[2])
    dz1[3, 2] = -p_c1[1] / (p_c1[2] * p_c1[2])
    d0 = np.zeros((3, 6))
    d0[:, :3] = skew(p_c0)
    d0[:, 3:] = -R_w_c0
    d1 = np.zeros((3, 6))
    d1[:, :3] = st.R_cam0_cam1 @ skew(p_c0)
    d1[:, 3:] = -R_w_c1
    H_x = dz0 @ d0 + dz1 @ d1
    # Q3 observability constraint (p_null == p by aliasing, Q5)
    u = np.zeros(6)
    u[:3] = to_rotation(cam.q_null) @ st.gravity
    u[3:] = skew(p_w - cam.p) @ st.gravity
    H_x = H_x - (H_x @ u)[:, None] * u / (u @ u)
    H_f = -H_x[:4, 3:6]
    r = z - np.array([*p_c0[:2] / p_c0[2], *p_c1[:2] / p_c1[2]])
    return H_x, H_f, r


def feature_jacobian(st: FilterState, p_w, obs: Sequence[Tuple[int, np.ndarray]]):
    """msckf.py:500-541.  ``obs`` = [(cam_id, z)] restricted to valid cams, in
    the order the reference iterates them.  Returns (H (k x D), r (k))."""
    keys = list(st.cams.keys())
    D = 21 + 6 * len(keys)
    rows = 4 * len(obs)
    Hxj = np.zeros((rows, D))
    Hfj = np.zeros((rows, 3))
    rj = np.zeros(rows)
    for i, (cid, z) in enumerate(obs):
        Hx, Hf, r = measurement_jacobian(st, st.cams[cid], p_w, z)
        idx = keys.index(cid)
        Hxj[4 * i:4 * i + 4, 21 + 6 * idx:27 + 6 * idx] = Hx
        Hfj[4 * i:4 * i + 4] = Hf
        rj[4 * i:4 * i + 4] = r
    U = np.linalg.svd(Hfj)[0]
    A = U[:, 3:]
    return A.T @ Hxj, A.T @ rj


def gating_gamma(st: FilterState, H, r):
    """msckf.py:606-609 -> gamma."""
    S = H @ st.P @ H.T + st.sigma2 * np.identity(len(H))
    return r @ np.linalg.solve(S, r)


# --------------------------------------------------------------------------
# EKF update and covariance compaction      (msckf.py:543-604, 803-818)
# --------------------------------------------------------------------------


def measurement_update(st: FilterState, H, r):
    """msckf.py:543-604."""
    if len(H) == 0 or len(r) == 0:
        return None
    if H.shape[0] > H.shape[1]:
        Q, R = np.linalg.qr(H)
        Ht, rt = R, Q.T @ r
    else:
        Ht, rt = H, r
    P = st.P
    S = Ht @ P @ Ht.T + st.sigma2 * np.identity(len(Ht))
    K = np.linalg.solve(S, Ht @ P).T
    dx = K @ rt
    apply_correction(st, dx)
    IKH = np.identity(len(K)) - K @ Ht
    Pn = IKH @ st.P
    st.P = (Pn + Pn.T) / 2.
    return dx


def apply_correction(st: FilterState, dx):
    """msckf.py:568-595 (Q5: the aliased null position/velocity move too)."""
    imu = st.imu
    d = dx[:21]
    imu.q = quaternion_multiplication(small_angle_quaternion(d[:3]), imu.q)
    imu.bg = imu.bg + d[3:6]
    imu.v = imu.v + d[6:9]
    imu.ba = imu.ba + d[9:12]
    imu.p = imu.p + d[12:15]
    if imu.nulls_alias:
        imu.v_null = imu.v
        imu.p_null = imu.p
    imu.R_imu_cam0 = to_rotation(small_angle_quaternion(d[15:18])) @ imu.R_imu_cam0
    imu.t_cam0_imu = imu.t_cam0_imu + d[18:21]
    for i, cam in enumerate(st.cams.values()):
        dc = dx[21 + 6 * i:27 + 6 * i]
        cam.q = quaternion_multiplication(small_angle_quaternion(dc[:3]), cam.q)
        cam.p = cam.p + dc[3:]


def remove_cam_cov(st: FilterState, cam_ids: Sequence[int]):
    """msckf.py:803-818 (ascending ids, one at a time)."""
    for cid in cam_ids:
        idx = list(st.cams.keys()).index(cid)
        s, e = 21 + 6 * idx, 27 + 6 * idx
        P = st.P.copy()
        if e < P.shape[0]:
            P[s:-6, :] = P[e:, :]
            P[:, s:-6] = P[:, e:]
        st.P = P[:-6, :-6]
        del st.cams[cid]


def check_motion(obs: "OrderedDict[int, np.ndarray]", cams: Dict[int, CamState], threshold: float) -> bool:
    """feature.py:124-165: enough translation between the first and the last
    observing cam, orthogonal to the first observation's ray, to triangulate."""
    if threshold < 0:
        return True
    ids = list(obs.keys())
    c0, c1 = cams[ids[0]], cams[ids[-1]]
    R0 = to_rotation(c0.q).T
    d = np.array([*obs[ids[0]][:2], 1.0])
    d = R0 @ (d / np.linalg.norm(d))
    tr = c1.p - c0.p
    orth = tr - (tr @ d) * d
    return bool(np.linalg.norm(orth) > threshold)


def find_redundant_cam_states(st: FilterState, tracking_rate: float):
    """msckf.py:691-727."""
    pairs = list(st.cams.items())
    key = len(pairs) - 4
    ci = key + 1
    first = 0
    kp = pairs[key][1].p
    kR = to_rotation(pairs[key][1].q)
    rm = []
    for _ in range(2):
        pos = pairs[ci][1].p
        Rc = to_rotation(pairs[ci][1].q)
        dist = np.linalg.norm(pos - kp)
        ang = 2 * np.arccos(to_quaternion(Rc @ kR.T)[-1])
        if ang < 0.2618 and dist < 0.4 and tracking_rate > 0.5:
            rm.append(pairs[ci][0])
            ci += 1
        else:
            rm.append(pairs[first][0])
            first += 1
            ci += 1
    return sorted(rm)


# --------------------------------------------------------------------------
# Whole filter (reference callback semantics)           (msckf.py:104-908)
# --------------------------------------------------------------------------


class OracleFeature:
    def __init__(self, fid):
        self.id = fid
        self.observations: "OrderedDict[int, np.ndarray]" = OrderedDict()
        self.position = np.zeros(3)
        self.is_initialized = False


class OracleMSCKF:
    """The reference filter's callback API restated on top of the functions
    above.  ``cfg`` is a ``msckf_amd.FilterConfig``-like object (duck-typed
    attribute names); ``chi2`` is a callable dof -> threshold."""

    def __init__(self, cfg, chi2):
        self.cfg = cfg
        self.chi2 = chi2
        oc = cfg.optimization
        self.lm = LMConfig(oc.huber_epsilon, oc.estimation_precision,
                           oc.initial_damping, oc.outer_loop_max_iteration,
                           oc.inner_loop_max_iteration, oc.translation_threshold)
        Qc = np.identity(12)
        Qc[:3, :3] *= cfg.gyro_noise
        Qc[3:6, 3:6] *= cfg.gyro_bias_noise
        Qc[6:9, 6:9] *= cfg.acc_noise
        Qc[9:, 9:] *= cfg.acc_bias_noise
        T_cam0_imu = np.linalg.inv(cfg.T_imu_cam0)
        imu = ImuState()
        imu.v = np.array(cfg.velocity, float)
        imu.R_imu_cam0 = T_cam0_imu[:3, :3].T
        imu.t_cam0_imu = T_cam0_imu[:3, 3]
        self.st = FilterState(imu, OrderedDict(), self._initial_cov(),
                              np.array(cfg.gravity, float), cfg.T_cn_cnm1[:3, :3],
                              cfg.T_cn_cnm1[:3, 3], Qc, cfg.observation_noise)
        self.T_imu_body = Iso(cfg.T_imu_body[:3, :3], cfg.T_imu_body[:3, 3])
        self.imu_buffer: list = []
        self.map: "OrderedDict[int, OracleFeature]" = OrderedDict()
        self.next_id = 0
        self.tracking_rate = None
        self.is_gravity_set = False
        self.is_first_img = True
        self.log: List[dict] = []      # per-frame decision log (tests)
        self.gate_log: List[tuple] = []   # (frame, dof, rows, accepted)
        self.shape_log: List[tuple] = []  # (frame, H rows, H cols)
        self.n_published = 0
        self.resets: List[int] = []       # frames after which online_reset fired

    def _initial_cov(self):
        """msckf.py:820-830"""
        c = self.cfg
        P = np.zeros((21, 21))
        P[3:6, 3:6] = c.gyro_bias_cov * I3
        P[6:9, 6:9] = c.velocity_cov * I3
        P[9:12, 9:12] = c.acc_bias_cov * I3
        P[15:18, 15:18] = c.extrinsic_rotation_cov * I3
        P[18:21, 18:21] = c.extrinsic_translation_cov * I3
        return P

    def imu_callback(self, t, gyro, acc):
        """msckf.py:166-178"""
        self.imu_buffer.append((t, np.asarray(gyro, float), np.asarray(acc, float)))
        if not self.is_gravity_set and len(self.imu_buffer) >= 200:
            self._init_gravity_and_bias()
            self.is_gravity_set = True

    def _init_gravity_and_bias(self):
        """msckf.py:235-258"""
        sw = np.zeros(3)
        sa = np.zeros(3)
        for (_, w, a) in self.imu_buffer:
            sw += w
            sa += a
        self.st.imu.bg = sw / len(self.imu_buffer)
        g_imu = sa / len(self.imu_buffer)
        self.st.gravity = np.array([0., 0., -np.linalg.norm(g_imu)])
        self.st.imu.q = from_two_vectors(-self.st.gravity, g_imu)

    def feature_callback(self, t, features):
        """msckf.py:180-233.  ``features`` = iterable of (id, u0, v0, u1, v1)."""
        if not self.is_gravity_set:
            return None
        if self.is_first_img:
            self.is_first_img = False
            self.st.imu.timestamp = t
        self.imu_buffer, self.next_id = batch_imu_processing(
            self.st, self.imu_buffer, t, self.next_id)
        state_augmentation(self.st, t, self.st.imu.id)
        self._add_observations(features)
        frame = {"t": t}
        frame["lost"] = self._remove_lost_features()
        frame["prune"] = self._prune_cam_state_buffer()
        self.log.append(frame)
        try:
            return self.publish(t)
        finally:
            self.n_published += 1
            self._online_reset()

    def _add_observations(self, features):
        """msckf.py:409-427"""
        sid = self.st.imu.id
        cur = len(self.map)
        tracked = 0
        for (fid, u0, v0, u1, v1) in features:
            z = np.array([u0, v0, u1, v1])
            if fid not in self.map:
                f = OracleFeature(fid)
                f.observations[sid] = z
                self.map[fid] = f
            else:
                self.map[fid].observations[sid] = z
                tracked += 1
        self.tracking_rate = tracked / (cur + 1e-5)

    def _initialize(self, f):
        p, ok, _ = triangulate(f.observations, self.st.cams, self.st.R_cam0_cam1,
                               self.st.t_cam0_cam1, self.lm)
        f.position = p
        f.is_initialized = ok
        return ok

    def _remove_lost_features(self):
        """msckf.py:616-689"""
        sid = self.st.imu.id
        invalid, processed = [], []
        for f in self.map.values():
            if sid in f.observations:
                continue
            if len(f.observations) < 3:
                invalid.append(f.id)
                continue
            if not f.is_initialized:
                if not check_motion(f.observations, self.st.cams, self.lm.translation_threshold):
                    invalid.append(f.id)
                    continue
                if not self._initialize(f):
                    invalid.append(f.id)
                    continue
            processed.append(f.id)
        for fid in invalid:
            del self.map[fid]
        info = {"processed": list(processed), "accepted": [], "rows": 0}
        if not processed:
            return info
        Hs, rs = [], []
        count = 0
        for fid in processed:
            f = self.map[fid]
            obs = list(f.observations.items())
            H, r = feature_jacobian(self.st, f.position, obs)
            gamma = gating_gamma(self.st, H, r)
            ok = gamma < self.chi2(len(obs) - 1)
            self.gate_log.append((self.n_published, len(obs) - 1, H.shape[0], int(ok)))
            if ok:
                Hs.append(H)
                rs.append(r)
                count += H.shape[0]
                info["accepted"].append(fid)
            if count > 1500:
                break
        info["rows"] = count
        D = 21 + 6 * len(self.st.cams)
        H = np.vstack(Hs) if Hs else np.zeros((0, D))
        r = np.concatenate(rs) if rs else np.zeros(0)
        self.shape_log.append((self.n_published, H.shape[0], H.shape[1]))
        measurement_update(self.st, H, r)
        for fid in processed:
            del self.map[fid]
        return info

    def _prune_cam_state_buffer(self):
        """msckf.py:730-818"""
        if len(self.st.cams) < self.cfg.max_cam_state_size:
            return None
        rm = find_redundant_cam_states(self.st, self.tracking_rate)
        for f in self.map.values():
            inv = [c for c in rm if c in f.observations]
            if len(inv) == 0:
                continue
            if len(inv) == 1:
                del f.observations[inv[0]]
                continue
            if not f.is_initialized:
                if (not check_motion(f.observations, self.st.cams, self.lm.translation_threshold)
                        or not self._initialize(f)):
                    for c in inv:
                        del f.observations[c]
                    continue
        Hs, rs = [], []
        info = {"removed": rm, "accepted": [], "rows": 0}
        for f in self.map.values():
            inv = [c for c in rm if c in f.observations]
            if len(inv) == 0:
                continue
            obs = [(c, f.observations[c]) for c in inv]
            H, r = feature_jacobian(self.st, f.position, obs)
            gamma = gating_gamma(self.st, H, r)
            ok = gamma < self.chi2(len(inv))
            self.gate_log.append((self.n_published, len(inv), H.shape[0], int(ok)))
            if ok:
                Hs.append(H)
                rs.append(r)
                info["accepted"].append(f.id)
            for c in inv:
                del f.observations[c]
        D = 21 + 6 * len(self.st.cams)
        H = np.vstack(Hs) if Hs else np.zeros((0, D))
        r = np.concatenate(rs) if rs else np.zeros(0)
        info["rows"] = H.shape[0]
        self.shape_log.append((self.n_published, H.shape[0], H.shape[1]))
        measurement_update(self.st, H, r)
        remove_cam_cov(self.st, rm)
        return info

    def _online_reset(self):
        """msckf.py:859-886"""
        thr = self.cfg.position_std_threshold
        if thr <= 0:
            return
        P = self.st.P
        if max(np.sqrt(P[12, 12]), np.sqrt(P[13, 13]), np.sqrt(P[14, 14])) < thr:
            return
        self.st.cams.clear()
        self.map.clear()
        self.st.P = self._initial_cov()
        self.resets.append(self.n_published - 1)   # the frame just published

    def publish(self, t):
        """msckf.py:888-908 -> dict(timestamp, pose (R, t), velocity, cam0_pose)."""
        imu = self.st.imu
        T_i_w = Iso(to_rotation(imu.q).T, imu.p)
        Tb = self.T_imu_body
        T_b_w = Tb * T_i_w * Tb.inverse()
        vel = Tb.R @ imu.v
        R_w_c = imu.R_imu_cam0 @ T_i_w.R.T
        t_c_w = imu.p + T_i_w.R @ imu.t_cam0_imu
        return {"timestamp": t, "pose": Iso(T_b_w.R, T_b_w.t), "velocity": vel,
                "cam0_pose": Iso(R_w_c.T, t_c_w)}
