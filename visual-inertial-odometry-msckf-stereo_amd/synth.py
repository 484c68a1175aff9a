"""Synthetic workloads (no datasets are reachable: no network).

* ``make_update_problem`` -- the fixed-shape EKF measurement-update problem of
  SURVEY.md section 8(d): N cam states, F features with contiguous tracks,
  exact stereo projections + pixel noise, random SPD covariance.
* ``make_sequence`` -- a deterministic stereo + IMU stream (static start for
  the reference's 200-sample gravity/bias initialisation, msckf.py:175-178),
  emitted as the reference's message tuples (imu_msg: dataset.py:56-57,
  feature_msg: image.py:436-437) so the same stream drives the reference
  filter, the oracle and this package.

All randomness is ``numpy.random.default_rng(seed)``.
"""
from __future__ import annotations

from collections import namedtuple
from dataclasses import dataclass
from typing import List

import numpy as np

from .config import FilterConfig
from .geometry import skew, to_rotation, to_quaternion, quaternion_multiplication

ImuMsg = namedtuple("imu_msg", ["vio_timestamp__", "angular_velocity", "linear_acceleration"])
FeatureMsg = namedtuple("vio_feature_msg__", ["timestamp", "vio_features"])


class FeatureMeasurement:
    """Same attributes as the reference front-end's message (image.py:23-32)."""
    __slots__ = ("id", "u0", "v0", "u1", "v1")

    def __init__(self, fid, u0, v0, u1, v1):
        self.id, self.u0, self.v0, self.u1, self.v1 = fid, u0, v0, u1, v1


def _expmap(w):
    th = np.linalg.norm(w)
    K = skew(w / th) if th > 0 else np.zeros((3, 3))
    return np.eye(3) + np.sin(th) * K + (1 - np.cos(th)) * K @ K


# --------------------------------------------------------------------------
# Fixed-shape update problem
# --------------------------------------------------------------------------


@dataclass
class UpdateProblem:
    N: int
    F: int
    cam_q: np.ndarray        # (N, 4) JPL, world->cam0
    cam_p: np.ndarray        # (N, 3) cam0 position in world
    cam_q_null: np.ndarray   # (N, 4) first-estimate orientation
    imu: dict                # q, p, v, bg, ba, q_null, p_null, v_null, R_imu_cam0, t_cam0_imu
    P: np.ndarray            # (D, D)
    gravity: np.ndarray
    R_cam0_cam1: np.ndarray
    t_cam0_cam1: np.ndarray
    landmarks: np.ndarray    # (F, 3) ground truth
    obs_off: np.ndarray      # (F+1,) int32 offsets into the observation rows
    obs_cam: np.ndarray      # (sum M,) int32 cam slot of each observation
    obs_z: np.ndarray        # (sum M, 4) (u0, v0, u1, v1)

    @property
    def D(self):
        return 21 + 6 * self.N

    def track_lengths(self):
        return np.diff(self.obs_off)


def make_update_problem(N=30, F=200, seed=0, full_tracks=False,
                        cfg: FilterConfig | None = None) -> UpdateProblem:
    cfg = cfg or FilterConfig()
    rng = np.random.default_rng(seed)
    Rcc = cfg.T_cn_cnm1[:3, :3]
    tcc = cfg.T_cn_cnm1[:3, 3]
    T_cam0_imu = np.linalg.inv(cfg.T_imu_cam0)
    i = np.arange(N)
    cam_p = np.stack([0.05 * i, 0.01 * np.sin(i), np.zeros(N)], 1) + 0.005 * rng.standard_normal((N, 3))
    cam_R = [_expmap(0.02 * rng.standard_normal(3)) for _ in range(N)]
    cam_q = np.stack([to_quaternion(R) for R in cam_R])
    cam_q_null = np.stack([quaternion_multiplication(
        to_quaternion(_expmap(1e-3 * rng.standard_normal(3))), q) for q in cam_q])
    lo, hi = np.array([-1.5, -1.5, 3.0]), np.array([3.0, 1.5, 8.0])
    L = lo + (hi - lo) * rng.random((F, 3))
    if full_tracks:
        M = np.full(F, N)
        start = np.zeros(F, int)
    else:
        M = rng.integers(3, N + 1, size=F)
        start = np.array([rng.integers(0, N - m + 1) for m in M])
    off = np.zeros(F + 1, np.int32)
    off[1:] = np.cumsum(M)
    cams = np.concatenate([np.arange(s, s + m) for s, m in zip(start, M)]).astype(np.int32)
    sig = 0.5 / 458.654
    z = np.empty((len(cams), 4))
    for f in range(F):
        for r in range(off[f], off[f + 1]):
            c = cams[r]
            R0 = cam_R[c]
            pc0 = R0 @ (L[f] - cam_p[c])
            R1 = Rcc @ R0
            pc1 = R1 @ (L[f] - (cam_p[c] - R1.T @ tcc))
            z[r] = [pc0[0] / pc0[2], pc0[1] / pc0[2], pc1[0] / pc1[2], pc1[1] / pc1[2]]
    z += sig * rng.standard_normal(z.shape)
    D = 21 + 6 * N
    A = 0.01 * rng.standard_normal((D, D))
    P = A @ A.T + 1e-4 * np.eye(D)
    q_imu = to_quaternion(_expmap(0.1 * rng.standard_normal(3)))
    imu = dict(q=q_imu, p=0.1 * rng.standard_normal(3), v=0.1 * rng.standard_normal(3),
               bg=1e-3 * rng.standard_normal(3), ba=1e-2 * rng.standard_normal(3),
               q_null=q_imu.copy(), p_null=np.zeros(3), v_null=np.zeros(3),
               R_imu_cam0=T_cam0_imu[:3, :3].T.copy(), t_cam0_imu=T_cam0_imu[:3, 3].copy())
    return UpdateProblem(N, F, cam_q, cam_p, cam_q_null, imu, P, np.array(cfg.gravity, float),
                         Rcc.copy(), tcc.copy(), L, off, cams, z)


# --------------------------------------------------------------------------
# Stereo + IMU stream
# --------------------------------------------------------------------------

# IMU -> world base attitude: IMU x up (world z), IMU z (camera optical axis,
# config.py:94-98) forward (world x).
_R0 = np.array([[0., 0., 1.], [0., -1., 0.], [1., 0., 0.]])


def _ramp(t, t0, tau=1.0):
    s = np.clip((t - t0) / tau, 0.0, 1.0)
    return s * s * s * (10 - 15 * s + 6 * s * s)


def _traj(t, t0):
    """(p, R_i_w) of the IMU at time t; static before t0."""
    s = _ramp(t, t0)
    tt = t - t0
    p = s * np.array([0.3 * np.sin(0.4 * tt), 1.2 * np.sin(0.5 * tt), 0.4 * np.sin(0.7 * tt)])
    roll = s * 0.15 * np.sin(0.9 * tt)
    pitch = s * 0.10 * np.sin(0.6 * tt + 0.3)
    yaw = s * 0.20 * np.sin(0.45 * tt)
    cr, sr, cp, sp, cy, sy = np.cos(roll), np.sin(roll), np.cos(pitch), np.sin(pitch), np.cos(yaw), np.sin(yaw)
    Rz = np.array([[cy, -sy, 0], [sy, cy, 0], [0, 0, 1]])
    Ry = np.array([[cp, 0, sp], [0, 1, 0], [-sp, 0, cp]])
    Rx = np.array([[1, 0, 0], [0, cr, -sr], [0, sr, cr]])
    return p, Rz @ Ry @ Rx @ _R0


@dataclass
class Sequence:
    imu: List[ImuMsg]
    frames: List[FeatureMsg]
    gt_t: np.ndarray          # (K,) frame times
    gt_p: np.ndarray          # (K, 3) true IMU positions at frame times
    gt_R: np.ndarray          # (K, 3, 3) true IMU->world rotations

    def events(self):
        """Messages merged in strict time order (IMU first on ties), the
        deterministic replay the reference harness lacks."""
        ev = [(m.vio_timestamp__, 0, m) for m in self.imu] + \
             [(f.timestamp, 1, f) for f in self.frames]
        ev.sort(key=lambda e: (e[0], e[1]))
        return [(kind, m) for (_, kind, m) in ev]


def make_sequence(n_frames=120, seed=0, imu_rate=200.0, cam_rate=20.0, static_s=1.2,
                  n_landmarks=600, max_features=150, drop_prob=0.03,
                  gyro_sigma=1e-3, acc_sigma=1e-2, pix_sigma=0.5 / 458.654,
                  cfg: FilterConfig | None = None, t_start=100.0) -> Sequence:
    cfg = cfg or FilterConfig()
    rng = np.random.default_rng(seed)
    g = np.array([0.0, 0.0, -9.81])
    R_ic = cfg.T_imu_cam0[:3, :3]      # IMU -> cam0 (config.py:91-98)
    t_ic = cfg.T_imu_cam0[:3, 3]
    Rcc = cfg.T_cn_cnm1[:3, :3]
    tcc = cfg.T_cn_cnm1[:3, 3]
    t0 = t_start + static_s
    t_end = t_start + static_s + n_frames / cam_rate
    h = 1e-4

    imu = []
    n_imu = int(np.floor((t_end - t_start) * imu_rate)) + 1
    for k in range(n_imu):
        t = t_start + k / imu_rate
        p_m, R_m = _traj(t - h, t0)
        p_0, R_0 = _traj(t, t0)
        p_p, R_p = _traj(t + h, t0)
        acc_w = (p_p - 2 * p_0 + p_m) / (h * h)
        Rdot = (R_p - R_m) / (2 * h)
        W = R_0.T @ Rdot
        w = np.array([W[2, 1] - W[1, 2], W[0, 2] - W[2, 0], W[1, 0] - W[0, 1]]) / 2
        a = R_0.T @ (acc_w - g)
        imu.append(ImuMsg(t, w + gyro_sigma * rng.standard_normal(3),
                          a + acc_sigma * rng.standard_normal(3)))

    lo = np.array([3.0, -4.0, -2.5])
    hi = np.array([8.0, 4.0, 2.5])
    L = lo + (hi - lo) * rng.random((n_landmarks, 3))
    frames, gt_t, gt_p, gt_R = [], [], [], []
    track_id = -np.ones(n_landmarks, int)
    next_id = 0
    n_cam = int(np.floor((t_end - t_start) * cam_rate))
    for k in range(n_cam):
        t = t_start + k / cam_rate                    # on an IMU tick
        p_i, R_iw = _traj(t, t0)
        R_w_c0 = R_ic @ R_iw.T                        # world -> cam0
        t_c0 = p_i + R_iw @ (-R_ic.T @ t_ic)          # cam0 centre in world
        R_w_c1 = Rcc @ R_w_c0
        t_c1 = t_c0 - R_w_c1.T @ tcc
        pc0 = (L - t_c0) @ R_w_c0.T
        pc1 = (L - t_c1) @ R_w_c1.T
        with np.errstate(divide="ignore", invalid="ignore"):
            u0, v0 = pc0[:, 0] / pc0[:, 2], pc0[:, 1] / pc0[:, 2]
            u1, v1 = pc1[:, 0] / pc1[:, 2], pc1[:, 1] / pc1[:, 2]
        vis = (pc0[:, 2] > 0.5) & (pc1[:, 2] > 0.5) & (np.abs(u0) < 0.75) & (np.abs(v0) < 0.5) \
            & (np.abs(u1) < 0.75) & (np.abs(v1) < 0.5)
        # tracks die when the landmark leaves view or at random (KLT loss)
        die = (~vis) | (rng.random(n_landmarks) < drop_prob)
        track_id[die & (track_id >= 0)] = -1
        cand = np.flatnonzero(vis)
        alive = cand[track_id[cand] >= 0]
        new = cand[track_id[cand] < 0]
        room = max(0, max_features - len(alive))
        if len(new) > room:
            new = rng.choice(new, room, replace=False)
        for j in np.sort(new):
            track_id[j] = next_id
            next_id += 1
        sel = np.sort(np.concatenate([alive, new])).astype(int)
        n = pix_sigma * rng.standard_normal((len(sel), 4))
        feats = [FeatureMeasurement(int(track_id[j]), u0[j] + n[q, 0], v0[j] + n[q, 1],
                                    u1[j] + n[q, 2], v1[j] + n[q, 3]) for q, j in enumerate(sel)]
        feats.sort(key=lambda f: f.id)
        frames.append(FeatureMsg(t, feats))
        gt_t.append(t)
        gt_p.append(p_i)
        gt_R.append(R_iw)
    return Sequence(imu, frames, np.array(gt_t), np.array(gt_p), np.array(gt_R))
