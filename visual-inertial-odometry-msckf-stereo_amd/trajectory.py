"""Trajectory evaluation: absolute trajectory error.

The reference reports no accuracy figure of its own (its ground-truth reader
cannot even open the file, dataset.py:41 passes mode '_vio_r__'); BASELINE's
metric names "ATE RMSE vs ref".  Two numbers are computed the usual way:

* ATE vs ground truth -- estimated positions associated to ground-truth
  samples by timestamp, aligned with the closed-form least-squares SE(3)
  (or Sim(3)) transform of Umeyama (1991), RMSE of the residual positions;
* ATE vs ref -- the same between this filter's trajectory and the reference
  filter's trajectory on the same replayed input (identical timestamps).

Plain numpy (host-side evaluation, not part of the filter path).
"""
from __future__ import annotations

from dataclasses import dataclass, field

import numpy as np


@dataclass
class Trajectory:
    """Timestamped body positions (K, 3) and, optionally, body->world
    rotations (K, 3, 3)."""
    t: np.ndarray
    p: np.ndarray
    R: np.ndarray | None = None
    meta: dict = field(default_factory=dict)

    def __len__(self):
        return len(self.t)

    @staticmethod
    def from_results(results):
        """From a list of ``vio_result`` (msckf.py:902-908): pose = body in world."""
        t = np.array([r.timestamp for r in results], float)
        p = np.array([r.pose._vio_t__ for r in results], float).reshape(-1, 3)
        R = np.array([r.pose._vio_R__ for r in results], float).reshape(-1, 3, 3)
        return Trajectory(t, p, R)


def associate(t_est, t_ref, max_dt=0.02):
    """Nearest-timestamp association of two sorted time series.  Returns index
    arrays (i_est, i_ref) of the pairs closer than ``max_dt`` seconds."""
    t_est = np.asarray(t_est, float)
    t_ref = np.asarray(t_ref, float)
    if len(t_est) == 0 or len(t_ref) == 0:
        return np.zeros(0, int), np.zeros(0, int)
    j = np.searchsorted(t_ref, t_est)
    j0 = np.clip(j - 1, 0, len(t_ref) - 1)
    j1 = np.clip(j, 0, len(t_ref) - 1)
    pick = np.where(np.abs(t_ref[j0] - t_est) <= np.abs(t_ref[j1] - t_est), j0, j1)
    ok = np.abs(t_ref[pick] - t_est) <= max_dt
    return np.flatnonzero(ok), pick[ok]


def umeyama(src, dst, with_scale=False):
    """Least-squares similarity transform dst ~ s R src + t (Umeyama 1991).
    src, dst: (K, 3).  Returns (R, t, s); s = 1 unless ``with_scale``."""
    src = np.asarray(src, float)
    dst = np.asarray(dst, float)
    if src.shape != dst.shape or src.ndim != 2 or src.shape[1] != 3:
        raise ValueError("umeyama: src and dst must both be (K, 3)")
    if len(src) < 3:
        raise ValueError("umeyama: need at least 3 point pairs")
    mu_s = src.mean(0)
    mu_d = dst.mean(0)
    xs = src - mu_s
    xd = dst - mu_d
    cov = xd.T @ xs / len(src)
    U, d, Vt = np.linalg.svd(cov)
    S = np.eye(3)
    if np.linalg.det(U) * np.linalg.det(Vt) < 0:
        S[2, 2] = -1.0
    R = U @ S @ Vt
    s = 1.0
    if with_scale:
        var_s = (xs ** 2).sum() / len(src)
        s = float(np.trace(np.diag(d) @ S) / var_s)
    t = mu_d - s * R @ mu_s
    return R, t, s


def ate_rmse(est_p, ref_p, align="se3"):
    """RMSE of the position residual after aligning ``est_p`` onto ``ref_p``
    ("se3", "sim3" or "none").  Both (K, 3), already associated."""
    est_p = np.asarray(est_p, float)
    ref_p = np.asarray(ref_p, float)
    if align == "none":
        e = est_p - ref_p
    else:
        R, t, s = umeyama(est_p, ref_p, with_scale=(align == "sim3"))
        e = (s * est_p @ R.T + t) - ref_p
    return float(np.sqrt(np.mean(np.sum(e * e, axis=1))))


def ate(est: Trajectory, ref: Trajectory, align="se3", max_dt=0.02, skip=0):
    """ATE RMSE of ``est`` against ``ref`` (ground truth or a reference run).
    ``skip`` drops the first estimated poses (e.g. before initialisation)."""
    i, j = associate(est.t[skip:], ref.t, max_dt)
    i = i + skip
    if len(i) < 3:
        raise ValueError("ate: fewer than 3 associated poses")
    return ate_rmse(est.p[i], ref.p[j], align)
