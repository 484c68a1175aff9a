"""Host-side SO(3) / JPL-quaternion helpers (reference MSCKF/utils.py:1-152).

Used only for host bookkeeping that stays in Python by design -- gravity
initialisation (msckf.py:235-258), keyframe selection (msckf.py:691-727) and
``publish`` (msckf.py:888-908) -- and by the synthetic generators.  The filter
arithmetic itself runs on the GPU (csrc/msckf_hip.hip has device versions).
Quaternions are JPL [x, y, z, w]; ``to_rotation(q)`` maps world -> body.
"""
import numpy as np


def skew(v):
    return np.array([[0.0, -v[2], v[1]], [v[2], 0.0, -v[0]], [-v[1], v[0], 0.0]])


def to_rotation(q):
    q = np.asarray(q, float) / np.linalg.norm(q)
    x, w = q[:3], q[3]
    return (2 * w * w - 1) * np.eye(3) - 2 * w * skew(x) + 2 * x[:, None] * x


def to_quaternion(R):
    # Same branch structure as utils.py:37-53 so the sign convention matches.
    if R[2, 2] < 0:
        if R[0, 0] > R[1, 1]:
            t = 1 + R[0, 0] - R[1, 1] - R[2, 2]
            q = (t, R[0, 1] + R[1, 0], R[2, 0] + R[0, 2], R[1, 2] - R[2, 1])
        else:
            t = 1 - R[0, 0] + R[1, 1] - R[2, 2]
            q = (R[0, 1] + R[1, 0], t, R[2, 1] + R[1, 2], R[2, 0] - R[0, 2])
    elif R[0, 0] < -R[1, 1]:
        t = 1 - R[0, 0] - R[1, 1] + R[2, 2]
        q = (R[0, 2] + R[2, 0], R[2, 1] + R[1, 2], t, R[0, 1] - R[1, 0])
    else:
        t = 1 + R[0, 0] + R[1, 1] + R[2, 2]
        q = (R[1, 2] - R[2, 1], R[2, 0] - R[0, 2], R[0, 1] - R[1, 0], t)
    q = np.array(q)
    return q / np.linalg.norm(q)


def quaternion_multiplication(q1, q2):
    a = np.asarray(q1, float) / np.linalg.norm(q1)
    b = np.asarray(q2, float) / np.linalg.norm(q2)
    L = np.array([[a[3], a[2], -a[1], a[0]],
                  [-a[2], a[3], a[0], a[1]],
                  [a[1], -a[0], a[3], a[2]],
                  [-a[0], -a[1], -a[2], a[3]]])
    q = L @ b
    return q / np.linalg.norm(q)


def from_two_vectors(v0, v1):
    """Rotation quaternion taking v0 to v1, returned in JPL convention."""
    a = v0 / np.linalg.norm(v0)
    b = v1 / np.linalg.norm(v1)
    d = a @ b
    if d < -0.999999:
        axis = np.cross([1, 0, 0], a)
        if np.linalg.norm(axis) < 0.000001:
            axis = np.cross([0, 1, 0], a)
        q = np.array([*axis, 0.0])
    elif d > 0.999999:
        q = np.array([0.0, 0.0, 0.0, 1.0])
    else:
        s = np.sqrt((1 + d) * 2)
        q = np.array([*(np.cross(a, b) / s), 0.5 * s])
    q = q / np.linalg.norm(q)
    return np.array([-q[0], -q[1], -q[2], q[3]])


class Isometry3d:
    """Rigid transform with the reference's attribute names (utils.py:132-152)."""

    def __init__(self, R, t):
        self._vio_R__ = R
        self._vio_t__ = t

    @property
    def R(self):
        return self._vio_R__

    @property
    def t(self):
        return self._vio_t__

    def matrix(self):
        m = np.identity(4)
        m[:3, :3] = self._vio_R__
        m[:3, 3] = self._vio_t__
        return m

    def inverse(self):
        return Isometry3d(self._vio_R__.T, -self._vio_R__.T @ self._vio_t__)

    def __mul__(self, o):
        return Isometry3d(self._vio_R__ @ o._vio_R__, self._vio_R__ @ o._vio_t__ + self._vio_t__)
