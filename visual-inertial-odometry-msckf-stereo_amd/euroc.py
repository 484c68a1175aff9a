"""EuRoC MAV dataset readers.

Restates the reference's readers (MSCKF/dataset.py) without their runtime
baggage (cv2 image loading, preload threads, wall-clock publishers):

* ``read_imu_csv``  -- ``mav0/imu0/data.csv``: t [ns], w_RS_S (3) [rad/s],
  a_RS_S (3) [m/s^2]; time scaled by 1e-9 (IMUDataReader, dataset.py:50-77,
  EuRoCDataset dataset.py:198-201);
* ``read_groundtruth_csv`` -- ``mav0/state_groundtruth_estimate0/data.csv``:
  t, p_RS_R (3), q_RS (w, x, y, z), v_RS_R (3), b_w (3), b_a (3)
  (GroundTruthReader.parse, dataset.py:19-38).  The reference's own reader
  opens the file with mode '_vio_r__' (dataset.py:41) and cannot run; this one
  reads it;
* ``list_images`` -- ``mav0/cam{0,1}/data/*.png`` sorted by their ns stamps
  (EuRoCDataset.list_imgs, dataset.py:217-221);
* ``EuRoC`` -- the dataset object: start time = max(first IMU stamp,
  Stereo.start_time()), and the reference's Stereo.start_time() returns the
  cam0 reader's *starttime* (-inf until set, dataset.py:180-181), so the start
  is the first IMU stamp; ``set_starttime(offset)`` shifts every stream
  (dataset.py:210-215; vio.py:88 uses offset 40 s).

Images are listed, never decoded: the stereo front-end (image.py) stays
outside this package (north star).  Its output is recorded into a replay
stream (``replay.Recorder``) wherever the front-end runs.
"""
from __future__ import annotations

import os
from collections import namedtuple

import numpy as np

from .synth import ImuMsg
from .trajectory import Trajectory

GtMsg = namedtuple("gt_msg", ["vio_timestamp__", "vio_p__", "vio_q__", "vio_v__", "bw_", "ba_"])


def _read_csv(path, ncols):
    rows = []
    with open(path, "r") as fh:
        next(fh)                                   # header line (dataset.py:42, 71)
        for line in fh:
            line = line.strip()
            if not line:
                continue
            vals = [float(x) for x in line.split(",")]
            if len(vals) < ncols:
                raise ValueError("%s: expected %d columns, got %d" % (path, ncols, len(vals)))
            rows.append(vals[:ncols])
    return np.array(rows, float).reshape(-1, ncols)


def read_imu_csv(path, scaler=1e-9):
    """(n, 7) array: t [s], w (3), a (3)."""
    a = _read_csv(path, 7)
    a[:, 0] *= scaler
    return a


def read_groundtruth_csv(path, scaler=1e-9):
    """(n, 17) array: t [s], p (3), q (w, x, y, z), v (3), bw (3), ba (3)."""
    a = _read_csv(path, 17)
    a[:, 0] *= scaler
    return a


def quat_wxyz_to_rotation(q):
    """Hamilton (w, x, y, z) -> rotation matrices (..., 3, 3) (EuRoC q_RS:
    body S -> world R)."""
    q = np.asarray(q, float)
    q = q / np.linalg.norm(q, axis=-1, keepdims=True)
    w, x, y, z = q[..., 0], q[..., 1], q[..., 2], q[..., 3]
    R = np.empty(q.shape[:-1] + (3, 3))
    R[..., 0, 0] = 1 - 2 * (y * y + z * z)
    R[..., 0, 1] = 2 * (x * y - z * w)
    R[..., 0, 2] = 2 * (x * z + y * w)
    R[..., 1, 0] = 2 * (x * y + z * w)
    R[..., 1, 1] = 1 - 2 * (x * x + z * z)
    R[..., 1, 2] = 2 * (y * z - x * w)
    R[..., 2, 0] = 2 * (x * z - y * w)
    R[..., 2, 1] = 2 * (y * z + x * w)
    R[..., 2, 2] = 1 - 2 * (x * x + y * y)
    return R


def list_images(dirpath, scaler=1e-9):
    """(paths, timestamps [s]) of the ``*.png`` files, sorted by stamp."""
    names = [n for n in os.listdir(dirpath) if n.endswith(".png")]
    names.sort(key=lambda n: float(n[:-4]))
    return [os.path.join(dirpath, n) for n in names], [float(n[:-4]) * scaler for n in names]


class EuRoC:
    """One EuRoC sequence directory (the one holding ``mav0/``)."""

    def __init__(self, path):
        self.path = path
        mav = os.path.join(path, "mav0")
        self.imu_path = os.path.join(mav, "imu0", "data.csv")
        self.gt_path = os.path.join(mav, "state_groundtruth_estimate0", "data.csv")
        self.imu = read_imu_csv(self.imu_path)
        self.cam0_paths, self.cam0_t = ([], [])
        self.cam1_paths, self.cam1_t = ([], [])
        for k in (0, 1):
            d = os.path.join(mav, "cam%d" % k, "data")
            if os.path.isdir(d):
                paths, ts = list_images(d)
                setattr(self, "cam%d_paths" % k, paths)
                setattr(self, "cam%d_t" % k, ts)
        if len(self.cam0_t) != len(self.cam1_t):
            raise ValueError("EuRoC: cam0 has %d images, cam1 %d (Stereo asserts equal, dataset.py:164)"
                             % (len(self.cam0_t), len(self.cam1_t)))
        for a, b in zip(self.cam0_t, self.cam1_t):
            if abs(a - b) >= 0.01:
                raise ValueError("EuRoC: unsynced stereo pair (dataset.py:174)")
        self.gt = read_groundtruth_csv(self.gt_path) if os.path.exists(self.gt_path) else None
        first_imu = self.imu[0, 0] if len(self.imu) else -np.inf
        self.starttime = max(first_imu, -np.inf)     # dataset.py:207 (see module docstring)
        self.offset = 0.0

    def set_starttime(self, offset):
        """dataset.py:210-215: every stream starts at starttime + offset."""
        self.offset = float(offset)

    @property
    def t0(self):
        return self.starttime + self.offset

    def imu_msgs(self):
        """imu_msg tuples (dataset.py:56-57) from the start time on."""
        for row in self.imu[self.imu[:, 0] >= self.t0]:
            yield ImuMsg(row[0], row[1:4].copy(), row[4:7].copy())

    def stereo_timestamps(self):
        return [t for t in self.cam0_t if t >= self.t0]

    def groundtruth_msgs(self):
        if self.gt is None:
            return
        for row in self.gt[self.gt[:, 0] >= self.t0]:
            yield GtMsg(row[0], row[1:4].copy(), row[4:8].copy(), row[8:11].copy(), row[11:14].copy(),
                        row[14:17].copy())

    def groundtruth(self) -> Trajectory:
        if self.gt is None:
            raise FileNotFoundError(self.gt_path)
        g = self.gt[self.gt[:, 0] >= self.t0]
        return Trajectory(g[:, 0].copy(), g[:, 1:4].copy(), quat_wxyz_to_rotation(g[:, 4:8]),
                          meta={"source": self.gt_path})


def write_euroc_layout(root, imu, gt=None, cam_t=None):
    """Writes the EuRoC directory layout (CSV headers as the dataset ships
    them) -- used to build test fixtures and synthetic sequences in the same
    format the loader reads.  imu: (n, 7) with t in s; gt: (n, 17); cam_t:
    image stamps in s (empty placeholder pngs)."""
    mav = os.path.join(root, "mav0")
    os.makedirs(os.path.join(mav, "imu0"), exist_ok=True)
    with open(os.path.join(mav, "imu0", "data.csv"), "w") as fh:
        fh.write("#timestamp [ns],w_RS_S_x [rad s^-1],w_RS_S_y [rad s^-1],w_RS_S_z [rad s^-1],"
                 "a_RS_S_x [m s^-2],a_RS_S_y [m s^-2],a_RS_S_z [m s^-2]\n")
        for r in imu:
            fh.write("%d,%s\n" % (int(round(r[0] * 1e9)), ",".join(repr(float(x)) for x in r[1:7])))
    if gt is not None:
        os.makedirs(os.path.join(mav, "state_groundtruth_estimate0"), exist_ok=True)
        with open(os.path.join(mav, "state_groundtruth_estimate0", "data.csv"), "w") as fh:
            fh.write("#timestamp, p_RS_R_x [m], p_RS_R_y [m], p_RS_R_z [m], q_RS_w [], q_RS_x [], q_RS_y [], "
                     "q_RS_z [], v_RS_R_x [m s^-1], v_RS_R_y [m s^-1], v_RS_R_z [m s^-1], b_w_RS_S_x [rad s^-1], "
                     "b_w_RS_S_y [rad s^-1], b_w_RS_S_z [rad s^-1], b_a_RS_S_x [m s^-2], b_a_RS_S_y [m s^-2], "
                     "b_a_RS_S_z [m s^-2]\n")
            for r in gt:
                fh.write("%d,%s\n" % (int(round(r[0] * 1e9)), ",".join(repr(float(x)) for x in r[1:17])))
    if cam_t is not None:
        for k in (0, 1):
            d = os.path.join(mav, "cam%d" % k, "data")
            os.makedirs(d, exist_ok=True)
            for t in cam_t:
                open(os.path.join(d, "%d.png" % int(round(t * 1e9))), "wb").close()
    return root
