"""Deterministic replay of a recorded stereo-feature + IMU stream
(SURVEY.md 8(f) item 1).

The reference harness is real-time paced and threaded: two publisher threads
sleep on the wall clock at a 0.4 ratio (dataset.py:250-271, vio.py:100), and
the IMU thread and the vio thread call the filter without a lock
(vio.py:46-65), so which IMU samples a frame sees depends on scheduling.  This
module fixes the order: every message is delivered in strict timestamp order,
IMU samples before a frame of the same stamp -- the order in which
``batch_imu_processing`` (msckf.py:262-287) consumes samples up to and
including the image time when the IMU thread is ahead.  The same stream then
drives the reference filter, the oracle and this package to comparable
trajectories.

Stream format (one ``.npz``, no pickles; or a directory of two CSV files):

  imu        float64 (n_imu, 7)     t [s], w (3) [rad/s], a (3) [m/s^2]
  frame_t    float64 (n_frames,)    image stamps [s]
  frame_off  int64   (n_frames+1,)  frame k owns feature rows [off[k], off[k+1])
  feat_id    int64   (n_rows,)      feature id (image.py:215, 388: unique, increasing)
  feat_z     float64 (n_rows, 4)    u0 v0 u1 v1, undistorted normalised coordinates
                                    of cam0 / cam1 (image.py:640-674)
  gt_t, gt_p, gt_R  (optional)      ground-truth body trajectory
  meta       JSON text              free-form (sequence name, source, config)

CSV form: ``imu.csv`` (t,wx,wy,wz,ax,ay,az) and ``features.csv``
(t,id,u0,v0,u1,v1; a frame with no features is one row with id -1).
"""
from __future__ import annotations

import json
import os
from dataclasses import dataclass, field

import numpy as np

from .synth import FeatureMeasurement, FeatureMsg, ImuMsg
from .trajectory import Trajectory


@dataclass
class FeatureStream:
    imu: np.ndarray
    frame_t: np.ndarray
    frame_off: np.ndarray
    feat_id: np.ndarray
    feat_z: np.ndarray
    gt: Trajectory | None = None
    meta: dict = field(default_factory=dict)

    # ------------------------------------------------------------ checks --
    def validate(self):
        imu, ft, off = self.imu, self.frame_t, self.frame_off
        if imu.ndim != 2 or imu.shape[1] != 7:
            raise ValueError("imu must be (n, 7)")
        if off.shape != (len(ft) + 1,) or off[0] != 0 or off[-1] != len(self.feat_id):
            raise ValueError("frame_off must be (n_frames + 1,) from 0 to n_rows")
        if np.any(np.diff(off) < 0):
            raise ValueError("frame_off must be non-decreasing")
        if self.feat_z.shape != (len(self.feat_id), 4):
            raise ValueError("feat_z must be (n_rows, 4)")
        if np.any(np.diff(imu[:, 0]) < 0) or np.any(np.diff(ft) < 0):
            raise ValueError("imu and frame stamps must be sorted")
        return self

    @property
    def n_frames(self):
        return len(self.frame_t)

    # ----------------------------------------------------------- messages --
    def imu_msgs(self):
        return [ImuMsg(r[0], r[1:4].copy(), r[4:7].copy()) for r in self.imu]

    def frame_msg(self, k):
        a, b = int(self.frame_off[k]), int(self.frame_off[k + 1])
        z = self.feat_z
        feats = [FeatureMeasurement(int(self.feat_id[i]), z[i, 0], z[i, 1], z[i, 2], z[i, 3])
                 for i in range(a, b)]
        return FeatureMsg(float(self.frame_t[k]), feats)

    def messages(self):
        """(IMU messages, frame messages) of the whole stream: the front-end's
        output, built once (a timed replay leaves their construction out)."""
        return self.imu_msgs(), [self.frame_msg(k) for k in range(self.n_frames)]

    def events(self):
        """(kind, msg) in strict time order, IMU first on ties; kind 0 = IMU,
        1 = frame."""
        ti = self.imu[:, 0]
        out, i = [], 0
        for k in range(self.n_frames):
            t = self.frame_t[k]
            j = int(np.searchsorted(ti, t, side="right"))
            for r in self.imu[i:j]:
                out.append((0, ImuMsg(r[0], r[1:4].copy(), r[4:7].copy())))
            i = j
            out.append((1, self.frame_msg(k)))
        for r in self.imu[i:]:
            out.append((0, ImuMsg(r[0], r[1:4].copy(), r[4:7].copy())))
        return out

    # ------------------------------------------------------- constructors --
    @staticmethod
    def from_messages(imu_msgs, feature_msgs, gt: Trajectory | None = None, meta=None):
        imu = np.array([[m.vio_timestamp__, *m.angular_velocity, *m.linear_acceleration] for m in imu_msgs],
                       float).reshape(-1, 7)
        ft, off, ids, zs = [], [0], [], []
        for fm in feature_msgs:
            ft.append(fm.timestamp)
            for f in fm.vio_features:
                ids.append(int(f.id))
                zs.append((f.u0, f.v0, f.u1, f.v1))
            off.append(len(ids))
        return FeatureStream(imu, np.array(ft, float), np.array(off, np.int64), np.array(ids, np.int64),
                             np.array(zs, float).reshape(-1, 4), gt, dict(meta or {})).validate()

    @staticmethod
    def from_synthetic(seq, meta=None):
        """From ``synth.Sequence`` (ground truth included)."""
        gt = Trajectory(np.asarray(seq.gt_t, float), np.asarray(seq.gt_p, float), np.asarray(seq.gt_R, float))
        return FeatureStream.from_messages(seq.imu, seq.frames, gt, meta)

    # ---------------------------------------------------------------- I/O --
    def save(self, path):
        arrs = dict(imu=self.imu, frame_t=self.frame_t, frame_off=self.frame_off, feat_id=self.feat_id,
                    feat_z=self.feat_z, meta=np.array(json.dumps(self.meta)))
        if self.gt is not None:
            arrs.update(gt_t=self.gt.t, gt_p=self.gt.p)
            if self.gt.R is not None:
                arrs["gt_R"] = self.gt.R
        np.savez_compressed(path, **arrs)
        return path

    @staticmethod
    def load(path):
        with np.load(path, allow_pickle=False) as d:
            gt = None
            if "gt_t" in d.files:
                gt = Trajectory(d["gt_t"], d["gt_p"], d["gt_R"] if "gt_R" in d.files else None)
            meta = json.loads(str(d["meta"])) if "meta" in d.files else {}
            return FeatureStream(d["imu"], d["frame_t"], d["frame_off"].astype(np.int64),
                                 d["feat_id"].astype(np.int64), d["feat_z"], gt, meta).validate()

    def save_csv(self, dirpath):
        os.makedirs(dirpath, exist_ok=True)
        with open(os.path.join(dirpath, "imu.csv"), "w") as fh:
            fh.write("t,wx,wy,wz,ax,ay,az\n")
            for r in self.imu:
                fh.write(",".join(repr(float(x)) for x in r) + "\n")
        with open(os.path.join(dirpath, "features.csv"), "w") as fh:
            fh.write("t,id,u0,v0,u1,v1\n")
            for k in range(self.n_frames):
                t = repr(float(self.frame_t[k]))
                a, b = int(self.frame_off[k]), int(self.frame_off[k + 1])
                if a == b:
                    fh.write("%s,-1,0,0,0,0\n" % t)
                for i in range(a, b):
                    fh.write("%s,%d,%s\n" % (t, int(self.feat_id[i]), ",".join(repr(float(x)) for x in self.feat_z[i])))
        return dirpath

    @staticmethod
    def load_csv(dirpath):
        imu = np.loadtxt(os.path.join(dirpath, "imu.csv"), delimiter=",", skiprows=1, ndmin=2)
        rows = np.loadtxt(os.path.join(dirpath, "features.csv"), delimiter=",", skiprows=1, ndmin=2)
        ft, off, ids, zs = [], [0], [], []
        k = 0
        while k < len(rows):
            t = rows[k, 0]
            j = k
            while j < len(rows) and rows[j, 0] == t:
                if rows[j, 1] >= 0:
                    ids.append(int(rows[j, 1]))
                    zs.append(rows[j, 2:6])
                j += 1
            ft.append(t)
            off.append(len(ids))
            k = j
        return FeatureStream(imu.reshape(-1, 7), np.array(ft, float), np.array(off, np.int64),
                             np.array(ids, np.int64), np.array(zs, float).reshape(-1, 4)).validate()


class Recorder:
    """Stands in for the filter in the reference harness (``VIO.msckf``,
    vio.py:19) wherever the stereo front-end runs: records the messages it is
    fed, then ``stream()`` returns them in the replay format."""

    def __init__(self):
        self.imu, self.frames = [], []

    def imu_callback(self, imu_msg):
        self.imu.append(imu_msg)

    def feature_callback(self, feature_msg):
        self.frames.append(feature_msg)
        return None

    def stream(self, gt=None, meta=None):
        imu = sorted(self.imu, key=lambda m: m.vio_timestamp__)
        frames = sorted(self.frames, key=lambda m: m.timestamp)
        return FeatureStream.from_messages(imu, frames, gt, meta)


def replay(flt, stream: FeatureStream, on_result=None, events=None) -> Trajectory:
    """Feeds ``stream`` to a filter exposing the reference API
    (imu_callback / feature_callback -> vio_result | None) and returns the
    published body trajectory.  ``events``: ``stream.events()`` built by the
    caller beforehand (the messages are the front-end's output, so a timed
    replay can leave their construction out)."""
    results = []
    for kind, msg in (stream.events() if events is None else events):
        if kind == 0:
            flt.imu_callback(msg)
        else:
            res = flt.feature_callback(msg)
            if res is not None:
                results.append(res)
                if on_result is not None:
                    on_result(res)
    return Trajectory.from_results(results)
