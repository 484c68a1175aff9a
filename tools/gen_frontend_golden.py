"""Fixture tests/golden/frontend_ref.npz: the reference's own ImageProcessor
(MSCKF/image.py:36-702) run IN THE BUILD CONTAINER ONLY on synthetic stereo
sequences, so that the GPU front-end's host bookkeeping (grid bucketing, id
assignment, lifetimes and pruning, the stereo-match gates, publish order) is
pinned against the reference code itself, not only against properties.

cv2 is not installed, so image.py is imported behind an in-memory ``cv2``
module whose operators are the CPU restatements of oracle/frontend_oracle.py
(FAST + non-max + mask, pyramidal LK, radtan / fisheye undistort and distort,
Rodrigues); numba's ``jit`` becomes the identity (tools/refload.py).  The
operators themselves therefore stay "parity unpinned" against cv2; what the
fixture pins is everything image.py does around them.  Nothing is written
into /root/reference and nothing from it is copied here: the fixture holds the
scene parameters, per-image checksums and the published messages (ids and
undistorted coordinates) only.

    python tools/gen_frontend_golden.py        (a few minutes: the LK oracle is numpy)
"""
import os
import sys
import types
from collections import namedtuple

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
import frontend_synth as fs  # noqa: E402
from oracle import frontend_oracle as fo  # noqa: E402

REF_DIR = "/root/reference/MSCKF"

# ------------------------------------------------------------ cv2 stand-in --


class _KeyPoint:
    __slots__ = ("pt", "response")

    def __init__(self, x, y, r):
        self.pt = (float(x), float(y))
        self.response = float(r)


class _Fast:
    def __init__(self, threshold):
        self.t = int(threshold)

    def detect(self, img, mask=None):
        xy, resp = fo.fast_detect(img, self.t, nonmax=True, mask=mask)
        return [_KeyPoint(x, y, r) for (x, y), r in zip(xy, resp)]


def _lk(prev, nxt, prev_pts, next_pts, winSize=(15, 15), maxLevel=3, criteria=(3, 30, 0.01), flags=0):
    p = np.asarray(prev_pts, np.float32).reshape(-1, 2)
    q = np.asarray(next_pts, np.float32).reshape(-1, 2)
    out, st = fo.lk_track(prev, nxt, p, q, win=int(winSize[0]), max_level=int(maxLevel),
                          max_iter=int(criteria[1]), eps=float(criteria[2]))
    return out.reshape(np.shape(next_pts)), st.reshape(-1, 1), np.zeros((len(p), 1), np.float32)


def _undistort(pts, K, D, Rdummy=None, R=None, P=None):
    K = np.asarray(K, float)
    P = np.eye(3) if P is None else np.asarray(P, float)
    R = np.eye(3) if R is None else np.asarray(R, float)
    out = fo.undistort_points(np.asarray(pts).reshape(-1, 2), (K[0, 0], K[1, 1], K[0, 2], K[1, 2]), "radtan",
                              np.asarray(D, float), R, (P[0, 0], P[1, 1], P[0, 2], P[1, 2]))
    return out.reshape(-1, 1, 2)


def _fisheye_undistort(pts, K, D, undistorted=None, R=None, P=None):
    # cv2.fisheye.undistortPoints(distorted, K, D[, undistorted[, R[, P]]]): the
    # reference passes its rectification as the 4th positional (the output
    # array) and K_new as R (image.py:669-670) -- restated as cv2 binds them
    K = np.asarray(K, float)
    P = np.eye(3) if P is None else np.asarray(P, float)
    R = np.eye(3) if R is None else np.asarray(R, float)
    out = fo.undistort_points(np.asarray(pts).reshape(-1, 2), (K[0, 0], K[1, 1], K[0, 2], K[1, 2]), "equidistant",
                              np.asarray(D, float), R, (P[0, 0], P[1, 1], P[0, 2], P[1, 2]))
    return out.reshape(-1, 1, 2)


def _fisheye_distort(pts, K, D):
    K = np.asarray(K, float)
    out = fo.distort_points(np.asarray(pts).reshape(-1, 2), (K[0, 0], K[1, 1], K[0, 2], K[1, 2]), "equidistant",
                            np.asarray(D, float))
    return out.reshape(-1, 1, 2)


def _to_homogeneous(pts):
    p = np.asarray(pts, float).reshape(-1, 2)
    return np.concatenate([p, np.ones((len(p), 1))], 1).reshape(-1, 1, 3)


def _project(pts3, rvec, tvec, K, D):
    p = np.asarray(pts3, float).reshape(-1, 3)
    assert not np.any(rvec) and not np.any(tvec)
    K = np.asarray(K, float)
    out = fo.distort_points(p[:, :2] / p[:, 2:3], (K[0, 0], K[1, 1], K[0, 2], K[1, 2]), "radtan",
                            np.asarray(D, float))
    return out.reshape(-1, 1, 2), None


def make_cv2_stub():
    cv = types.ModuleType("cv2")
    cv.TERM_CRITERIA_EPS, cv.TERM_CRITERIA_COUNT, cv.OPTFLOW_USE_INITIAL_FLOW = 2, 1, 4
    cv.FastFeatureDetector_create = lambda t=10: _Fast(t)
    cv.calcOpticalFlowPyrLK = _lk
    cv.Rodrigues = lambda r: (fo.rodrigues(r), None)
    cv.undistortPoints = _undistort
    cv.convertPointsToHomogeneous = _to_homogeneous
    cv.projectPoints = _project
    cv.fisheye = types.SimpleNamespace(undistortPoints=_fisheye_undistort, distortPoints=_fisheye_distort)
    return cv


def load_image_module():
    sys.dont_write_bytecode = True
    nb = types.ModuleType("numba")
    nb.jit = lambda *a, **k: (lambda f: f)
    sys.modules["numba"] = nb
    sys.modules["cv2"] = make_cv2_stub()
    if REF_DIR not in sys.path:
        sys.path.insert(0, REF_DIR)
    import config  # noqa: E402
    import image  # noqa: E402
    return config, image


# ------------------------------------------------------------------ scenes --
W, H = 376, 240
SCENES = {
    # rectified pinhole pair, no distortion, baseline along x: a uniform disparity
    "rectified": dict(seed=4, intrinsics=[225.0, 225.0, 188.0, 120.0], distortion=[0.0, 0.0, 0.0, 0.0],
                      T_imu_cam0=np.eye(4).tolist(),
                      T_imu_cam1=[[1, 0, 0, -0.11], [0, 1, 0, 0], [0, 0, 1, 0], [0, 0, 0, 1]],
                      disparity=12.0, step=[1.5, -0.5], gyro=[0.0, 0.0, 0.02], frames=8),
    # the reference's own calibration (radtan distortion, EuRoC extrinsics), intrinsics halved for
    # the half-size images; the same rendered pair (cam1 = cam0 shifted) so many matches fail
    # the epipolar gate -- that gate is part of what is pinned
    "euroc": dict(seed=7, intrinsics=None, distortion=None, T_imu_cam0=None, T_imu_cam1=None,
                  disparity=9.0, step=[-1.0, 0.75], gyro=[0.01, -0.02, 0.0], frames=6),
}

StereoMsg = namedtuple("stereo_msg", ["vio_timestamp__", "cam0_msg", "cam1_msg"])
ImgMsg = namedtuple("img_msg", ["vio_timestamp__", "image"])
ImuMsg = namedtuple("imu_msg", ["vio_timestamp__", "angular_velocity", "linear_acceleration"])


def scene_config(config, sc):
    cfg = config.ConfigEuRoC()
    if sc["intrinsics"] is None:   # the reference calibration, scaled to the half-size images
        for c in ("cam0", "cam1"):
            k = np.array(getattr(cfg, "_vio_%s_intrinsics__" % c), float) * 0.5
            setattr(cfg, "_vio_%s_intrinsics__" % c, k)
            setattr(cfg, "_vio_%s_resolution__" % c, np.array([W, H]))
        sc["intrinsics"] = cfg._vio_cam0_intrinsics__.tolist()
        sc["intrinsics1"] = cfg._vio_cam1_intrinsics__.tolist()
        sc["distortion"] = np.asarray(cfg._vio_cam0_distortion_coeffs__).tolist()
        sc["distortion1"] = np.asarray(cfg._vio_cam1_distortion_coeffs__).tolist()
        sc["T_imu_cam0"] = np.asarray(cfg._vio_T_imu_cam0__).tolist()
        sc["T_imu_cam1"] = np.asarray(cfg._vio_T_imu_cam1__).tolist()
    else:
        for c in ("cam0", "cam1"):
            setattr(cfg, "_vio_%s_intrinsics__" % c, np.array(sc["intrinsics"], float))
            setattr(cfg, "_vio_%s_distortion_coeffs__" % c, np.array(sc["distortion"], float))
            setattr(cfg, "_vio_%s_resolution__" % c, np.array([W, H]))
        cfg._vio_T_imu_cam0__ = np.array(sc["T_imu_cam0"], float)
        cfg._vio_T_imu_cam1__ = np.array(sc["T_imu_cam1"], float)
        sc["intrinsics1"], sc["distortion1"] = sc["intrinsics"], sc["distortion"]
    return cfg


def scene_frames(sc):
    """(t, imu messages before the frame, cam0 image, cam1 image) per frame --
    the same generator the GPU test uses (tests/frontend_synth.py)."""
    f = fs.texture_fn(sc["seed"], W=W, H=H)
    out = []
    for k in range(sc["frames"]):
        t = 0.05 * k
        imu = [(t - 0.05 + 0.005 * j, np.array(sc["gyro"], float), np.array([0.0, 0.0, 9.81])) for j in range(10)]
        dx, dy = np.array(sc["step"]) * k
        out.append((t, imu, fs.render(f, W, H, dx, dy), fs.render(f, W, H, dx - sc["disparity"], dy)))
    return out


def main():
    config, image = load_image_module()
    rec = {}
    for name, sc in SCENES.items():
        cfg = scene_config(config, sc)
        ip = image.ImageProcessor(cfg)
        for k, (t, imu, im0, im1) in enumerate(scene_frames(sc)):
            for ts, w, a in imu:
                ip.imu_callback(ImuMsg(ts, w, a))
            msg = ip.stareo_callback(StereoMsg(t, ImgMsg(t, im0), ImgMsg(t, im1)))
            ids = np.array([m.id for m in msg.vio_features], np.int64)
            uv = np.array([[m.u0, m.v0, m.u1, m.v1] for m in msg.vio_features], float).reshape(-1, 4)
            rec["%s_f%d_ids" % (name, k)] = ids
            rec["%s_f%d_uv" % (name, k)] = uv
            rec["%s_f%d_checksum" % (name, k)] = np.array([int(im0.astype(np.int64).sum()),
                                                            int(im1.astype(np.int64).sum())])
            rec["%s_f%d_counts" % (name, k)] = np.array([ip.num_features[key] for key in
                                                          ("before_tracking", "after_tracking", "after_matching")])
            print(name, k, "published", len(ids), "counts", rec["%s_f%d_counts" % (name, k)].tolist(), flush=True)
        for key in ("intrinsics", "intrinsics1", "distortion", "distortion1", "T_imu_cam0", "T_imu_cam1",
                    "step", "gyro"):
            rec["%s_%s" % (name, key)] = np.array(sc[key], float)
        for key in ("seed", "frames", "disparity"):
            rec["%s_%s" % (name, key)] = np.array(sc[key])
    rec["size"] = np.array([W, H])
    out = os.path.join(ROOT, "tests", "golden", "frontend_ref.npz")
    np.savez_compressed(out, **rec)
    print("wrote", out)


if __name__ == "__main__":
    main()
