"""GPU stereo front-end throughput: the drop-in ImageProcessor
(msckf_amd.frontend) over a synthetic rectified stereo stream at the EuRoC
resolution (752 x 480; textured plane, known per-frame motion and disparity).
Prints one JSON line: frames/s end to end (host bookkeeping + uploads +
kernels), features published per frame, and the per-operator wall times of
one frame.

    python tools/bench_frontend.py [--frames 60]
"""
import argparse
import json
import os
import sys
import time
from collections import namedtuple

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
import msckf_pkg  # noqa: E402,F401
import msckf_amd.frontend as fe_mod  # noqa: E402
import frontend_synth as fs  # noqa: E402

StereoMsg = namedtuple("stereo_msg", ["vio_timestamp__", "cam0_image", "cam1_image", "cam0_msg", "cam1_msg"])
ImgMsg = namedtuple("img_msg", ["vio_timestamp__", "image"])
ImuMsg = namedtuple("imu_msg", ["vio_timestamp__", "angular_velocity", "linear_acceleration"])


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--frames", type=int, default=60)
    a = ap.parse_args()
    W, H = 752, 480
    f = fs.texture_fn(4, W=W, H=H)
    K = np.array([450.0, 450.0, 376.0, 240.0])
    Ti1 = np.eye(4)
    Ti1[0, 3] = -0.11
    cfg = fe_mod.FrontendConfig(T_imu_cam0=np.eye(4), T_imu_cam1=Ti1, cam0_distortion_coeffs=np.zeros(4),
                                cam1_distortion_coeffs=np.zeros(4), cam0_intrinsics=K, cam1_intrinsics=K)
    frames = []
    for k in range(a.frames):   # rendered up front: not part of the timing
        dx, dy = 1.5 * (k % 40), -0.5 * (k % 40)
        frames.append((fs.render(f, W, H, dx, dy), fs.render(f, W, H, dx - 12.0, dy)))
    ip = fe_mod.ImageProcessor(cfg)
    nfeat = []
    t0 = None
    for k, (c0, c1) in enumerate(frames):
        t = 0.05 * k
        for j in range(10):
            ip.imu_callback(ImuMsg(t - 0.05 + 0.005 * j, np.zeros(3), np.array([0.0, 0.0, 9.81])))
        if k == 2:
            t0 = time.perf_counter()
        msg = ip.stareo_callback(StereoMsg(t, c0, c1, ImgMsg(t, c0), ImgMsg(t, c1)))
        nfeat.append(len(msg.vio_features))
    el = time.perf_counter() - t0
    fe = ip.fe
    c0 = frames[0][0]
    ops = {}
    t1 = time.perf_counter(); fe.upload(0, c0); ops["upload_pyramid_ms"] = (time.perf_counter() - t1) * 1e3
    t1 = time.perf_counter(); xy, _ = fe.fast(0, 15); ops["fast_ms"] = (time.perf_counter() - t1) * 1e3
    pts = xy[:200]
    fe.upload(1, frames[1][0])
    t1 = time.perf_counter(); fe.lk(0, 1, pts, pts); ops["lk_200pts_ms"] = (time.perf_counter() - t1) * 1e3
    print(json.dumps({"component": "stereo front-end (image.py) on GPU", "resolution": [W, H],
                      "frames_per_s": round((a.frames - 2) / el, 1), "features_per_frame": float(np.mean(nfeat)),
                      "fast_keypoints_frame0": int(len(xy)), "op_wall_ms": {k: round(v, 3) for k, v in ops.items()},
                      "note": "host bookkeeping in Python; synthetic stream; cv2 absent (no reference timing)"}))


if __name__ == "__main__":
    main()
