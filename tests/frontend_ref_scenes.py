"""Scenes of tests/golden/frontend_ref.npz (tools/gen_frontend_golden.py):
the same synthetic stereo sequences, rebuilt from the fixture's parameters,
and a driver that runs an ImageProcessor over them and returns the published
messages.  Shared by the CPU bookkeeping test and the GPU test."""
from collections import namedtuple

import numpy as np

import frontend_synth as fs
from conftest import golden

SCENES = ("rectified", "euroc")
StereoMsg = namedtuple("stereo_msg", ["vio_timestamp__", "cam0_msg", "cam1_msg"])
ImgMsg = namedtuple("img_msg", ["vio_timestamp__", "image"])
ImuMsg = namedtuple("imu_msg", ["vio_timestamp__", "angular_velocity", "linear_acceleration"])


def scene_config(g, name):
    from msckf_amd.frontend import FrontendConfig
    W, H = (int(v) for v in g["size"])
    return FrontendConfig(T_imu_cam0=g[name + "_T_imu_cam0"], T_imu_cam1=g[name + "_T_imu_cam1"],
                          cam0_intrinsics=g[name + "_intrinsics"], cam1_intrinsics=g[name + "_intrinsics1"],
                          cam0_distortion_coeffs=g[name + "_distortion"],
                          cam1_distortion_coeffs=g[name + "_distortion1"],
                          cam0_resolution=np.array([W, H]), cam1_resolution=np.array([W, H]))


def run_scene(ip, g, name):
    """Feeds the scene's IMU and stereo messages; returns [(ids, uv (n, 4))] per frame."""
    W, H = (int(v) for v in g["size"])
    f = fs.texture_fn(int(g[name + "_seed"]), W=W, H=H)
    step, gyro, disp = g[name + "_step"], g[name + "_gyro"], float(g[name + "_disparity"])
    out = []
    for k in range(int(g[name + "_frames"])):
        t = 0.05 * k
        for j in range(10):
            ip.imu_callback(ImuMsg(t - 0.05 + 0.005 * j, np.array(gyro, float), np.array([0.0, 0.0, 9.81])))
        dx, dy = np.array(step) * k
        im0, im1 = fs.render(f, W, H, dx, dy), fs.render(f, W, H, dx - disp, dy)
        cs = g["%s_f%d_checksum" % (name, k)]
        assert int(im0.astype(np.int64).sum()) == cs[0] and int(im1.astype(np.int64).sum()) == cs[1], \
            "scene images differ from the fixture's (texture generator drift)"
        msg = ip.stareo_callback(StereoMsg(t, ImgMsg(t, im0), ImgMsg(t, im1)))
        ids = np.array([m.id for m in msg.vio_features], np.int64)
        uv = np.array([[m.u0, m.v0, m.u1, m.v1] for m in msg.vio_features], float).reshape(-1, 4)
        out.append((ids, uv))
    return out


def reference_frames(g, name):
    return [(g["%s_f%d_ids" % (name, k)], g["%s_f%d_uv" % (name, k)]) for k in range(int(g[name + "_frames"]))]
