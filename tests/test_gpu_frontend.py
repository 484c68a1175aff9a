"""GPU stereo front-end (csrc/msckf_frontend.hip, include/msckf_frontend.h)
against the oracle restatement of the OpenCV operators
(oracle/frontend_oracle.py; parity unpinned against cv2 itself, which is not
installed):
  * FAST: keypoints and responses bit-exact (integer work), with and without
    a mask, at the EuRoC resolution;
  * LK: the same integer fixed-point arithmetic and float32 updates as the
    oracle -- positions within 1e-4 px, status identical -- and a known motion
    of a continuous scene recovered;
  * camera models: fp64, <= 1e-12 relative;
  * ImageProcessor (host mirror of image.py:36-702) on a synthetic stereo
    sequence: ids persist across frames, the tracked motion and the stereo
    disparity are the rendered ones."""
from collections import namedtuple

import numpy as np
import pytest

import msckf_amd.frontend as fe_mod
from oracle import frontend_oracle as fo
import frontend_synth as fs

pytestmark = pytest.mark.gpu
W, H = 752, 480


@pytest.fixture(scope="module")
def scene():
    f = fs.texture_fn(2, W=W, H=H)
    return f, fs.render(f, W, H), fs.render(f, W, H, 2.6, -1.3)


@pytest.fixture(scope="module")
def fe():
    ctx = fe_mod.Frontend(W, H, nslot=3, max_level=3)
    yield ctx
    ctx.close()


def test_fast_matches_oracle(fe, scene):
    _, img, _ = scene
    fe.upload(0, img)
    xy, resp = fe.fast(0, 15)
    xo, ro = fo.fast_detect(img, 15)
    assert len(xo) > 1000
    np.testing.assert_array_equal(xy, xo)
    np.testing.assert_array_equal(resp, ro.astype(np.float32))
    mask = np.ones((H, W), np.uint8)
    mask[100:300, 200:500] = 0
    xm, rm = fe.fast(0, 15, mask=mask)
    keep = mask[xo[:, 1].astype(int), xo[:, 0].astype(int)] != 0
    np.testing.assert_array_equal(xm, xo[keep])
    np.testing.assert_array_equal(rm, ro[keep].astype(np.float32))
    small, _ = fe.fast(0, 15, max_kp=10)
    np.testing.assert_array_equal(small, xo[:10])


def test_lk_matches_oracle_and_motion(fe, scene):
    _, img, moved = scene
    fe.upload(0, img)
    fe.upload(1, moved)
    xo, _ = fo.fast_detect(img, 15)
    rng = np.random.default_rng(0)
    pts = xo[rng.choice(len(xo), 120, replace=False)]
    pts = np.concatenate([pts, [[2.0, 3.0], [749.5, 477.0], [-30.0, 10.0]]]).astype(np.float32)   # borders, outside
    guess = pts + np.float32([1.0, 0.0])
    g, sg = fe.lk(0, 1, pts, guess)
    o, so = fo.lk_track(img, moved, pts, guess)
    np.testing.assert_array_equal(sg, so)
    np.testing.assert_allclose(g[so == 1], o[so == 1], atol=1e-4)
    inner = (so == 1) & (pts[:, 0] > 20) & (pts[:, 0] < W - 20) & (pts[:, 1] > 20) & (pts[:, 1] < H - 20)
    assert inner.sum() >= 90
    err = np.abs(g[inner] - pts[inner] - np.array([2.6, -1.3]))
    assert np.median(err) < 0.02, np.median(err)


@pytest.mark.parametrize("model,coeffs", [(0, [-0.28340811, 0.07395907, 0.00019359, 1.76187114e-05]),
                                          (1, [0.01, -0.005, 0.001, -0.0002])])
def test_camera_models_match_oracle(fe, model, coeffs):
    K = np.array([458.654, 457.296, 367.215, 248.375])
    name = "equidistant" if model == 1 else "radtan"
    rng = np.random.default_rng(5)
    px = rng.uniform([0, 0], [W, H], (300, 2))
    R = np.array([[0.999997256477881, 0.002312067192424, 0.000376008102415],
                  [-0.002317135723281, 0.999898048506644, 0.014089835846648],
                  [-0.000343393120525, -0.014090668452714, 0.999900662637729]])
    u = fe.undistort(px, K, model, coeffs, R, [1, 1, 0, 0])
    np.testing.assert_allclose(u, fo.undistort_points(px, K, name, coeffs, R=R), rtol=1e-12, atol=1e-14)
    d = fe.distort(u, K, model, coeffs)
    np.testing.assert_allclose(d, fo.distort_points(u, K, name, coeffs), rtol=1e-12, atol=1e-9)


def test_fisheye_rejection_matches_oracle(fe):
    """cv2 4.x fisheye.undistortPoints rejection (non-converged / flipped
    theta -> (-1e6, -1e6)) and early Newton stop, GPU against the oracle:
    with k = (-1, 0, 0, 0) theta_d > 0.385 has no solution."""
    k = [-1.0, 0.0, 0.0, 0.0]
    px = np.array([[0.6, 0.0], [0.2, 0.1], [0.0, 0.3], [0.5, 0.5], [1e-9, 0.0]])
    u = fe.undistort(px, np.array([1.0, 1.0, 0.0, 0.0]), 1, k, np.eye(3), [1, 1, 0, 0])
    o = fo.undistort_points(px, (1, 1, 0, 0), "equidistant", k)
    np.testing.assert_allclose(u, o, rtol=1e-12, atol=1e-14)
    assert (u[0] == -1000000.0).all() and (u[3] == -1000000.0).all() and (u[1] > -1).all()


StereoMsg = namedtuple("stereo_msg", ["vio_timestamp__", "cam0_image", "cam1_image", "cam0_msg", "cam1_msg"])
ImgMsg = namedtuple("img_msg", ["vio_timestamp__", "image"])
ImuMsg = namedtuple("imu_msg", ["vio_timestamp__", "angular_velocity", "linear_acceleration"])


def test_image_processor_synthetic_stereo():
    """Fronto-parallel textured plane, rectified pinhole pair (no distortion,
    baseline along x): cam1 sees the scene shifted by a uniform disparity,
    and every frame moves the scene by (1.5, -0.5) px."""
    f = fs.texture_fn(4, W=W, H=H)
    K = np.array([450.0, 450.0, 376.0, 240.0])
    Ti0 = np.eye(4)
    Ti1 = np.eye(4)
    Ti1[0, 3] = -0.11                 # p_cam1 = p_imu - b x: features move left by f b / Z
    disp = 12.0
    cfg = fe_mod.FrontendConfig(T_imu_cam0=Ti0, T_imu_cam1=Ti1,
                                cam0_distortion_coeffs=np.zeros(4), cam1_distortion_coeffs=np.zeros(4),
                                cam0_intrinsics=K, cam1_intrinsics=K)
    ip = fe_mod.ImageProcessor(cfg)
    step = np.array([1.5, -0.5])
    prev = None
    for k in range(5):
        t = 0.05 * k
        for j in range(10):
            ip.imu_callback(ImuMsg(t - 0.05 + 0.005 * j, np.zeros(3), np.array([0, 0, 9.81])))
        dx, dy = step * k
        c0 = ImgMsg(t, fs.render(f, W, H, dx, dy))
        c1 = ImgMsg(t, fs.render(f, W, H, dx - disp, dy))
        msg = ip.stareo_callback(StereoMsg(t, c0.image, c1.image, c0, c1))
        assert msg.timestamp == t
        feats = {m.id: m for m in msg.vio_features}
        assert len(feats) >= 40
        u0 = np.array([[m.u0, m.v0] for m in feats.values()])
        u1 = np.array([[m.u1, m.v1] for m in feats.values()])
        # the reference's own gates are loose (round trip < 3 px, epipolar < 5 px): a few
        # matches on weak texture pass with sub-pixel errors; the bulk is exact
        derr = np.abs((u0 - u1) * K[0] - np.array([disp, 0.0]))
        assert np.median(derr) < 0.01 and np.quantile(derr, 0.9) < 0.1 and derr.max() < 3, derr.max()
        if prev is not None:
            common = sorted(set(prev) & set(feats))
            assert len(common) >= 0.8 * len(prev)
            mv = np.array([[feats[i].u0 - prev[i].u0, feats[i].v0 - prev[i].v0] for i in common]) * K[0]
            assert np.median(np.abs(mv - step)) < 0.05, np.median(np.abs(mv - step))
        prev = feats
    assert ip.num_features["after_tracking"] > 0


@pytest.mark.parametrize("name", ["rectified", "euroc"])
def test_image_processor_vs_reference(name):
    """The GPU front-end against the reference's own ImageProcessor
    (tests/golden/frontend_ref.npz, tools/gen_frontend_golden.py: image.py run
    in the build container on the oracle operators).  The bookkeeping is
    checked exactly on CPU (tests/test_frontend_ref.py); here the HIP
    operators run under it: every frame's published ids identical, in order,
    and the cam0 / cam1 coordinates within 1e-4 px (normalised coordinates x
    the focal length)."""
    from conftest import golden
    from frontend_ref_scenes import scene_config, run_scene, reference_frames
    g = golden("frontend_ref")
    ip = fe_mod.ImageProcessor(scene_config(g, name))
    got = run_scene(ip, g, name)
    fx = np.array([g[name + "_intrinsics"][0], g[name + "_intrinsics"][1],
                   g[name + "_intrinsics1"][0], g[name + "_intrinsics1"][1]])
    worst = 0.0
    for k, ((ids, uv), (rids, ruv)) in enumerate(zip(got, reference_frames(g, name))):
        np.testing.assert_array_equal(ids, rids, err_msg="frame %d" % k)
        err = np.abs(uv - ruv) * fx
        worst = max(worst, float(err.max()) if err.size else 0.0)
        assert err.max() <= 1e-4, (k, err.max())
    print("%s: %d frames, ids identical, worst coordinate deviation %.2e px" % (name, len(got), worst))
