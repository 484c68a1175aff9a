"""GPU stereo front-end: drop-in host mirror of the
reference ``ImageProcessor`` (MSCKF/image.py:36-702).

The host keeps what the reference keeps in Python -- the grid bookkeeping,
feature ids and lifetimes, pruning, the stereo-match inlier logic and the
published message -- and every image operator runs in the HIP kernels of
``csrc/msckf_frontend.hip`` behind ``include/msckf_frontend.h``:

  reference (cv2)                              here
  FastFeatureDetector.detect (image.py:175,333) mfe_fast   (k_fast, k_fast_rows)
  calcOpticalFlowPyrLK (image.py:254,581,585)   mfe_lk     (k_lk; pyramids + Scharr
                                                            built by mfe_upload)
  undistortPoints / fisheye (image.py:640-674)  mfe_undistort
  projectPoints / fisheye (image.py:676-702)    mfe_distort

cv2 is absent here and on the GPU box: the kernels restate the published
OpenCV 4.x algorithms (oracle/frontend_oracle.py), parity unpinned against cv2
itself.  Method names, arguments and the message layout follow the reference
(including its spelling ``stareo_callback``), so ``vio.py`` can construct this
class in place of its own.  The reference's stubs are kept as they are: RANSAC
marks every match an inlier (image.py:292-293) and ``rescale_points`` is unused.
There is no CPU fallback: without the HIP library or a GPU the constructor
raises.
"""
from __future__ import annotations

import ctypes as C
from collections import defaultdict, namedtuple
from dataclasses import dataclass, field
from itertools import chain

import numpy as np

from . import _lib
from .config import _default_T_imu_cam0

RADTAN, EQUIDISTANT = 0, 1

FeatureMeasurement = namedtuple("FeatureMeasurement", ["id", "u0", "v0", "u1", "v1"])
FeatureMsg = namedtuple("vio_feature_msg__", ["timestamp", "vio_features"])


def _default_T_imu_cam1():
    return np.array([
        [0.012555267089103, 0.999598781151433, -0.025389800891747, -0.044901980682509],
        [-0.999755099723116, 0.013011905181504, 0.017900583825251, -0.020569771258915],
        [0.018223771455443, 0.025158836311552, 0.999517347077547, -0.008638135126028],
        [0, 0, 0, 1.000000000000000]])


@dataclass
class FrontendConfig:
    """Image-processor fields of the reference ConfigEuRoC (config.py:22-44,
    94-121); defaults are the reference's."""
    grid_row: int = 4
    grid_col: int = 5
    grid_min_feature_num: int = 3
    grid_max_feature_num: int = 5
    fast_threshold: int = 15
    ransac_threshold: float = 3
    stereo_threshold: float = 5
    max_iteration: int = 30
    track_precision: float = 0.01
    pyramid_levels: int = 3
    patch_size: int = 15
    T_imu_cam0: np.ndarray = field(default_factory=_default_T_imu_cam0)
    T_imu_cam1: np.ndarray = field(default_factory=_default_T_imu_cam1)
    cam0_distortion_model: str = "radtan"
    cam0_distortion_coeffs: np.ndarray = field(
        default_factory=lambda: np.array([-0.28340811, 0.07395907, 0.00019359, 1.76187114e-05]))
    cam0_intrinsics: np.ndarray = field(default_factory=lambda: np.array([458.654, 457.296, 367.215, 248.375]))
    cam0_resolution: np.ndarray = field(default_factory=lambda: np.array([752, 480]))
    cam1_distortion_model: str = "radtan"
    cam1_distortion_coeffs: np.ndarray = field(
        default_factory=lambda: np.array([-0.28368365, 0.07451284, -0.00010473, -3.55590700e-05]))
    cam1_intrinsics: np.ndarray = field(default_factory=lambda: np.array([457.587, 456.134, 379.999, 255.238]))
    cam1_resolution: np.ndarray = field(default_factory=lambda: np.array([752, 480]))

    @property
    def grid_num(self):
        return self.grid_row * self.grid_col

    @classmethod
    def from_reference(cls, ref_cfg) -> "FrontendConfig":
        g = lambda n: getattr(ref_cfg, "_vio_%s__" % n)
        kw = {}
        for f in cls.__dataclass_fields__:
            try:
                kw[f] = g(f)
            except AttributeError:
                pass
        return cls(**kw)


class FeatureMetaData:
    """Reference FeatureMetaData (image.py:11-20)."""
    __slots__ = ("id", "response", "lifetime", "cam0_point", "cam1_point")

    def __init__(self):
        self.id = None
        self.response = None
        self.lifetime = None
        self.cam0_point = None
        self.cam1_point = None


def _inv_T(T):
    T = np.asarray(T, float)
    out = np.eye(4)
    out[:3, :3] = T[:3, :3].T
    out[:3, 3] = -T[:3, :3].T @ T[:3, 3]
    return out


def _rodrigues(r):
    """cv2.Rodrigues of a rotation vector (image.py:482)."""
    r = np.asarray(r, float).reshape(3)
    th = float(np.linalg.norm(r))
    if th < 1e-300:
        return np.eye(3)
    k = r / th
    K = np.array([[0.0, -k[2], k[1]], [k[2], 0.0, -k[0]], [-k[1], k[0], 0.0]])
    return np.cos(th) * np.eye(3) + (1 - np.cos(th)) * np.outer(k, k) + np.sin(th) * K


def _skew(v):
    x, y, z = v
    return np.array([[0, -z, y], [z, 0, -x], [-y, x, 0]], float)


def _select(data, selectors):
    """Reference select (image.py:728-729)."""
    return [d for d, s in zip(data, selectors) if s]


class Frontend:
    """Device context of the image operators (C-ABI ``mfe_*``)."""

    def __init__(self, width, height, nslot=4, max_level=3, max_points=4096, device=0):
        self.lib = _lib.load_library()
        self.W, self.H, self.max_points = int(width), int(height), int(max_points)
        h = C.c_void_p()
        self._check(self.lib.mfe_create(device, self.W, self.H, nslot, max_level, self.max_points, C.byref(h)))
        self.h = h

    def _check(self, rc):
        if rc < 0:
            raise _lib.MsckfError("mfe: %s (rc=%d)" % (self.lib.mfe_last_error().decode(), rc))
        return rc

    def close(self):
        if getattr(self, "h", None):
            self.lib.mfe_destroy(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def upload(self, slot, image):
        img = np.ascontiguousarray(image, np.uint8)
        if img.shape != (self.H, self.W):
            raise ValueError("image shape %s, context %dx%d" % (img.shape, self.W, self.H))
        self._check(self.lib.mfe_upload(self.h, slot, img.ctypes.data_as(C.POINTER(C.c_uint8))))

    def fast(self, slot, threshold, mask=None, max_kp=1 << 16):
        m = None if mask is None else np.ascontiguousarray(mask, np.uint8)
        xy = np.zeros((max_kp, 2), np.float32)
        resp = np.zeros(max_kp, np.float32)
        n = C.c_int(0)
        self._check(self.lib.mfe_fast(self.h, slot, int(threshold),
                                      None if m is None else m.ctypes.data_as(C.POINTER(C.c_uint8)),
                                      max_kp, xy.ctypes.data_as(C.POINTER(C.c_float)),
                                      resp.ctypes.data_as(C.POINTER(C.c_float)), C.byref(n)))
        k = min(n.value, max_kp)
        return xy[:k].copy(), resp[:k].copy()

    def lk(self, slot_prev, slot_next, prev_pts, next_pts, win=15, max_level=3, max_iter=30, eps=0.01):
        p = np.ascontiguousarray(np.asarray(prev_pts, np.float32).reshape(-1, 2))
        q = np.ascontiguousarray(np.asarray(next_pts, np.float32).reshape(-1, 2)).copy()
        n = len(p)
        st = np.zeros(n, np.uint8)
        if n == 0:
            return q, st
        if n > self.max_points:
            raise ValueError("%d points exceed the context's %d" % (n, self.max_points))
        self._check(self.lib.mfe_lk(self.h, slot_prev, slot_next, n, p.ctypes.data_as(C.POINTER(C.c_float)),
                                    q.ctypes.data_as(C.POINTER(C.c_float)), st.ctypes.data_as(C.POINTER(C.c_uint8)),
                                    int(win), int(max_level), int(max_iter), float(eps)))
        return q, st

    def _cam(self, fn, pts, *args):
        p = np.ascontiguousarray(np.asarray(pts, float).reshape(-1, 2))
        out = np.zeros_like(p)
        if len(p) == 0:
            return out
        if len(p) > self.max_points:
            raise ValueError("%d points exceed the context's %d" % (len(p), self.max_points))
        dp = C.POINTER(C.c_double)
        conv = [a.ctypes.data_as(dp) if isinstance(a, np.ndarray) else a for a in args]
        self._check(fn(self.h, len(p), p.ctypes.data_as(dp), out.ctypes.data_as(dp), *conv))
        return out

    def undistort(self, pts, intrinsics, model, coeffs, R=None, new_intrinsics=None):
        f64 = lambda a: None if a is None else np.ascontiguousarray(np.asarray(a, float).ravel())
        return self._cam(self.lib.mfe_undistort, pts, f64(intrinsics), int(model), f64(coeffs), f64(R),
                         f64(new_intrinsics))

    def distort(self, pts, intrinsics, model, coeffs):
        f64 = lambda a: np.ascontiguousarray(np.asarray(a, float).ravel())
        return self._cam(self.lib.mfe_distort, pts, f64(intrinsics), int(model), f64(coeffs))


def _model(name):
    return EQUIDISTANT if name == "equidistant" else RADTAN


class ImageProcessor:
    """Reference ImageProcessor (image.py:36-702) on the GPU image operators.
    Messages: stereo_msg with ``cam0_msg`` / ``cam1_msg`` (each ``image`` and
    ``vio_timestamp__``), imu_msg with ``vio_timestamp__`` and
    ``angular_velocity`` (dataset.py:56-57, 101, 169-170)."""

    # image slots: the previous cam0 image and the current pair rotate over three
    def __init__(self, config=None, device=0):
        if config is None:
            config = FrontendConfig()
        elif not isinstance(config, FrontendConfig):
            config = FrontendConfig.from_reference(config)
        self.config = config
        self.is_first_img = True
        self.next_feature_id = 0
        self.imu_msg_buffer = []
        self.cam0_prev_img_msg = None
        self.cam0_curr_img_msg = None
        self.cam1_curr_img_msg = None
        self.prev_features = [[] for _ in range(config.grid_num)]
        self.curr_features = [[] for _ in range(config.grid_num)]
        self.num_features = defaultdict(int)
        self.cam0_resolution = np.asarray(config.cam0_resolution)
        self.cam0_intrinsics = np.asarray(config.cam0_intrinsics, float)
        self.cam0_distortion_model = config.cam0_distortion_model
        self.cam0_distortion_coeffs = np.asarray(config.cam0_distortion_coeffs, float)
        self.cam1_resolution = np.asarray(config.cam1_resolution)
        self.cam1_intrinsics = np.asarray(config.cam1_intrinsics, float)
        self.cam1_distortion_model = config.cam1_distortion_model
        self.cam1_distortion_coeffs = np.asarray(config.cam1_distortion_coeffs, float)
        self.T_cam0_imu = _inv_T(config.T_imu_cam0)
        self.R_cam0_imu = self.T_cam0_imu[:3, :3]
        self.t_cam0_imu = self.T_cam0_imu[:3, 3]
        self.T_cam1_imu = _inv_T(config.T_imu_cam1)
        self.R_cam1_imu = self.T_cam1_imu[:3, :3]
        self.t_cam1_imu = self.T_cam1_imu[:3, 3]
        W, H = int(self.cam0_resolution[0]), int(self.cam0_resolution[1])
        self.fe = Frontend(W, H, nslot=3, max_level=config.pyramid_levels, max_points=1 << 16, device=device)
        self._slot_prev, self._slot_c0, self._slot_c1 = 0, 1, 2
        self.lk_kw = dict(win=config.patch_size, max_level=config.pyramid_levels,
                          max_iter=config.max_iteration, eps=config.track_precision)

    # ---- callbacks (image.py:95-147) ----
    def stareo_callback(self, stereo_msg):
        self.cam0_curr_img_msg = stereo_msg.cam0_msg
        self.cam1_curr_img_msg = stereo_msg.cam1_msg
        self.create_image_pyramids()
        if self.is_first_img:
            self.initialize_first_frame()
            self.is_first_img = False
        else:
            self.track_features()
            self.add_new_features()
            self.prune_features()
        try:
            return self.publish()
        finally:
            self.cam0_prev_img_msg = self.cam0_curr_img_msg
            self.prev_features = self.curr_features
            # the current cam0 slot becomes the previous one (its pyramid stays on the device)
            self._slot_prev, self._slot_c0 = self._slot_c0, self._slot_prev
            self.curr_features = [[] for _ in range(self.config.grid_num)]

    stereo_callback = stareo_callback

    def imu_callback(self, msg):
        self.imu_msg_buffer.append(msg)

    def create_image_pyramids(self):
        """image.py:149-164 -- here the device builds the pyramids (and the
        Scharr derivatives LK needs) once per image."""
        self.fe.upload(self._slot_c0, self.cam0_curr_img_msg.image)
        self.fe.upload(self._slot_c1, self.cam1_curr_img_msg.image)

    # ---- detection / tracking (image.py:166-404) ----
    def _grid_code(self, pt, gh, gw):
        return int(pt[1] / gh) * self.config.grid_col + int(pt[0] / gw)

    def _collect_new(self, cam0_points, responses):
        gh, gw = self.get_grid_size(self.cam0_curr_img_msg.image)
        cam1_points, inliers = self.stereo_match(cam0_points)
        grid_new = [[] for _ in range(self.config.grid_num)]
        for i, ok in enumerate(inliers):
            if not ok:
                continue
            f = FeatureMetaData()
            f.response = responses[i]
            f.cam0_point = cam0_points[i]
            f.cam1_point = cam1_points[i]
            grid_new[self._grid_code(cam0_points[i], gh, gw)].append(f)
        for i, feats in enumerate(grid_new):
            for f in sorted(feats, key=lambda x: x.response, reverse=True)[:self.config.grid_min_feature_num]:
                self.curr_features[i].append(f)
                f.id = self.next_feature_id
                f.lifetime = 1
                self.next_feature_id += 1

    def initialize_first_frame(self):
        """image.py:166-217."""
        xy, resp = self.fe.fast(self._slot_c0, self.config.fast_threshold)
        self._collect_new([tuple(p) for p in xy], list(resp))

    def track_features(self):
        """image.py:219-313."""
        img = self.cam0_curr_img_msg.image
        gh, gw = self.get_grid_size(img)
        cam0_R_p_c, cam1_R_p_c = self.integrate_imu_data()
        prev_ids, prev_lifetime, prev_cam0_points, prev_cam1_points = [], [], [], []
        for f in chain.from_iterable(self.prev_features):
            prev_ids.append(f.id)
            prev_lifetime.append(f.lifetime)
            prev_cam0_points.append(f.cam0_point)
            prev_cam1_points.append(f.cam1_point)
        prev_cam0_points = np.array(prev_cam0_points, dtype=np.float32).reshape(-1, 2)
        self.num_features["before_tracking"] = len(prev_cam0_points)
        if len(prev_cam0_points) == 0:
            return
        curr_cam0_points = self.predict_feature_tracking(prev_cam0_points, cam0_R_p_c, self.cam0_intrinsics)
        curr_cam0_points, track_inliers = self.fe.lk(self._slot_prev, self._slot_c0, prev_cam0_points,
                                                     curr_cam0_points, **self.lk_kw)
        track_inliers = track_inliers.astype(bool)
        for i, p in enumerate(curr_cam0_points):
            if not track_inliers[i]:
                continue
            if p[0] < 0 or p[0] > img.shape[1] - 1 or p[1] < 0 or p[1] > img.shape[0] - 1:
                track_inliers[i] = False
        prev_tracked_ids = _select(prev_ids, track_inliers)
        prev_tracked_lifetime = _select(prev_lifetime, track_inliers)
        curr_tracked_cam0_points = _select(curr_cam0_points, track_inliers)
        self.num_features["after_tracking"] = len(curr_tracked_cam0_points)
        curr_cam1_points, match_inliers = self.stereo_match(curr_tracked_cam0_points)
        prev_matched_ids = _select(prev_tracked_ids, match_inliers)
        prev_matched_lifetime = _select(prev_tracked_lifetime, match_inliers)
        curr_matched_cam0_points = _select(curr_tracked_cam0_points, match_inliers)
        curr_matched_cam1_points = _select(curr_cam1_points, match_inliers)
        self.num_features["after_matching"] = len(curr_matched_cam0_points)
        after_ransac = 0
        for i in range(len(curr_matched_cam0_points)):   # RANSAC stub: all inliers (image.py:292-293)
            f = FeatureMetaData()
            f.id = prev_matched_ids[i]
            f.lifetime = prev_matched_lifetime[i] + 1
            f.cam0_point = curr_matched_cam0_points[i]
            f.cam1_point = curr_matched_cam1_points[i]
            self.curr_features[self._grid_code(curr_matched_cam0_points[i], gh, gw)].append(f)
            after_ransac += 1
        self.num_features["after_ransac"] = after_ransac

    def add_new_features(self):
        """image.py:317-390."""
        img = self.cam0_curr_img_msg.image
        gh, gw = self.get_grid_size(img)
        mask = np.ones(img.shape[:2], dtype=np.uint8)
        for f in chain.from_iterable(self.curr_features):
            x, y = map(int, f.cam0_point)
            mask[y - 3:y + 4, x - 3:x + 4] = 0   # the reference's slice, negative starts included
        xy, resp = self.fe.fast(self._slot_c0, self.config.fast_threshold, mask=mask)
        sieve = [[] for _ in range(self.config.grid_num)]
        for p, r in zip(xy, resp):
            sieve[self._grid_code(p, gh, gw)].append((tuple(p), r))
        picked = []
        for feats in sieve:
            if len(feats) > self.config.grid_max_feature_num:
                feats = sorted(feats, key=lambda x: x[1], reverse=True)[:self.config.grid_max_feature_num]
            picked.extend(feats)
        self._collect_new([p for p, _ in picked], [r for _, r in picked])

    def prune_features(self):
        """image.py:392-404."""
        for i, feats in enumerate(self.curr_features):
            if len(feats) <= self.config.grid_max_feature_num:
                continue
            self.curr_features[i] = sorted(feats, key=lambda x: x.lifetime,
                                           reverse=True)[:self.config.grid_max_feature_num]

    def publish(self):
        """image.py:406-438."""
        ids, c0, c1 = [], [], []
        for f in chain.from_iterable(self.curr_features):
            ids.append(f.id)
            c0.append(f.cam0_point)
            c1.append(f.cam1_point)
        u0 = self.undistort_points(c0, self.cam0_intrinsics, self.cam0_distortion_model, self.cam0_distortion_coeffs)
        u1 = self.undistort_points(c1, self.cam1_intrinsics, self.cam1_distortion_model, self.cam1_distortion_coeffs)
        feats = [FeatureMeasurement(ids[i], u0[i][0], u0[i][1], u1[i][0], u1[i][1]) for i in range(len(ids))]
        return FeatureMsg(self.cam0_curr_img_msg.vio_timestamp__, feats)

    # ---- geometry helpers (image.py:440-702) ----
    def integrate_imu_data(self):
        """image.py:440-487."""
        begin = next((i for i, m in enumerate(self.imu_msg_buffer)
                      if m.vio_timestamp__ >= self.cam0_prev_img_msg.vio_timestamp__ - 0.01), None)
        end = next((i for i, m in enumerate(self.imu_msg_buffer)
                    if m.vio_timestamp__ >= self.cam0_curr_img_msg.vio_timestamp__ - 0.004), None)
        if begin is None or end is None:
            return np.identity(3), np.identity(3)
        mean = np.zeros(3)
        for i in range(begin, end):
            mean += self.imu_msg_buffer[i].angular_velocity
        if end > begin:
            mean /= (end - begin)
        cam0_w = self.R_cam0_imu.T @ mean
        cam1_w = self.R_cam1_imu.T @ mean
        dt = self.cam0_curr_img_msg.vio_timestamp__ - self.cam0_prev_img_msg.vio_timestamp__
        R0 = _rodrigues(cam0_w * dt).T
        R1 = _rodrigues(cam1_w * dt).T
        self.imu_msg_buffer = self.imu_msg_buffer[end:]
        return R0, R1

    def get_grid_size(self, img):
        """image.py:513-519."""
        return (int(np.ceil(img.shape[0] / self.config.grid_row)),
                int(np.ceil(img.shape[1] / self.config.grid_col)))

    def predict_feature_tracking(self, input_pts, R_p_c, intrinsics):
        """image.py:521-552."""
        if len(input_pts) == 0:
            return np.zeros((0, 2), np.float32)
        K = np.array([[intrinsics[0], 0.0, intrinsics[2]], [0.0, intrinsics[1], intrinsics[3]], [0.0, 0.0, 1.0]])
        Hm = K @ R_p_c @ np.linalg.inv(K)
        p = np.concatenate([np.asarray(input_pts, float).reshape(-1, 2), np.ones((len(input_pts), 1))], 1)
        q = p @ Hm.T
        return (q[:, :2] / q[:, 2:3]).astype(np.float32)

    def stereo_match(self, cam0_points):
        """image.py:554-638: project into cam1 through the extrinsics, LK
        cam0 -> cam1 and back, and the vertical-disparity, round-trip and
        epipolar tests."""
        cam0_points = np.asarray(cam0_points, float).reshape(-1, 2)
        if len(cam0_points) == 0:
            return [], []
        R_cam0_cam1 = self.R_cam1_imu.T @ self.R_cam0_imu
        und = self.undistort_points(cam0_points, self.cam0_intrinsics, self.cam0_distortion_model,
                                    self.cam0_distortion_coeffs, R_cam0_cam1)
        cam1_points = self.distort_points(und, self.cam1_intrinsics, self.cam1_distortion_model,
                                          self.cam1_distortion_coeffs)
        cam1_copy = cam1_points.copy()
        c0 = cam0_points.astype(np.float32)
        c1, inliers = self.fe.lk(self._slot_c0, self._slot_c1, c0, cam1_points.astype(np.float32), **self.lk_kw)
        c0_back, _ = self.fe.lk(self._slot_c1, self._slot_c0, c1, c0.copy(), **self.lk_kw)
        err = np.linalg.norm(c0 - c0_back, axis=1)
        disparity = np.abs(cam1_copy[:, 1] - c1[:, 1])
        inliers = np.logical_and.reduce([inliers.reshape(-1).astype(bool), err < 3, disparity < 20])
        img1 = self.cam1_curr_img_msg.image
        for i, p in enumerate(c1):
            if not inliers[i]:
                continue
            if p[0] < 0 or p[0] > img1.shape[1] - 1 or p[1] < 0 or p[1] > img1.shape[0] - 1:
                inliers[i] = False
        t_cam0_cam1 = self.R_cam1_imu.T @ (self.t_cam0_imu - self.t_cam1_imu)
        E = _skew(t_cam0_cam1) @ R_cam0_cam1
        u0 = self.undistort_points(c0, self.cam0_intrinsics, self.cam0_distortion_model, self.cam0_distortion_coeffs)
        u1 = self.undistort_points(c1, self.cam1_intrinsics, self.cam1_distortion_model, self.cam1_distortion_coeffs)
        norm_pixel_unit = 4.0 / (self.cam0_intrinsics[0] + self.cam0_intrinsics[1] +
                                 self.cam1_intrinsics[0] + self.cam1_intrinsics[1])
        for i in range(len(u0)):
            if not inliers[i]:
                continue
            pt0 = np.array([u0[i][0], u0[i][1], 1.0])
            pt1 = np.array([u1[i][0], u1[i][1], 1.0])
            line = E @ pt0
            error = abs((pt1 * line)[0]) / np.linalg.norm(line[:2])
            if error > self.config.stereo_threshold * norm_pixel_unit:
                inliers[i] = False
        return [tuple(p) for p in c1], list(inliers)

    def undistort_points(self, pts_in, intrinsics, distortion_model, distortion_coeffs,
                         rectification_matrix=np.identity(3), new_intrinsics=np.array([1, 1, 0, 0])):
        """image.py:640-674 (cv2.undistortPoints / cv2.fisheye.undistortPoints).
        Quirk kept: for 'equidistant' the reference passes its rectification
        matrix in cv2.fisheye.undistortPoints' output slot and K_new in its R
        slot (image.py:669-670, positional arguments), so cv2 rotates by K_new
        and returns normalised points; the rectification is never applied."""
        if len(pts_in) == 0:
            return np.zeros((0, 2))
        model = _model(distortion_model)
        if model == EQUIDISTANT:
            n = np.asarray(new_intrinsics, float)
            K_new = np.array([[n[0], 0.0, n[2]], [0.0, n[1], n[3]], [0.0, 0.0, 1.0]])
            return self.fe.undistort(pts_in, intrinsics, model, distortion_coeffs, K_new, np.array([1.0, 1.0, 0.0, 0.0]))
        return self.fe.undistort(pts_in, intrinsics, model, distortion_coeffs, rectification_matrix, new_intrinsics)

    def distort_points(self, pts_in, intrinsics, distortion_model, distortion_coeffs):
        """image.py:676-702 (cv2.projectPoints / cv2.fisheye.distortPoints)."""
        if len(pts_in) == 0:
            return np.zeros((0, 2))
        return self.fe.distort(pts_in, intrinsics, _model(distortion_model), distortion_coeffs)
