"""CPU restatement of the stereo front-end's image operators -- TEST
INFRASTRUCTURE ONLY (imported by tests/, never by the product package).

The reference front-end (MSCKF/image.py:95-702) calls OpenCV for every image
operator:

  * cv2.FastFeatureDetector_create(15).detect (image.py:50, 175, 333): FAST
    9/16 segment test, corner score, 3x3 non-max suppression, mask filter;
  * cv2.calcOpticalFlowPyrLK (image.py:254, 581, 585) with the lk_params of
    config.py:37-44: 15x15 window, maxLevel 3, 30 iterations / 0.01 px,
    OPTFLOW_USE_INITIAL_FLOW -- pyramids by pyrDown, Scharr derivatives,
    14-bit fixed-point bilinear weights, float accumulations;
  * cv2.undistortPoints / cv2.projectPoints (radtan) and cv2.fisheye
    (equidistant) (image.py:640-702); cv2.Rodrigues (image.py:482).

cv2 is not installed in this image or on the GPU box, so this module restates
the published OpenCV 4.x algorithms (features2d fast.cpp / fast_score.cpp,
imgproc pyramids.cpp, video lkpyramid.cpp, calib3d undistort.cpp /
fisheye.cpp) in numpy.  PARITY UNPINNED against cv2 itself: the reference
repository holds no images, fixtures or tests for image.py and cv2 cannot run
here.  The restatement is pinned by analytic cases instead
(tests/test_frontend_oracle.py: synthetic corners, known sub-pixel shifts,
distort / undistort round trips, Rodrigues identities), and the HIP kernels are
checked against it (tests/test_gpu_frontend.py).
"""
from __future__ import annotations

import numpy as np

# FAST 9/16 Bresenham circle of radius 3 (fast.cpp makeOffsets, patternSize 16): (dx, dy)
FAST_CIRCLE = np.array([(0, 3), (1, 3), (2, 2), (3, 1), (3, 0), (3, -1), (2, -2), (1, -3),
                        (0, -3), (-1, -3), (-2, -2), (-3, -1), (-3, 0), (-3, 1), (-2, 2), (-1, 3)], np.int64)

W_BITS = 14                      # lkpyramid.cpp fixed-point interpolation weights
FLT_SCALE = 1.0 / (1 << 20)
MIN_EIG_THRESHOLD = 1e-4         # calcOpticalFlowPyrLK default minEigThreshold


def _descale(x, n):
    return (x + (1 << (n - 1))) >> n


# ----------------------------------------------------------------- FAST ----
def _corner_score(d, threshold):
    """cornerScore<16> (fast_score.cpp): d[k] = v - circle[k mod 16], k = 0..24;
    the largest threshold at which the pixel stays a corner, minus one."""
    d = [int(x) for x in d]
    a0 = threshold
    for k in range(0, 16, 2):
        a = min(d[k + 1], d[k + 2], d[k + 3])
        if a <= a0:
            continue
        a = min(a, d[k + 4], d[k + 5], d[k + 6], d[k + 7], d[k + 8])
        a0 = max(a0, min(a, d[k]))
        a0 = max(a0, min(a, d[k + 9]))
    b0 = -a0
    for k in range(0, 16, 2):
        b = max(d[k + 1], d[k + 2], d[k + 3], d[k + 4], d[k + 5])
        if b >= b0:
            continue
        b = max(b, d[k + 6], d[k + 7], d[k + 8])
        b0 = min(b0, max(b, d[k]))
        b0 = min(b0, max(b, d[k + 9]))
    return -b0 - 1


def fast_corner_mask(img, threshold):
    """Segment test (FAST_t<16>, fast.cpp): an arc of >= 9 contiguous circle
    pixels all brighter than v + t or all darker than v - t.  Returns the
    boolean corner map over the whole image (False within 3 px of the border)
    and the (25, H, W) int difference stack d = v - circle (wrapped)."""
    img = np.asarray(img, np.uint8)
    H, W = img.shape
    v = img.astype(np.int32)
    corner = np.zeros((H, W), bool)
    d = np.zeros((25, H, W), np.int32)
    if H < 7 or W < 7:
        return corner, d
    inner = (slice(3, H - 3), slice(3, W - 3))
    circ = np.stack([v[3 + dy:H - 3 + dy, 3 + dx:W - 3 + dx] for dx, dy in FAST_CIRCLE])
    c = v[inner]
    bright = circ > c + threshold
    dark = circ < c - threshold
    bb = np.concatenate([bright, bright[:8]])
    dd = np.concatenate([dark, dark[:8]])
    isc = np.zeros_like(c, bool)
    for k in range(16):
        isc |= bb[k:k + 9].all(0) | dd[k:k + 9].all(0)
    corner[inner] = isc
    dif = c[None] - circ
    d[:, 3:H - 3, 3:W - 3] = np.concatenate([dif, dif[:9]])
    return corner, d


def fast_detect(img, threshold, nonmax=True, mask=None):
    """FastFeatureDetector (TYPE_9_16) detect: keypoints in raster order (the
    order fast.cpp emits them).  Returns (xy (n, 2) float32, response (n,)
    int32).  With nonmax, a corner survives if its score is strictly greater
    than the scores of its 8 neighbours (non-corners score 0).  The mask
    (KeyPointsFilter::runByPixelsMask) is applied after the suppression."""
    img = np.asarray(img, np.uint8)
    H, W = img.shape
    corner, d = fast_corner_mask(img, threshold)
    score = np.zeros((H, W), np.int32)
    ys, xs = np.nonzero(corner)
    for y, x in zip(ys, xs):
        score[y, x] = _corner_score(d[:, y, x], threshold)
    keep = corner.copy()
    if nonmax:
        pad = np.zeros((H + 2, W + 2), np.int32)
        pad[1:-1, 1:-1] = score
        for dy in (-1, 0, 1):
            for dx in (-1, 0, 1):
                if dy == 0 and dx == 0:
                    continue
                keep &= score > pad[1 + dy:H + 1 + dy, 1 + dx:W + 1 + dx]
    if mask is not None:
        keep &= np.asarray(mask) != 0
    ys, xs = np.nonzero(keep)
    return np.stack([xs, ys], 1).astype(np.float32), score[ys, xs].astype(np.int32)


# -------------------------------------------------------------- pyramids --
def reflect101(i, n):
    """BORDER_REFLECT_101 index map (gfedcb|abcdefgh|gfedcba)."""
    i = np.asarray(i)
    if n == 1:
        return np.zeros_like(i)
    period = 2 * n - 2
    i = np.mod(i, period)
    return np.where(i >= n, period - i, i)


def pyr_down(img):
    """cv2.pyrDown of an 8-bit image: 5x5 Gaussian [1 4 6 4 1]^2 / 256 with
    BORDER_REFLECT_101, integer sums rounded as (s + 128) >> 8; output size
    ((W + 1) / 2, (H + 1) / 2)."""
    src = np.asarray(img, np.int64)
    H, W = src.shape
    h2, w2 = (H + 1) // 2, (W + 1) // 2
    k = np.array([1, 4, 6, 4, 1], np.int64)
    cols = reflect101(2 * np.arange(w2)[:, None] + np.arange(-2, 3)[None], W)   # (w2, 5)
    rows = reflect101(2 * np.arange(h2)[:, None] + np.arange(-2, 3)[None], H)   # (h2, 5)
    hs = (src[:, cols] * k).sum(-1)            # (H, w2)
    vs = (hs[rows] * k[None, :, None]).sum(1)  # (h2, w2)
    return ((vs + 128) >> 8).astype(np.uint8)


def build_pyramid(img, max_level):
    pyr = [np.asarray(img, np.uint8)]
    for _ in range(max_level):
        pyr.append(pyr_down(pyr[-1]))
    return pyr


def scharr(img):
    """calcScharrDeriv (lkpyramid.cpp): int16 (Ix, Iy) with 3-10-3 Scharr
    kernels, BORDER_REFLECT_101."""
    v = np.asarray(img, np.int32)
    H, W = v.shape
    yy = reflect101(np.arange(-1, H + 1), H)
    xx = reflect101(np.arange(-1, W + 1), W)
    p = v[yy][:, xx]
    ix = 3 * (p[:-2, 2:] + p[2:, 2:]) + 10 * p[1:-1, 2:] - (3 * (p[:-2, :-2] + p[2:, :-2]) + 10 * p[1:-1, :-2])
    iy = 3 * (p[2:, :-2] + p[2:, 2:]) + 10 * p[2:, 1:-1] - (3 * (p[:-2, :-2] + p[:-2, 2:]) + 10 * p[:-2, 1:-1])
    return ix.astype(np.int16), iy.astype(np.int16)


def _weights(a, b):
    """cvRound((1 - a) (1 - b) 2^14) etc., in float32 like lkpyramid.cpp
    (round half to even)."""
    a, b = np.float32(a), np.float32(b)
    one, sc = np.float32(1.0), np.float32(1 << W_BITS)
    iw00 = int(np.rint((one - a) * (one - b) * sc))
    iw01 = int(np.rint(a * (one - b) * sc))
    iw10 = int(np.rint((one - a) * b * sc))
    return iw00, iw01, iw10, (1 << W_BITS) - iw00 - iw01 - iw10


def _patch(src, x0, y0, win, w, zero_border=False):
    """Bilinear window (win x win) at integer corner (x0, y0) with fixed-point
    weights.  Beyond the edges the image is read with BORDER_REFLECT_101 (the
    pyramid's border) and the derivatives as zeros (zero_border): given raw
    images, calcOpticalFlowPyrLK pads derivI with copyMakeBorder(...,
    BORDER_CONSTANT) (lkpyramid.cpp), while calcScharrDeriv itself reflects
    inside the image."""
    H, W = src.shape
    ys, xs = np.arange(y0, y0 + win + 1), np.arange(x0, x0 + win + 1)
    if zero_border:
        inside = ((ys >= 0) & (ys < H))[:, None] & ((xs >= 0) & (xs < W))[None, :]
        p = np.where(inside, src[np.clip(ys, 0, H - 1)][:, np.clip(xs, 0, W - 1)], 0).astype(np.int64)
    else:
        p = src[reflect101(ys, H)][:, reflect101(xs, W)].astype(np.int64)
    return p[:-1, :-1] * w[0] + p[:-1, 1:] * w[1] + p[1:, :-1] * w[2] + p[1:, 1:] * w[3]


def lk_track(prev_img, next_img, prev_pts, next_pts, win=15, max_level=3, max_iter=30, eps=0.01):
    """calcOpticalFlowPyrLK with OPTFLOW_USE_INITIAL_FLOW (LKTrackerInvoker,
    lkpyramid.cpp): coarse-to-fine Lucas-Kanade per point.  Returns
    (next_pts (n, 2) float32, status (n,) uint8)."""
    prev_pts = np.asarray(prev_pts, np.float32).reshape(-1, 2)
    nxt = np.asarray(next_pts, np.float32).reshape(-1, 2).copy()
    n = len(prev_pts)
    status = np.ones(n, np.uint8)
    pp = build_pyramid(prev_img, max_level)
    npyr = build_pyramid(next_img, max_level)
    derivs = [scharr(p) for p in pp]
    half = np.float32((win - 1) * 0.5)
    for level in range(max_level, -1, -1):
        I, J = pp[level], npyr[level]
        Ix, Iy = derivs[level]
        H, W = I.shape
        for i in range(n):
            if not status[i] and level == 0:
                continue
            prev_pt = prev_pts[i] * np.float32(1.0 / (1 << level)) - half
            if level == max_level:
                nextp = nxt[i] * np.float32(1.0 / (1 << level))
            else:
                nextp = nxt[i] * np.float32(2.0)
            nxt[i] = nextp
            nextp = (nextp - half).astype(np.float32)
            ipx, ipy = int(np.floor(prev_pt[0])), int(np.floor(prev_pt[1]))
            if ipx < -win or ipx >= W or ipy < -win or ipy >= H:
                if level == 0:
                    status[i] = 0
                continue
            a, b = prev_pt[0] - np.float32(ipx), prev_pt[1] - np.float32(ipy)
            w = _weights(a, b)
            ival = _descale(_patch(I, ipx, ipy, win, w), W_BITS - 5)
            ixv = _descale(_patch(Ix, ipx, ipy, win, w, zero_border=True), W_BITS)
            iyv = _descale(_patch(Iy, ipx, ipy, win, w, zero_border=True), W_BITS)
            # window sums of integer products, exact (cv2 accumulates them in float;
            # the difference is below float32 resolution of the sums' ratio)
            A11 = np.float32(np.sum(ixv * ixv)) * np.float32(FLT_SCALE)
            A12 = np.float32(np.sum(ixv * iyv)) * np.float32(FLT_SCALE)
            A22 = np.float32(np.sum(iyv * iyv)) * np.float32(FLT_SCALE)
            D = A11 * A22 - A12 * A12
            min_eig = (A22 + A11 - np.sqrt((A11 - A22) * (A11 - A22) + 4.0 * A12 * A12)) / (2 * win * win)
            if min_eig < MIN_EIG_THRESHOLD or D < np.finfo(np.float32).eps:
                if level == 0:
                    status[i] = 0
                continue
            D = np.float32(1.0) / D
            prev_delta = np.zeros(2, np.float32)
            for j in range(max_iter):
                inx, iny = int(np.floor(nextp[0])), int(np.floor(nextp[1]))
                if inx < -win or inx >= W or iny < -win or iny >= H:
                    if level == 0:
                        status[i] = 0
                    break
                a, b = nextp[0] - np.float32(inx), nextp[1] - np.float32(iny)
                w = _weights(a, b)
                diff = _descale(_patch(J, inx, iny, win, w), W_BITS - 5) - ival
                b1 = np.float32(np.sum(diff * ixv)) * np.float32(FLT_SCALE)
                b2 = np.float32(np.sum(diff * iyv)) * np.float32(FLT_SCALE)
                delta = np.array([(A12 * b2 - A22 * b1) * D, (A12 * b1 - A11 * b2) * D], np.float32)
                nextp = (nextp + delta).astype(np.float32)
                nxt[i] = nextp + half
                if float(delta[0]) ** 2 + float(delta[1]) ** 2 <= eps * eps:   # delta.ddot(delta), double
                    break
                if j > 0 and abs(delta[0] + prev_delta[0]) < 0.01 and abs(delta[1] + prev_delta[1]) < 0.01:
                    nxt[i] -= delta * np.float32(0.5)
                    break
                prev_delta = delta
    return nxt, status


# --------------------------------------------------- camera models ----
def undistort_points(pts, intrinsics, model, coeffs, R=np.eye(3), new_intrinsics=(1, 1, 0, 0), iters=None):
    """cv2.undistortPoints (radtan: 5 fixed-point iterations, undistort.cpp)
    or cv2.fisheye.undistortPoints (equidistant: Newton on theta, at most 10
    steps, stopping below 1e-8; cv2 4.x's rejection of non-converged or
    sign-flipped theta as (-1e6, -1e6)), then the rectification R and the
    new camera matrix."""
    pts = np.asarray(pts, float).reshape(-1, 2)
    fx, fy, cx, cy = map(float, intrinsics)
    k = np.asarray(coeffs, float)
    x = (pts[:, 0] - cx) / fx
    y = (pts[:, 1] - cy) / fy
    bad = np.zeros(len(x), bool)
    if model == "equidistant":
        # cv2 4.x with its default criteria (COUNT + EPS, 10, 1e-8):
        # theta_d clamped to pi / 2, Newton until |step| < 1e-8, scale 0 at
        # theta_d <= 1e-8; non-converged or sign-flipped solutions -> (-1e6, -1e6)
        td = np.minimum(np.sqrt(x * x + y * y), np.pi / 2)
        th = td.copy()
        conv = td <= 1e-8
        for _ in range(iters or 10):
            t2 = th * th
            t4 = t2 * t2
            t6 = t4 * t2
            t8 = t6 * t2
            k0t2, k1t4, k2t6, k3t8 = k[0] * t2, k[1] * t4, k[2] * t6, k[3] * t8
            fix = (th * (1 + k0t2 + k1t4 + k2t6 + k3t8) - td) / (1 + 3 * k0t2 + 5 * k1t4 + 7 * k2t6 + 9 * k3t8)
            step = ~conv
            th = np.where(step, th - fix, th)
            conv = conv | (step & (np.abs(fix) < 1e-8))
        scale = np.where(td > 1e-8, np.tan(th) / np.where(td > 1e-8, td, 1), 0.0)
        bad = ~conv | (th < 0)
        x, y = x * scale, y * scale
    else:
        k1, k2, p1, p2 = k[:4]
        k3 = k[4] if len(k) > 4 else 0.0
        x0, y0 = x.copy(), y.copy()
        for _ in range(iters or 5):
            r2 = x * x + y * y
            icdist = 1.0 / (1 + ((k3 * r2 + k2) * r2 + k1) * r2)
            dx = 2 * p1 * x * y + p2 * (r2 + 2 * x * x)
            dy = p1 * (r2 + 2 * y * y) + 2 * p2 * x * y
            x = (x0 - dx) * icdist
            y = (y0 - dy) * icdist
    R = np.asarray(R, float)
    X = R[0, 0] * x + R[0, 1] * y + R[0, 2]
    Y = R[1, 0] * x + R[1, 1] * y + R[1, 2]
    Wz = R[2, 0] * x + R[2, 1] * y + R[2, 2]
    nfx, nfy, ncx, ncy = map(float, new_intrinsics)
    out = np.stack([nfx * X / Wz + ncx, nfy * Y / Wz + ncy], 1)
    out[bad] = -1000000.0
    return out


def distort_points(pts, intrinsics, model, coeffs):
    """cv2.projectPoints of (x, y, 1) with zero pose (radtan) or
    cv2.fisheye.distortPoints (equidistant)."""
    pts = np.asarray(pts, float).reshape(-1, 2)
    fx, fy, cx, cy = map(float, intrinsics)
    k = np.asarray(coeffs, float)
    x, y = pts[:, 0], pts[:, 1]
    if model == "equidistant":
        r = np.sqrt(x * x + y * y)
        th = np.arctan(r)
        t2 = th * th
        td = th * (1 + k[0] * t2 + k[1] * (t2 * t2) + k[2] * (t2 * t2 * t2) + k[3] * (t2 * t2 * t2 * t2))
        s = np.where(r > 1e-8, td / np.where(r > 1e-8, r, 1), 1.0)
        xd, yd = x * s, y * s
    else:
        k1, k2, p1, p2 = k[:4]
        k3 = k[4] if len(k) > 4 else 0.0
        r2 = x * x + y * y
        radial = 1 + k1 * r2 + k2 * r2 * r2 + k3 * r2 * r2 * r2
        xd = x * radial + 2 * p1 * x * y + p2 * (r2 + 2 * x * x)
        yd = y * radial + p1 * (r2 + 2 * y * y) + 2 * p2 * x * y
    return np.stack([fx * xd + cx, fy * yd + cy], 1)


def rodrigues(rvec):
    """cv2.Rodrigues (rotation vector -> matrix)."""
    r = np.asarray(rvec, float).reshape(3)
    th = np.linalg.norm(r)
    if th < 1e-300:
        return np.eye(3)
    k = r / th
    K = np.array([[0, -k[2], k[1]], [k[2], 0, -k[0]], [-k[1], k[0], 0]])
    return np.cos(th) * np.eye(3) + (1 - np.cos(th)) * np.outer(k, k) + np.sin(th) * K
