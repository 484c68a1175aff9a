"""CPU checks pinning the front-end oracle (oracle/frontend_oracle.py).  cv2
is absent here, so the restated OpenCV operators are pinned by analytic
properties instead of cv2 outputs (parity unpinned against cv2 itself):
FAST's score is the largest threshold keeping the corner, non-max keeps
strict local maxima, pyrDown preserves constants, Scharr differentiates a ramp
exactly, LK recovers a known sub-pixel motion of a continuous scene, the camera
models invert each other and Rodrigues builds rotations."""
import numpy as np
import pytest

from oracle import frontend_oracle as fo
import frontend_synth as fs


@pytest.fixture(scope="module")
def tex():
    f = fs.texture_fn(1, W=200, H=150)
    return f, fs.render(f, 200, 150)


def test_fast_score_is_largest_threshold(tex):
    _, img = tex
    corner, d = fo.fast_corner_mask(img, 15)
    ys, xs = np.nonzero(corner)
    assert len(ys) > 100
    for y, x in list(zip(ys, xs))[::7]:
        s = fo._corner_score(d[:, y, x], 15)
        assert s >= 15
        assert fo.fast_corner_mask(img, s)[0][y, x]
        assert not fo.fast_corner_mask(img, s + 1)[0][y, x]


def test_fast_nonmax_and_mask(tex):
    _, img = tex
    xy_all, r_all = fo.fast_detect(img, 15, nonmax=False)
    xy, r = fo.fast_detect(img, 15)
    assert 0 < len(xy) < len(xy_all)
    corner, d = fo.fast_corner_mask(img, 15)
    score = np.zeros(img.shape, int)
    for (x, y), s in zip(xy_all.astype(int), r_all):
        score[y, x] = s
    for (x, y), s in zip(xy.astype(int), r):
        nb = score[y - 1:y + 2, x - 1:x + 2].copy()
        nb[1, 1] = -1
        assert s > nb.max()
    # raster order, and the mask only removes points
    order = xy[:, 1] * 10000 + xy[:, 0]
    assert (np.diff(order) > 0).all()
    mask = np.ones(img.shape, np.uint8)
    mask[:, :100] = 0
    xm, _ = fo.fast_detect(img, 15, mask=mask)
    np.testing.assert_array_equal(xm, xy[xy[:, 0] >= 100])
    # degenerate plateaus (axis-aligned squares) keep no corner: ties are not maxima
    sq, _ = fs.squares()
    assert len(fo.fast_detect(sq, 15)[0]) == 0 and len(fo.fast_detect(sq, 15, nonmax=False)[0]) > 0


def test_pyr_down_and_scharr():
    c = np.full((37, 51), 93, np.uint8)
    p = fo.pyr_down(c)
    assert p.shape == (19, 26) and (p == 93).all()
    ramp = (np.arange(40)[None, :] * 3 + np.zeros((30, 1), int)).astype(np.uint8)
    ix, iy = fo.scharr(ramp)
    assert (ix[:, 1:-1] == 32 * 3).all() and (iy == 0).all()
    assert (ix[:, 0] == 0).all() and (ix[:, -1] == 0).all()   # REFLECT_101 mirrors the ramp at the edges


def test_lk_recovers_known_motion(tex):
    f, img = tex
    moved = fs.render(f, 200, 150, 1.35, -0.8)
    xy, _ = fo.fast_detect(img, 15)
    pts = xy[(xy[:, 0] > 30) & (xy[:, 0] < 170) & (xy[:, 1] > 30) & (xy[:, 1] < 120)][:30]
    nxt, st = fo.lk_track(img, moved, pts, pts)
    assert st.all()
    err = np.abs(nxt - pts - np.array([1.35, -0.8]))
    assert np.median(err) < 0.02 and err.max() < 0.1
    # a larger motion needs the pyramid
    far = fs.render(f, 200, 150, 9.0, 5.5)
    nxt, st = fo.lk_track(img, far, pts, pts)
    ok = st.astype(bool)
    assert ok.mean() > 0.8
    assert np.median(np.abs(nxt[ok] - pts[ok] - np.array([9.0, 5.5]))) < 0.05


@pytest.mark.parametrize("model,coeffs", [("radtan", [-0.28340811, 0.07395907, 0.00019359, 1.76187114e-05]),
                                          ("equidistant", [0.01, -0.005, 0.001, -0.0002])])
def test_camera_models_invert(model, coeffs):
    K = [458.654, 457.296, 367.215, 248.375]
    rng = np.random.default_rng(3)
    xn = rng.uniform(-0.3, 0.3, (50, 2))
    px = fo.distort_points(xn, K, model, coeffs)
    back = fo.undistort_points(px, K, model, coeffs, iters=50)
    np.testing.assert_allclose(back, xn, atol=1e-9)
    # the reference's 5 fixed-point iterations (radtan) stay within 1e-3 normalised units here
    np.testing.assert_allclose(fo.undistort_points(px, K, model, coeffs), xn, atol=1e-3)
    # rectification and new intrinsics: a pure rotation about the optical axis
    c, s = np.cos(0.1), np.sin(0.1)
    R = np.array([[c, -s, 0], [s, c, 0], [0, 0, 1]])
    out = fo.undistort_points(px, K, model, coeffs, R=R, new_intrinsics=(2, 3, 1, -1), iters=50)
    np.testing.assert_allclose(out, np.stack([2 * (c * xn[:, 0] - s * xn[:, 1]) + 1,
                                              3 * (s * xn[:, 0] + c * xn[:, 1]) - 1], 1), atol=1e-9)


def test_rodrigues():
    r = np.array([0.3, -0.2, 0.5])
    R = fo.rodrigues(r)
    np.testing.assert_allclose(R @ R.T, np.eye(3), atol=1e-14)
    np.testing.assert_allclose(R @ r, r, atol=1e-14)
    assert np.isclose(np.arccos((np.trace(R) - 1) / 2), np.linalg.norm(r))


def test_lk_derivatives_zero_beyond_image():
    """calcOpticalFlowPyrLK, given raw images, pads the Scharr derivatives
    with zeros (copyMakeBorder BORDER_CONSTANT, lkpyramid.cpp) while the
    image pyramid reflects.  Hand-worked window: a horizontal ramp
    v = 4 x has Ix = 16 (v(x+1) - v(x-1)) = 128 inside the image, 0 in column
    0 (Scharr's own REFLECT_101 there) and Iy = 0.  The 15 x 15 window at
    integer corner (-5, 20) with unit weights covers columns -5..9: five
    zero-padded columns, column 0 and nine columns of 128, so
    A11 = 15 * 9 * 128^2 (a reflected border would count 14 columns)."""
    W, H = 64, 48
    img = np.tile((4 * np.arange(W)).astype(np.uint8), (H, 1))
    ix, iy = fo.scharr(img)
    assert (ix[:, 1:W - 1] == 128).all() and (ix[:, 0] == 0).all() and (iy == 0).all()
    w = (1 << fo.W_BITS, 0, 0, 0)
    ixv = fo._descale(fo._patch(ix, -5, 20, 15, w, zero_border=True), fo.W_BITS)
    iyv = fo._descale(fo._patch(iy, -5, 20, 15, w, zero_border=True), fo.W_BITS)
    assert int(np.sum(ixv.astype(np.int64) ** 2)) == 15 * 9 * 128 ** 2
    assert int(np.sum(ixv.astype(np.int64) * iyv)) == 0 and int(np.sum(iyv.astype(np.int64) ** 2)) == 0
    refl = fo._descale(fo._patch(ix, -5, 20, 15, w), fo.W_BITS)   # the image border rule, for contrast
    assert int(np.sum(refl.astype(np.int64) ** 2)) == 15 * 14 * 128 ** 2


def test_fisheye_undistort_rejects_unsolvable_theta():
    """cv2 4.x fisheye.undistortPoints: Newton stops below 1e-8 and a
    non-converged or sign-flipped theta comes back as (-1e6, -1e6).  With
    k = (-1, 0, 0, 0), theta_d = theta (1 - theta^2) peaks at 0.385 (theta =
    1/sqrt 3): theta_d = 0.6 has no solution, theta_d = 0.2 has one that the
    forward model maps back."""
    k = [-1.0, 0.0, 0.0, 0.0]
    bad = fo.undistort_points([[0.6, 0.0]], (1, 1, 0, 0), "equidistant", k)
    assert (bad == -1000000.0).all()
    good = fo.undistort_points([[0.2, 0.1]], (1, 1, 0, 0), "equidistant", k)
    assert np.isfinite(good).all() and (good > -1000.0).all()
    back = fo.distort_points(good, (1, 1, 0, 0), "equidistant", k)
    np.testing.assert_allclose(back, [[0.2, 0.1]], atol=1e-9)
