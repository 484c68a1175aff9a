"""The front-end host mirror (msckf_amd.frontend.ImageProcessor) against the
reference's own ImageProcessor (MSCKF/image.py:36-702), whose published
messages were recorded in the build container behind a cv2 stand-in made of
the oracle operators (tools/gen_frontend_golden.py -> frontend_ref.npz).

Here (CPU) the mirror runs on the SAME oracle operators -- a stand-in for the
device context, like bench.py --stub -- so everything image.py does around
cv2 is checked exactly: grid bucketing, id assignment, response and lifetime
ordering, pruning, the stereo gates (round trip < 3 px, vertical disparity <
20 px, epipolar), the IMU rotation prediction and the publish order.  Ids
must be identical and coordinates equal to 1e-12.  tests/test_gpu_frontend.py
repeats it on the HIP operators.  (The operators stay parity-unpinned against
cv2 itself: DESIGN.md section 5.10.)"""
import numpy as np
import pytest

import msckf_amd.frontend as fe_mod
from conftest import golden
from frontend_ref_scenes import SCENES, scene_config, run_scene, reference_frames
from oracle import frontend_oracle as fo


class OracleFrontend:
    """The mfe_* operators of msckf_amd.frontend.Frontend, restated on the CPU
    oracle (test stand-in for the device context)."""

    def __init__(self, width, height, nslot=4, max_level=3, max_points=4096, device=0):
        self.W, self.H, self.slots = int(width), int(height), {}

    def upload(self, slot, image):
        self.slots[slot] = np.ascontiguousarray(image, np.uint8)

    def fast(self, slot, threshold, mask=None, max_kp=1 << 16):
        xy, resp = fo.fast_detect(self.slots[slot], threshold, nonmax=True, mask=mask)
        return xy, resp.astype(np.float32)

    def lk(self, slot_prev, slot_next, prev_pts, next_pts, win=15, max_level=3, max_iter=30, eps=0.01):
        return fo.lk_track(self.slots[slot_prev], self.slots[slot_next], prev_pts, next_pts, win=win,
                           max_level=max_level, max_iter=max_iter, eps=eps)

    def undistort(self, pts, intrinsics, model, coeffs, R=None, new_intrinsics=None):
        return fo.undistort_points(pts, intrinsics, "equidistant" if model == fe_mod.EQUIDISTANT else "radtan",
                                   coeffs, np.eye(3) if R is None else R,
                                   (1, 1, 0, 0) if new_intrinsics is None else new_intrinsics)

    def distort(self, pts, intrinsics, model, coeffs):
        return fo.distort_points(pts, intrinsics, "equidistant" if model == fe_mod.EQUIDISTANT else "radtan", coeffs)

    def close(self):
        pass


@pytest.mark.parametrize("name", SCENES)
def test_image_processor_bookkeeping_vs_reference(name, monkeypatch):
    g = golden("frontend_ref")
    monkeypatch.setattr(fe_mod, "Frontend", OracleFrontend)
    ip = fe_mod.ImageProcessor(scene_config(g, name))
    got = run_scene(ip, g, name)
    for k, ((ids, uv), (rids, ruv)) in enumerate(zip(got, reference_frames(g, name))):
        np.testing.assert_array_equal(ids, rids, err_msg="frame %d" % k)
        np.testing.assert_allclose(uv, ruv, rtol=0, atol=1e-12, err_msg="frame %d" % k)
    assert len(got) == int(g[name + "_frames"]) and len(got[-1][0]) >= 50
