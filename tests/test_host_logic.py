"""Host-side logic of the drop-in MSCKF class (no GPU): the pieces the
reference keeps in Python and this package keeps on the host too (SURVEY.md
8(b)) -- check_motion and the keyframe choice -- against fixtures generated
by running the reference (tools/gen_golden.py)."""
from collections import OrderedDict

import numpy as np

from conftest import golden
import msckf_amd
from msckf_amd.msckf import MSCKF, check_motion


def test_check_motion_matches_reference():
    """feature.py:124-165 at thresholds -1, 0.2 and 0.4."""
    g = golden("check_motion")
    cams = {i: dict(q=g["cam_q"][i], p=g["cam_p"][i]) for i in range(len(g["cam_q"]))}
    for thr, key in ((-1.0, "ok_m1"), (0.2, "ok_2"), (0.4, "ok_4")):
        res = []
        for j in range(len(g["first"])):
            obs = OrderedDict((c, g["z"][j] + 0.01 * (c - g["first"][j]))
                              for c in range(int(g["first"][j]), int(g["last"][j]) + 1))
            res.append(check_motion(obs, cams, thr))
        np.testing.assert_array_equal(res, g[key])


def test_find_redundant_cam_states_matches_reference():
    """msckf.py:691-727 through the product's host method, at tracking rates
    0.3 and 0.9 (reference outputs rm_3 / rm_9)."""
    g = golden("prune")
    flt = MSCKF.__new__(MSCKF)          # host logic only: no device context
    n = int(g["N"])
    flt.cam_ids = list(range(n))
    cams_arr = np.hstack([g["cam_q"], g["cam_p"], g["cam_q_null"]])
    for tr, key in ((0.3, "rm_3"), (0.9, "rm_9")):
        flt.tracking_rate = tr
        assert flt._find_redundant_cam_states(cams_arr) == [int(c) for c in g[key]]
    assert list(g["rm_3"]) != list(g["rm_9"])
