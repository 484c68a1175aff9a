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


class _FakePending:
    def __init__(self, res):
        self.res, self.reads = res, 0

    def get(self):
        self.reads += 1
        return self.res


def test_deferred_update_log_and_fused_triangulation():
    """The update request goes down without a wait: features to initialise carry
    NaN positions (triangulated in the same device chain), and the decision
    log / new positions are applied at the next sync point, in the order the
    reference's measurement loop logs them (msckf.py:640-682): a failed
    triangulation is never gated, and logging stops at the row-cap break."""
    from msckf_amd.msckf import Feature
    flt = MSCKF.__new__(MSCKF)          # host logic only: no device context
    flt.cam_ids = list(range(6))
    flt._n_published = 7
    flt.gate_log, flt.gamma_log, flt.shape_log, flt._deferred = [], [], [], []
    feats = []
    for k in range(4):
        f = Feature(k)
        for c in range(k, k + 3):
            f.observations[c] = (0.0, 0.0, 0.0, 0.0)
        f.position = np.array([1.0, 2.0, 3.0 + k])
        f.is_initialized = k % 2 == 0
        feats.append(f)
    to_init = [f for f in feats if not f.is_initialized]           # features 1 and 3
    cam_lists = [list(f.observations) for f in feats]
    gen = flt._update(feats, cam_lists, [2] * 4, 15, to_init)
    req = next(gen)
    assert req[0] == "update" and req[6] == 15
    pw = req[4]
    assert np.isnan(pw[1]).all() and np.isnan(pw[3]).all()
    np.testing.assert_array_equal(pw[0], [1.0, 2.0, 3.0])
    # device: feature 1's triangulation fails; 0, 2 and 3 pass the gate (chi2.ppf(0.05, 2) = 0.103)
    p = np.arange(12.0).reshape(4, 3)
    res = (np.array([1, 0, 1, 0], bool), np.array([0.01, np.nan, 0.02, 0.03]), p,
           np.array([1, 0, 1, 1], bool), 18)
    pend = _FakePending(res)
    try:
        gen.send(pend)
    except StopIteration:
        pass
    assert flt.gate_log == [] and pend.reads == 0                   # nothing read yet
    flt._settle()
    assert pend.reads == 1
    # 9 rows each: the cap of 15 breaks after feature 2 (count 18), so 3 is never logged
    assert flt.gate_log == [(7, 2, 9, 1), (7, 2, 9, 1)]
    assert flt.shape_log == [(7, 18, 21 + 36)]
    assert feats[1].is_initialized is False and feats[3].is_initialized is True
    np.testing.assert_array_equal(feats[3].position, p[3])
    np.testing.assert_array_equal(feats[0].position, [1.0, 2.0, 3.0])   # given positions untouched
    assert [fid for fid, _ in flt.gamma_log] == [0, 2]
    # every candidate needs triangulation and every one fails: the reference's
    # processed list is empty, so it returns before measurement_update and
    # logs neither a decision nor a stacked shape (msckf.py:652-654)
    flt.gate_log, flt.gamma_log, flt.shape_log = [], [], []
    gen = flt._update(feats[1:4:2], cam_lists[1:4:2], [2] * 2, 15, feats[1:4:2])
    next(gen)
    pend = _FakePending((np.zeros(2, bool), np.full(2, np.nan), np.zeros((2, 3)), np.zeros(2, bool), 0))
    try:
        gen.send(pend)
    except StopIteration:
        pass
    flt._settle()
    assert flt.gate_log == [] and flt.shape_log == [] and flt.gamma_log == []
