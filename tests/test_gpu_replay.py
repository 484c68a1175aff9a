"""Deterministic replay through the drop-in MSCKF class on the GPU
(SURVEY.md 8(f) items 1-2): ATE vs the reference filter's own trajectory on
golden sequence_s1 (north-star tolerance 1e-6 relative on the state, here as
an absolute position RMSE) and ATE vs the synthetic ground truth."""
import numpy as np
import pytest

import msckf_amd
from conftest import golden
from msckf_amd import synth
from msckf_amd.replay import FeatureStream, replay
from msckf_amd.trajectory import Trajectory, ate

pytestmark = pytest.mark.gpu


def test_replay_ate_vs_reference():
    g = golden("sequence_s1")
    st = FeatureStream.from_synthetic(synth.make_sequence(int(g["n_frames"]), int(g["seed"])))
    flt = msckf_amd.MSCKF()
    try:
        traj = replay(flt, st)
    finally:
        flt.close()
    ref = Trajectory(g["rec"][:, 0], g["rec"][:, 5:8])
    np.testing.assert_array_equal(traj.t, ref.t)
    scale = np.sqrt(np.mean(np.sum(ref.p ** 2, axis=1)))
    e_ref = ate(traj, ref, align="none")
    e_gt = ate(traj, st.gt)
    print("replay: ATE vs ref %.3e m (path rms %.2f m), ATE vs GT %.4f m" % (e_ref, scale, e_gt))
    assert e_ref <= 1e-6 * scale
    assert e_gt < 0.05
