"""Batched multi-sequence scheduler on the GPU:
several sequences on one context, every request kind served by one batched
launch, must reproduce each sequence run alone through the drop-in class --
and the golden lane must still match the reference filter's own run."""
import numpy as np
import pytest

import msckf_amd
from conftest import golden
from msckf_amd import synth
from msckf_amd.replay import FeatureStream, replay
from msckf_amd.scheduler import MultiMSCKF
from msckf_amd.trajectory import Trajectory, ate

pytestmark = pytest.mark.gpu


def _late_start(st: FeatureStream, k0):
    """The same stream with its first k0 frames dropped (its prune rounds then
    fall on other lock-step rounds than the other lanes')."""
    a = int(st.frame_off[k0])
    return FeatureStream(st.imu, st.frame_t[k0:], st.frame_off[k0:] - a, st.feat_id[a:], st.feat_z[a:], st.gt)


def _streams():
    g = golden("sequence_s1")
    s1 = FeatureStream.from_synthetic(synth.make_sequence(int(g["n_frames"]), int(g["seed"])))
    s2 = FeatureStream.from_synthetic(synth.make_sequence(90, 7))
    s3 = _late_start(FeatureStream.from_synthetic(synth.make_sequence(140, 11)), 7)
    return g, [s1, s2, s3]


def _single(st):
    flt = msckf_amd.MSCKF()
    try:
        traj = replay(flt, st)
        return traj, flt.gate_log, flt.shape_log, flt.state_cov()
    finally:
        flt.close()


def test_scheduler_matches_single_filter_runs():
    g, streams = _streams()
    multi = MultiMSCKF(len(streams))
    try:
        trajs = multi.run_streams(streams)
        logs = [(ln.gate_log, ln.shape_log, ln.state_cov()) for ln in multi.lanes]
        launches = dict(multi.launches)
    finally:
        multi.close()
    for i, st in enumerate(streams):
        t1, gl, sl, P = _single(st)
        np.testing.assert_array_equal(trajs[i].t, t1.t)
        assert np.array(logs[i][0]).tolist() == np.array(gl).tolist(), i
        assert np.array(logs[i][1]).tolist() == np.array(sl).tolist(), i
        assert np.abs(trajs[i].p - t1.p).max() <= 1e-9 * max(1.0, np.abs(t1.p).max()), i
        assert np.linalg.norm(logs[i][2] - P) <= 1e-9 * np.linalg.norm(P), i
    # the golden lane against the reference filter's own trajectory
    ref = Trajectory(g["rec"][:, 0], g["rec"][:, 5:8])
    assert ate(trajs[0], ref, align="none") <= 1e-6 * np.sqrt(np.mean(np.sum(ref.p ** 2, 1)))
    # one batched launch per kind per round, not one per filter
    n_rounds = max(s.n_frames for s in streams)
    assert launches["augment"] <= n_rounds
    print("scheduler launches:", launches)


def test_scheduler_fp32_runs_and_tracks():
    streams = [FeatureStream.from_synthetic(synth.make_sequence(80, s)) for s in (21, 22, 23, 24)]
    multi = MultiMSCKF(len(streams), dtype=np.float32)
    try:
        trajs = multi.run_streams(streams)
    finally:
        multi.close()
    for st, tr in zip(streams, trajs):
        assert ate(tr, st.gt) < 0.1
