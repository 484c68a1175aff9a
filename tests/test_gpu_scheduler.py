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
    try:   # messages built beforehand, as tools/bench_sequences.py times it
        trajs = multi.run_streams(streams, messages=[s.messages() for s in streams])
    finally:
        multi.close()
    for st, tr in zip(streams, trajs):
        assert ate(tr, st.gt) < 0.1


def test_readback_equals_separate_reads():
    """msckf_readback (a frame's sync point in one synchronisation) returns what
    msckf_get_states_batch, msckf_get_cov_diag_batch and msckf_batch_results
    return separately -- bit for bit -- and settles the outstanding deferred
    batch, so the Pending needs no read of its own."""
    g, streams = _streams()
    ms = MultiMSCKF(3)
    try:
        ms.run_streams([s for s in streams])
        ctx = ms.ctx
        slots = [0, 2, 1]
        lane = ms.lanes[0]
        # one deferred update on lane 0's current features (positions from the map)
        feats = [f for f in lane.map_server.values() if f.is_initialized and len(f.observations) >= 2][:12]
        assert feats, "no initialised features left in the map"
        cl = [list(f.observations) for f in feats]
        off, cams, zs = lane._pack(feats, cl)
        pw = np.array([f.position for f in feats])
        pend = ctx.update_async(0, off, cams, zs, pw, np.full(len(feats), 1e9), 0)
        imu, cl_rb, cv = ctx.readback(slots, cov=(12, 3))
        assert ctx._pending is None and pend.grp.res is not None    # settled by the readback
        acc, gam, p, v, rows = pend.get()
        imu2, cl2 = ctx.get_states_batch(slots)
        cv2 = ctx.cov_diag_batch(slots, 12, 3)
        acc2, gam2, p2, v2, rows2 = ctx.batch_results()
        np.testing.assert_array_equal(imu, imu2)
        for a, b in zip(cl_rb, cl2):
            np.testing.assert_array_equal(a, b)
        np.testing.assert_array_equal(cv, cv2)
        np.testing.assert_array_equal(acc, acc2[:len(feats)])
        np.testing.assert_array_equal(gam, gam2[:len(feats)])
        np.testing.assert_array_equal(p, p2[:len(feats)])
        np.testing.assert_array_equal(v, v2[:len(feats)])
        assert rows == int(rows2[0]) and rows > 0
    finally:
        ms.close()


@pytest.mark.parametrize("B", [4, 600])
def test_readback_gather_and_copy_paths(B):
    """msckf_readback moves a sync point's arrays to the host either with one
    gather kernel that stores into the pinned buffer (<= 8 arrays and <= 1 MiB:
    B = 4) or with one runtime copy per array (B = 600: the cam records of the
    context alone are ~3 MB).  Both must return exactly what set_state stored
    (fp64 context: bit-exact) and the listed filters' covariance diagonals, for
    a scrambled filter list."""
    from msckf_amd import FilterConfig
    from msckf_amd._lib import CAM_LEN, IMU_LEN, Context
    rng = np.random.default_rng(B)
    N = 32
    ctx = Context(FilterConfig(), n_filters=B, n_cam_capacity=N, dtype=np.float64)
    try:
        imus, camss, diags = [], [], []
        for f in range(B):
            n = int(rng.integers(2, N + 1))
            D = 21 + 6 * n
            imu = rng.standard_normal(IMU_LEN)
            cams = rng.standard_normal((n, CAM_LEN))
            P = np.diag(rng.uniform(0.5, 2.0, D)) + 1e-3 * np.ones((D, D))
            ctx.set_state(f, imu, cams, P)
            imus.append(imu)
            camss.append(cams)
            diags.append(np.diag(P).copy())
        filters = rng.permutation(B)[:min(B, 64)]
        imu_rb, cl, cv = ctx.readback(filters, cov=(3, 10))
        for w, f in enumerate(filters):
            np.testing.assert_array_equal(imu_rb[w], imus[f])
            np.testing.assert_array_equal(cl[w], camss[f])
            np.testing.assert_array_equal(cv[w], diags[f][3:13])
    finally:
        ctx.close()
