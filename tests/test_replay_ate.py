"""Replay stream format, EuRoC readers and the ATE evaluator (SURVEY.md 8(f)
items 1-2) -- CPU only.  The oracle replay at the end pins the deterministic
driver to the reference filter's own 200-frame run (golden sequence_s1)."""
import os

import numpy as np
import pytest

from conftest import golden
from msckf_amd import synth, FilterConfig, chi2_threshold
from msckf_amd.euroc import EuRoC, write_euroc_layout, quat_wxyz_to_rotation
from msckf_amd.geometry import to_quaternion
from msckf_amd.replay import FeatureStream, Recorder
from msckf_amd.trajectory import Trajectory, associate, umeyama, ate_rmse, ate


def _rot(rng):
    q, _ = np.linalg.qr(rng.standard_normal((3, 3)))
    return q * np.sign(np.linalg.det(q))


def test_umeyama_recovers_transform():
    rng = np.random.default_rng(0)
    src = rng.standard_normal((50, 3))
    R, t, s = _rot(rng), rng.standard_normal(3), 1.7
    dst = s * src @ R.T + t
    R1, t1, s1 = umeyama(src, dst, with_scale=True)
    np.testing.assert_allclose(R1, R, atol=1e-12)
    np.testing.assert_allclose(t1, t, atol=1e-12)
    assert abs(s1 - s) < 1e-12
    R2, t2, s2 = umeyama(src, src @ R.T + t)
    np.testing.assert_allclose(R2, R, atol=1e-12)
    assert s2 == 1.0
    assert ate_rmse(src, src @ R.T + t) < 1e-12
    assert ate_rmse(src, dst, align="sim3") < 1e-12


def test_umeyama_reflection_guard_and_errors():
    rng = np.random.default_rng(1)
    src = rng.standard_normal((20, 3))
    dst = src * np.array([1, 1, -1])            # a reflection is not a rotation
    R, _, _ = umeyama(src, dst)
    assert np.linalg.det(R) > 0
    with pytest.raises(ValueError):
        umeyama(src[:2], dst[:2])
    with pytest.raises(ValueError):
        umeyama(src, dst[:, :2])


def test_ate_rmse_of_known_noise():
    rng = np.random.default_rng(2)
    p = np.cumsum(rng.standard_normal((400, 3)) * 0.1, axis=0)
    off = np.array([0.01, 0.0, 0.0])
    e = ate_rmse(p + off * np.where(np.arange(400) % 2, 1, -1)[:, None], p, align="none")
    assert abs(e - 0.01) < 1e-12


def test_associate():
    ta = np.array([0.0, 0.1, 0.2, 0.31, 5.0])
    tb = np.arange(0, 1, 0.05) + 0.001
    i, j = associate(ta, tb, max_dt=0.02)
    np.testing.assert_array_equal(i, [0, 1, 2, 3])
    np.testing.assert_allclose(tb[j], [0.001, 0.101, 0.201, 0.301])
    i, j = associate([], tb)
    assert len(i) == 0


@pytest.fixture(scope="module")
def seq():
    return synth.make_sequence(40, seed=3)


def test_stream_roundtrips(tmp_path, seq):
    st = FeatureStream.from_synthetic(seq, meta={"name": "synthetic-s3"})
    assert st.n_frames == len(seq.frames)
    ld = FeatureStream.load(st.save(str(tmp_path / "s.npz")))
    for k in ("imu", "frame_t", "frame_off", "feat_id", "feat_z"):
        np.testing.assert_array_equal(getattr(ld, k), getattr(st, k))
    np.testing.assert_array_equal(ld.gt.p, seq.gt_p)
    assert ld.meta == {"name": "synthetic-s3"}
    cv = FeatureStream.load_csv(st.save_csv(str(tmp_path / "csv")))
    for k in ("imu", "frame_t", "frame_off", "feat_id", "feat_z"):
        np.testing.assert_array_equal(getattr(cv, k), getattr(st, k))


def test_stream_events_match_sequence_order(seq):
    st = FeatureStream.from_synthetic(seq)
    ev = st.events()
    ref = seq.events()
    assert [k for k, _ in ev] == [k for k, _ in ref]
    for (k, a), (_, b) in zip(ev, ref):
        if k == 0:
            assert a.vio_timestamp__ == b.vio_timestamp__
            np.testing.assert_array_equal(a.angular_velocity, b.angular_velocity)
        else:
            assert a.timestamp == b.timestamp
            assert [f.id for f in a.vio_features] == [f.id for f in b.vio_features]
            assert [f.u1 for f in a.vio_features] == [f.u1 for f in b.vio_features]


def test_stream_empty_frames_and_validation(tmp_path):
    imu = np.array([[0.0, 0, 0, 0, 0, 0, 9.81], [0.005, 0, 0, 0, 0, 0, 9.81]])
    st = FeatureStream(imu, np.array([0.0, 0.05]), np.array([0, 0, 1]), np.array([7]),
                       np.array([[0.1, 0.2, 0.05, 0.2]])).validate()
    cv = FeatureStream.load_csv(st.save_csv(str(tmp_path / "c")))
    np.testing.assert_array_equal(cv.frame_off, [0, 0, 1])
    assert [k for k, _ in st.events()] == [0, 1, 0, 1]
    with pytest.raises(ValueError):
        FeatureStream(imu, np.array([0.0]), np.array([0, 2]), np.array([7]), np.zeros((1, 4))).validate()
    with pytest.raises(ValueError):
        FeatureStream(imu[::-1], np.array([0.0]), np.array([0, 0]), np.zeros(0, np.int64),
                      np.zeros((0, 4))).validate()


def test_recorder_builds_stream(seq):
    rec = Recorder()
    for kind, m in seq.events():
        (rec.imu_callback if kind == 0 else rec.feature_callback)(m)
    st = rec.stream()
    ref = FeatureStream.from_synthetic(seq)
    np.testing.assert_array_equal(st.feat_z, ref.feat_z)
    np.testing.assert_array_equal(st.imu, ref.imu)


def test_euroc_layout_roundtrip(tmp_path, seq):
    st = FeatureStream.from_synthetic(seq)
    # ground truth rows: t, p, q (w x y z, body -> world), v, bw, ba
    q_jpl = np.array([to_quaternion(R.T) for R in seq.gt_R])          # JPL world->body == Hamilton body->world
    q_wxyz = np.concatenate([q_jpl[:, 3:4], q_jpl[:, :3]], axis=1)
    gt = np.zeros((len(seq.gt_t), 17))
    gt[:, 0], gt[:, 1:4], gt[:, 4:8] = seq.gt_t, seq.gt_p, q_wxyz
    root = write_euroc_layout(str(tmp_path / "MH_synth"), st.imu, gt, st.frame_t)
    ds = EuRoC(root)
    assert ds.starttime == pytest.approx(st.imu[0, 0], abs=1e-9)
    np.testing.assert_allclose(ds.imu[:, 0], st.imu[:, 0], atol=1e-9)
    np.testing.assert_array_equal(ds.imu[:, 1:], st.imu[:, 1:])
    np.testing.assert_allclose(ds.stereo_timestamps(), st.frame_t, atol=1e-9)
    g = ds.groundtruth()
    np.testing.assert_allclose(g.R, seq.gt_R, atol=1e-12)
    np.testing.assert_array_equal(g.p, seq.gt_p)
    ds.set_starttime(1.0)
    msgs = list(ds.imu_msgs())
    assert msgs[0].vio_timestamp__ >= ds.starttime + 1.0 and len(msgs) == np.sum(ds.imu[:, 0] >= ds.t0)
    assert all(m.vio_timestamp__ >= ds.t0 for m in ds.groundtruth_msgs())


def test_euroc_rejects_unsynced_stereo(tmp_path):
    root = write_euroc_layout(str(tmp_path / "x"), np.zeros((2, 7)) + [[0.0] * 7, [1e-3] + [0.0] * 6],
                              None, [0.0, 0.05])
    os.remove(os.path.join(root, "mav0", "cam1", "data", "50000000.png"))
    open(os.path.join(root, "mav0", "cam1", "data", "80000000.png"), "wb").close()
    with pytest.raises(ValueError):
        EuRoC(root)


def test_quat_wxyz_identity():
    np.testing.assert_allclose(quat_wxyz_to_rotation([1, 0, 0, 0]), np.eye(3))
    c = np.cos(np.pi / 4)
    np.testing.assert_allclose(quat_wxyz_to_rotation([c, 0, 0, c]), [[0, -1, 0], [1, 0, 0], [0, 0, 1]], atol=1e-15)


def test_oracle_replay_ate_vs_reference():
    """The deterministic driver feeding the oracle reproduces the reference
    filter's trajectory on golden sequence_s1 (ATE vs ref at rounding level),
    and that trajectory tracks the synthetic ground truth to ~1 cm."""
    from oracle import msckf_oracle as O
    g = golden("sequence_s1")
    seq = synth.make_sequence(int(g["n_frames"]), int(g["seed"]))
    st = FeatureStream.from_synthetic(seq)

    class Adapter:        # oracle callbacks take plain arrays
        def __init__(self):
            self.o = O.OracleMSCKF(FilterConfig(), chi2_threshold)

        def imu_callback(self, m):
            self.o.imu_callback(m.vio_timestamp__, m.angular_velocity, m.linear_acceleration)

        def feature_callback(self, m):
            r = self.o.feature_callback(m.timestamp, [(f.id, f.u0, f.v0, f.u1, f.v1) for f in m.vio_features])
            if r is None:
                return None
            return synth_result(r)

    from msckf_amd.msckf import VioResult
    from msckf_amd.geometry import Isometry3d

    def synth_result(r):
        return VioResult(r["timestamp"], Isometry3d(r["pose"].R, r["pose"].t), r["velocity"],
                         Isometry3d(r["cam0_pose"].R, r["cam0_pose"].t))

    from msckf_amd.replay import replay
    traj = replay(Adapter(), st)
    ref = Trajectory(g["rec"][:, 0], g["rec"][:, 5:8])
    np.testing.assert_array_equal(traj.t, ref.t)
    assert ate(traj, ref, align="none") < 1e-9
    e_gt = ate(traj, st.gt)
    assert e_gt < 0.05, e_gt


def test_stream_messages_are_its_events(seq):
    """messages() (built once before a timed replay) holds the same IMU and
    frame messages as events(), split by kind."""
    st = FeatureStream.from_synthetic(seq)
    imu, frames = st.messages()
    ev = st.events()
    assert len(imu) == sum(1 for k, _ in ev if k == 0) and len(frames) == st.n_frames
    for a, (_, b) in zip(imu, [e for e in ev if e[0] == 0]):
        assert a.vio_timestamp__ == b.vio_timestamp__
        np.testing.assert_array_equal(a.linear_acceleration, b.linear_acceleration)
    for a, (_, b) in zip(frames, [e for e in ev if e[0] == 1]):
        assert a.timestamp == b.timestamp
        assert [(f.id, f.u0, f.v1) for f in a.vio_features] == [(f.id, f.u0, f.v1) for f in b.vio_features]
