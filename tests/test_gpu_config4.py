"""SURVEY config 4 at its size: "all 11 EuRoC sequences batched" (BASELINE.json
configs[3]; reference harness vio.py:23-65, dataset.py:250-271) -- on
synthetic stereo+IMU streams of the EuRoC shape (no EuRoC data exists on
either box).  Eleven sequences run through ONE device context by the
multi-sequence scheduler (fp64); every lane must equal its own
single-filter run through the drop-in class, and the golden lanes
(sequence_s1..s3, written by tools/gen_golden.py from the reference filter)
must still match the reference to the north-star tolerance."""
import numpy as np
import pytest

import msckf_amd
from conftest import golden, rel
from helpers import sequence_config
from msckf_amd import synth
from msckf_amd.replay import FeatureStream, replay
from msckf_amd.scheduler import MultiMSCKF
from msckf_amd.trajectory import Trajectory, ate

pytestmark = pytest.mark.gpu

N_SEQ = 11
GOLDEN = ["sequence_s1", "sequence_s2", "sequence_s3"]
# s4 rides as a plain lane: its reference decisions are rounding noise on
# degenerate features (test_gpu_parity.py::test_sequence_s4_degenerate)
EXTRA = ["sequence_s4"]


def _lanes():
    gs = [golden(n) for n in GOLDEN]
    streams = [FeatureStream.from_synthetic(synth.make_sequence(int(g["n_frames"]), int(g["seed"]))) for g in gs]
    cfgs = [sequence_config(g) for g in gs]
    for name in EXTRA:
        ge = golden(name)
        streams.append(FeatureStream.from_synthetic(synth.make_sequence(int(ge["n_frames"]), int(ge["seed"]))))
        cfgs.append(sequence_config(ge))
    for i in range(N_SEQ - len(streams)):   # the other seven: EuRoC-shaped synthetic streams of varied length
        streams.append(FeatureStream.from_synthetic(synth.make_sequence(120 + 20 * (i % 4), 300 + i)))
        cfgs.append(msckf_amd.FilterConfig())
    return gs, streams, cfgs


def _single(st, cfg):
    flt = msckf_amd.MSCKF(cfg)
    try:
        traj = replay(flt, st)
        return traj, list(flt.gate_log), list(flt.shape_log), list(flt.reset_log), flt.state_cov()
    finally:
        flt.close()


@pytest.mark.timeout(600)
def test_config4_eleven_sequences_one_context():
    gs, streams, cfgs = _lanes()
    assert len(streams) == N_SEQ
    multi = MultiMSCKF(N_SEQ, lane_configs=cfgs)
    try:
        trajs = multi.run_streams(streams)
        lanes = [(list(ln.gate_log), list(ln.shape_log), list(ln.reset_log), ln.state_cov()) for ln in multi.lanes]
        launches = dict(multi.launches)
    finally:
        multi.close()
    for i, (st, cfg) in enumerate(zip(streams, cfgs)):
        t1, gl, sl, rl, P = _single(st, cfg)
        np.testing.assert_array_equal(trajs[i].t, t1.t)
        assert np.array(lanes[i][0]).tolist() == np.array(gl).tolist(), i     # gate log: decisions identical
        assert np.array(lanes[i][1]).tolist() == np.array(sl).tolist(), i     # stacked-H shapes identical
        assert lanes[i][2] == rl, i                                            # online-reset frames
        assert np.abs(trajs[i].p - t1.p).max() <= 1e-9 * max(1.0, np.abs(t1.p).max()), i
        assert rel(lanes[i][3], P) <= 1e-9, i
    for i, g in enumerate(gs):        # golden lanes vs the reference filter's own runs
        np.testing.assert_array_equal(np.array(lanes[i][0]), g["gates"])
        np.testing.assert_array_equal(np.array(lanes[i][1]), g["shapes"])
        np.testing.assert_array_equal(lanes[i][2], g["resets"] if "resets" in g else [])
        assert rel(lanes[i][3], g["P_final"]) < 1e-6, GOLDEN[i]
        ref = Trajectory(g["rec"][:, 0], g["rec"][:, 5:8])
        assert ate(trajs[i], ref, align="none") <= 1e-6 * np.sqrt(np.mean(np.sum(ref.p ** 2, 1))), GOLDEN[i]
    # one batched launch per request kind per lock-step round, not one per lane
    n_rounds = max(s.n_frames for s in streams)
    assert launches["augment"] <= n_rounds and launches["propagate"] <= n_rounds
    for st, tr in zip(streams[len(gs):], trajs[len(gs):]):
        assert ate(tr, st.gt) < 0.1
    print("config 4: %d lanes, %d rounds, launches %s" % (N_SEQ, n_rounds, launches))
