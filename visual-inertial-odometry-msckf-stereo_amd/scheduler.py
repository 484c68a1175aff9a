"""Batched multi-sequence scheduler.

Many independent filters -- one per sequence -- share one device context
(one filter slot each, P of all of them resident in HBM side by side).  Each
filter keeps its own host bookkeeping (an ``MSCKF`` lane: feature map, cam ids,
IMU buffer), and its frame is the same request generator the single-filter
``feature_callback`` drives.  The scheduler advances all lanes that have a
frame in lock step and serves every kind of request for all waiting lanes
with ONE batched launch:

  propagate   -> msckf_propagate_batch   (IMU propagation fused across filters)
  augment     -> msckf_augment_batch
  triangulate -> msckf_batch_load + msckf_batch_triangulate
  update      -> msckf_batch_load + msckf_batch_update (per row cap), results
                 read back at the lanes' next sync point (one read per batch)
  states      -> msckf_readback          (publish + online_reset's diagonal,
                 keyframe selection; the deferred update results ride along)
  prune       -> msckf_prune_batch
  cov_diag    -> msckf_get_cov_diag_batch (online reset)

Lanes whose frames diverge (one triangulates, another is already at its
update) wait at the earliest pipeline stage first, so requests of the same
kind merge again.  Results are identical to running each filter alone: the
batched kernels compute every filter independently.
"""
from __future__ import annotations

from collections import defaultdict

import numpy as np

from . import _lib
from .config import FilterConfig
from .msckf import MSCKF
from .trajectory import Trajectory

# pipeline order: a lane waiting at an earlier stage is served first
_ORDER = {"set_state": 0, "propagate": 1, "augment": 2, "triangulate": 3, "update": 4, "states": 5,
          "prune": 6, "cov_diag": 7}


class MultiMSCKF:
    """``n`` filters (one per sequence) on one device context."""

    def __init__(self, n, config=None, dtype=np.float64, device=0, cam_capacity=None, lane_configs=None):
        """``lane_configs`` (optional, one per lane): per-sequence host-side
        settings (check_motion's translation threshold, online_reset's
        position std threshold, window size).  The device context is shared,
        so every lane must agree on what the device computes with (noise,
        extrinsics, LM parameters: the C-ABI msckf_config_t)."""
        config = config or FilterConfig()
        if not isinstance(config, FilterConfig):
            config = FilterConfig.from_reference(config)
        cfgs = [config] * n if lane_configs is None else [
            c if isinstance(c, FilterConfig) else FilterConfig.from_reference(c) for c in lane_configs]
        if len(cfgs) != n:
            raise ValueError("%d lane configs for %d lanes" % (len(cfgs), n))
        dev0 = bytes(_lib.make_config(cfgs[0]))
        for i, c in enumerate(cfgs):
            if bytes(_lib.make_config(c)) != dev0:
                raise ValueError("lane %d: device-side filter parameters differ from lane 0's" % i)
        cap = cam_capacity or max(c.max_cam_state_size for c in cfgs) + 2
        self.config = cfgs[0]
        self.ctx = _lib.Context(cfgs[0], n_filters=n, n_cam_capacity=cap, dtype=dtype, device=device)
        self.lanes = [MSCKF(cfgs[i], ctx=self.ctx, slot=i) for i in range(n)]
        self.launches = defaultdict(int)       # batched device calls per request kind

    def __len__(self):
        return len(self.lanes)

    def close(self):
        self.ctx.close()

    # ------------------------------------------------------------ callbacks --
    def imu_callback(self, i, imu_msg):
        self.lanes[i].imu_callback(imu_msg)

    def feature_callbacks(self, msgs):
        """``msgs``: {lane index: feature_msg}.  Returns {lane index:
        vio_result | None}, as the lanes' own feature_callback would."""
        gens, pending, out = {}, {}, {}
        for i, m in msgs.items():
            g = self.lanes[i]._frame_steps(m)
            gens[i] = g
            self._advance(i, g, None, pending, out, first=True)
        while pending:
            kind = min((r[0] for r in pending.values()), key=lambda k: _ORDER[k])
            group = [i for i, r in pending.items() if r[0] == kind]
            if kind == "update":          # the row cap is per call: lost path 1500, prune path none
                cap = min(pending[i][6] for i in group)
                group = [i for i in group if pending[i][6] == cap]
            elif kind in ("cov_diag", "states"):
                key = pending[group[0]][1:3]
                group = [i for i in group if pending[i][1:3] == key]
            results = self._serve(kind, group, [pending[i] for i in group])
            for i, res in zip(group, results):
                del pending[i]
                self._advance(i, gens[i], res, pending, out)
        return out

    def _advance(self, i, gen, value, pending, out, first=False):
        try:
            req = next(gen) if first else gen.send(value)
            pending[i] = req
        except StopIteration as e:
            out[i] = e.value

    # --------------------------------------------------------- batched calls --
    def _serve(self, kind, group, reqs):
        ctx = self.ctx
        slots = [self.lanes[i].slot for i in group]
        self.launches[kind] += 1
        if kind == "propagate":
            off = np.concatenate([[0], np.cumsum([len(r[1]) for r in reqs])]).astype(np.int32)
            ctx.propagate_batch(slots, off, np.concatenate([r[1] for r in reqs]),
                                np.concatenate([r[2] for r in reqs]), np.concatenate([r[3] for r in reqs]))
            return [None] * len(group)
        if kind == "augment":
            ctx.augment_batch(slots)
            return [None] * len(group)
        if kind == "triangulate":
            self._load(slots, reqs, with_pw=False)
            ctx.batch_triangulate()
            _, _, p, v, _ = ctx.batch_results()
            return self._split(slots, reqs, lambda a, b, _s: (p[a:b].copy(), v[a:b].copy()))
        if kind == "update":   # deferred: each lane reads its share at its next sync point
            self._load(slots, reqs, with_pw=True)
            tri = any(not np.isfinite(np.asarray(r[4], float)).all() for r in reqs)
            ctx.batch_update(row_cap=reqs[0][6], triangulate=tri)
            return ctx.pending([(s,) + self._ranges[s] for s in slots])
        if kind == "states":   # one read for the group (with the deferred batch, if any)
            cov = reqs[0][1:3] if len(reqs[0]) > 1 else None
            imu, cams, cv = ctx.readback(slots, cov=cov)
            if cv is None:
                return [(imu[w], cams[w]) for w in range(len(group))]
            return [(imu[w], cams[w], cv[w]) for w in range(len(group))]
        if kind == "prune":
            off = np.concatenate([[0], np.cumsum([len(r[1]) for r in reqs])]).astype(np.int32)
            ctx.prune_batch(slots, off, np.concatenate([r[1] for r in reqs]))
            return [None] * len(group)
        if kind == "cov_diag":
            d = ctx.cov_diag_batch(slots, reqs[0][1], reqs[0][2])
            return [d[w] for w in range(len(group))]
        if kind == "set_state":
            for s, r in zip(slots, reqs):
                ctx.set_state(s, r[1], r[2], r[3])
            return [None] * len(group)
        raise ValueError("unknown request %r" % (kind,))

    def _load(self, slots, reqs, with_pw):
        """Concatenates the lanes' feature lists into one batch over all
        filter slots (slots without a request get no features)."""
        B = self.ctx.B
        by_slot = dict(zip(slots, reqs))
        feat_off, obs_off, cams, zs, pws, chis = [0], [0], [], [], [], []
        self._ranges = {}
        for s in range(B):
            r = by_slot.get(s)
            if r is not None:
                off, oc, oz = r[1], r[2], r[3]
                nf = len(off) - 1
                self._ranges[s] = (feat_off[-1], feat_off[-1] + nf)
                obs_off.extend(list(obs_off[-1] + np.asarray(off[1:], np.int64)))
                cams.append(np.asarray(oc, np.int32))
                zs.append(np.asarray(oz, float).reshape(-1, 4))
                if with_pw:
                    pws.append(np.asarray(r[4], float).reshape(-1, 3))
                    chis.append(np.asarray(r[5], float))
                feat_off.append(feat_off[-1] + nf)
            else:
                feat_off.append(feat_off[-1])
        cat = lambda xs, shape: np.concatenate(xs) if xs else np.zeros(shape)  # noqa: E731
        self.ctx.batch_load(np.array(feat_off), np.array(obs_off), cat(cams, (0,)).astype(np.int32),
                            cat(zs, (0, 4)), cat(pws, (0, 3)) if with_pw else None,
                            cat(chis, (0,)) if with_pw else None)

    def _split(self, slots, reqs, take):
        out = []
        for s in slots:
            a, b = self._ranges[s]
            out.append(take(a, b, s))
        return out

    # -------------------------------------------------------------- streams --
    def run_streams(self, streams, on_frame=None, messages=None):
        """Replays ``streams`` (replay.FeatureStream, one per lane) in lock
        step -- frame k of every stream in one batched round, each lane fed
        its own IMU samples up to its frame stamp first (IMU first on ties,
        as replay.FeatureStream.events) -- and returns one Trajectory per lane.
        ``messages``: the streams' ``messages()`` built by the caller
        beforehand (the front-end's output; a timed run leaves them out)."""
        if len(streams) > len(self.lanes):
            raise ValueError("%d streams for %d filter slots" % (len(streams), len(self.lanes)))
        if messages is not None and len(messages) != len(streams):
            raise ValueError("%d message sets for %d streams" % (len(messages), len(streams)))
        imu_pos = [0] * len(streams)
        results = [[] for _ in streams]
        n_rounds = max(s.n_frames for s in streams) if streams else 0
        for k in range(n_rounds):
            msgs = {}
            for i, st in enumerate(streams):
                if k >= st.n_frames:
                    continue
                t = st.frame_t[k]
                j = int(np.searchsorted(st.imu[:, 0], t, side="right"))
                if messages is None:
                    for r in st.imu[imu_pos[i]:j]:
                        self.imu_callback(i, _imu_msg(r))
                    msgs[i] = st.frame_msg(k)
                else:
                    for m in messages[i][0][imu_pos[i]:j]:
                        self.imu_callback(i, m)
                    msgs[i] = messages[i][1][k]
                imu_pos[i] = j
            out = self.feature_callbacks(msgs)
            for i, res in out.items():
                if res is not None:
                    results[i].append(res)
            if on_frame is not None:
                on_frame(k, out)
        for i, st in enumerate(streams):        # trailing IMU samples
            if messages is None:
                for r in st.imu[imu_pos[i]:]:
                    self.imu_callback(i, _imu_msg(r))
            else:
                for m in messages[i][0][imu_pos[i]:]:
                    self.imu_callback(i, m)
        return [Trajectory.from_results(r) for r in results]


def _imu_msg(r):
    from .synth import ImuMsg
    return ImuMsg(r[0], r[1:4].copy(), r[4:7].copy())
