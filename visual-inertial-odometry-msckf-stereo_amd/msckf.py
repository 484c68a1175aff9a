"""Drop-in host class for the reference filter (MSCKF/msckf.py:104-908).

``MSCKF(config)`` keeps the reference's public API -- ``imu_callback(imu_msg)``
and ``feature_callback(feature_msg) -> vio_result | None`` with the same
message tuples -- so it sits behind the existing stereo front-end unchanged.

What stays in Python (host bookkeeping, as SURVEY.md section 8(b) prescribes):
the IMU message buffer walk, the feature map and its observation dicts, cam-id
<-> slot bookkeeping, the chi2 table lookup, the ordered 1500-row cap inputs,
keyframe selection, the online-reset decision and ``publish``.
What runs on the GPU (through the C-ABI, libmsckf_hip.so): IMU covariance
propagation, state augmentation, triangulation, measurement Jacobians +
nullspace projection, gating, stacking, compression of the stacked rows
(information assembly), the Kalman update and covariance compaction.  There is
no CPU fallback.

Every device interaction of a frame is expressed as a request yielded by a
step generator (``_frame_steps``); ``feature_callback`` serves the requests
one by one on this filter's slot, while ``scheduler.MultiMSCKF`` advances many
filters' generators in lock step and serves each kind of request for all of
them with one batched launch.  Both paths run the same host logic.

Differences from the reference that are deliberate:
* the reference's IMU-buffer race between the IMU and vio threads
  (msckf.py:173 vs 287) is removed -- every call holds the context lock;
* class-level globals (gravity, next ids, cam0->cam1 extrinsics; quirk Q7) are
  per-instance, so several filters can live in one process.
"""
from __future__ import annotations

import threading
from collections import OrderedDict, namedtuple

import numpy as np

from . import _lib
from .config import FilterConfig, chi2_threshold
from .geometry import Isometry3d, from_two_vectors, to_quaternion, to_rotation

VioResult = namedtuple("vio_result", ["timestamp", "pose", "velocity", "cam0_pose"])


class Feature:
    """Host record of a map feature (reference Feature fields, feature.py:15-31)."""
    __slots__ = ("id", "observations", "position", "is_initialized")

    def __init__(self, fid):
        self.id = fid
        self.observations: "OrderedDict[int, np.ndarray]" = OrderedDict()
        self.position = np.zeros(3)
        self.is_initialized = False


def check_motion(observations, cams, threshold):
    """Feature.check_motion (feature.py:124-165): is the translation between the
    first and the last observing cam, orthogonal to the first observation's
    ray, above ``threshold``?  ``cams``: cam id -> dict(q, p).  A negative
    threshold (the EuRoC config, config.py:10) accepts every feature."""
    if threshold < 0:
        return True
    ids = list(observations.keys())
    c0, c1 = cams[ids[0]], cams[ids[-1]]
    d = np.array([*observations[ids[0]][:2], 1.0])
    d = to_rotation(np.asarray(c0["q"], float)).T @ (d / np.linalg.norm(d))
    tr = np.asarray(c1["p"], float) - np.asarray(c0["p"], float)
    orth = tr - (tr @ d) * d
    return bool(np.linalg.norm(orth) > threshold)


class MSCKF:
    ROW_CAP = 1500   # msckf.py:678

    def __init__(self, config=None, dtype=np.float64, device=0, cam_capacity=None, ctx=None, slot=0):
        if config is None:
            config = FilterConfig()
        elif not isinstance(config, FilterConfig):
            config = FilterConfig.from_reference(config)
        self.config = config
        cap = cam_capacity or (config.max_cam_state_size + 2)
        self._own_ctx = ctx is None
        self.ctx = ctx if ctx is not None else _lib.Context(config, n_filters=1, n_cam_capacity=cap, dtype=dtype,
                                                            device=device)
        self.slot = slot
        self._lock = threading.RLock()
        self.imu_msg_buffer = []
        self.map_server: "OrderedDict[int, Feature]" = OrderedDict()
        self.cam_ids: list = []            # cam-state ids in slot order (oldest first)
        self.imu_timestamp = None
        self.imu_id = None
        self._next_id = 0
        self.tracking_rate = None
        self.is_gravity_set = False
        self.is_first_img = True
        self.gate_log = []                 # (frame, dof, rows, accepted) like tools/gen_golden.py
        self.gamma_log = []                # (feature id, gamma), one per gate_log entry
        self.shape_log = []
        self.reset_log = []                # frames after which online_reset fired
        self._deferred = []                # (Pending, callback): update results not read back yet
        self._n_published = 0
        T_cam0_imu = np.linalg.inv(config.T_imu_cam0)
        self._T_imu_body = Isometry3d(config.T_imu_body[:3, :3], config.T_imu_body[:3, 3])
        imu = _lib.pack_imu(q=[0, 0, 0, 1], p=np.zeros(3), v=config.velocity, bg=np.zeros(3), ba=np.zeros(3),
                            q_null=[0, 0, 0, 1], p_null=np.zeros(3), v_null=np.zeros(3),
                            R_imu_cam0=T_cam0_imu[:3, :3].T, t_cam0_imu=T_cam0_imu[:3, 3],
                            gravity=config.gravity, alias=False)
        self.ctx.set_state(self.slot, imu, None, self._initial_cov())

    # ------------------------------------------------------------ helpers --
    def _initial_cov(self):
        """msckf.py:820-830"""
        c = self.config
        P = np.zeros((21, 21))
        P[3:6, 3:6] = c.gyro_bias_cov * np.eye(3)
        P[6:9, 6:9] = c.velocity_cov * np.eye(3)
        P[9:12, 9:12] = c.acc_bias_cov * np.eye(3)
        P[15:18, 15:18] = c.extrinsic_rotation_cov * np.eye(3)
        P[18:21, 18:21] = c.extrinsic_translation_cov * np.eye(3)
        return P

    def imu_state(self):
        imu, _, _ = self.ctx.get_state(self.slot, want_P=False)
        return _lib.unpack_imu(imu)

    def cam_states(self):
        """OrderedDict cam id -> dict(q, p, q_null) in slot order."""
        _, cams, _ = self.ctx.get_state(self.slot, want_P=False)
        return self._cam_dict(cams)

    def _cam_dict(self, cams):
        return OrderedDict((cid, dict(q=cams[i, 0:4], p=cams[i, 4:7], q_null=cams[i, 7:11]))
                           for i, cid in enumerate(self.cam_ids))

    def state_cov(self):
        return self.ctx.get_state(self.slot, want_P=True)[2]

    # ------------------------------------------------- device request server --
    def _serve(self, req):
        """Executes one request of the step generators on this filter's slot."""
        kind, f, ctx = req[0], self.slot, self.ctx
        if kind == "propagate":
            return ctx.propagate(f, req[1], req[2], req[3])
        if kind == "augment":
            return ctx.augment(f)
        if kind == "triangulate":
            return ctx.triangulate(f, req[1], req[2], req[3])
        if kind == "update":
            return ctx.update_async(f, *req[1:])
        if kind == "states":   # ("states"[, i0, n]): one read, with P's diagonal [i0, i0 + n) if asked
            imu, cams, cv = ctx.readback([f], cov=req[1:3] if len(req) > 1 else None)
            return (imu[0], cams[0]) if cv is None else (imu[0], cams[0], cv[0])
        if kind == "prune":
            return ctx.prune(f, req[1])
        if kind == "cov_diag":
            return ctx.cov_diag(f, req[1], req[2])
        if kind == "set_state":
            return ctx.set_state(f, req[1], req[2], req[3])
        raise ValueError("unknown request %r" % (kind,))

    def _settle(self):
        """Applies the deferred update results (gate / shape logs, new
        positions) in request order.  Called at the frame's synchronisation
        points -- after a ``states`` read, when the device has drained anyway."""
        d, self._deferred = self._deferred, []
        for pend, fn in d:
            fn(*pend.get())

    def _drive(self, gen):
        try:
            req = next(gen)
            while True:
                req = gen.send(self._serve(req))
        except StopIteration as e:
            return e.value

    # ----------------------------------------------------------- callbacks --
    def imu_callback(self, imu_msg):
        """msckf.py:166-178"""
        with self._lock:
            self.imu_msg_buffer.append(imu_msg)
            if not self.is_gravity_set and len(self.imu_msg_buffer) >= 200:
                self._drive(self._initialize_gravity_and_bias())
                self.is_gravity_set = True

    def _initialize_gravity_and_bias(self):
        """msckf.py:235-258"""
        sw = np.zeros(3)
        sa = np.zeros(3)
        for m in self.imu_msg_buffer:
            sw += m.angular_velocity
            sa += m.linear_acceleration
        bg = sw / len(self.imu_msg_buffer)
        g_imu = sa / len(self.imu_msg_buffer)
        g = np.array([0.0, 0.0, -np.linalg.norm(g_imu)])
        imu, _ = yield ("states",)
        imu = imu.copy()
        imu[_lib.I_BG:_lib.I_BG + 3] = bg
        imu[_lib.I_G:_lib.I_G + 3] = g
        imu[_lib.I_Q:_lib.I_Q + 4] = from_two_vectors(-g, g_imu)
        yield ("set_state", imu, None, self._initial_cov() if not self.cam_ids else None)

    def feature_callback(self, feature_msg):
        """msckf.py:180-233"""
        with self._lock:
            return self._drive(self._frame_steps(feature_msg))

    def _frame_steps(self, feature_msg):
        """The body of feature_callback as a request generator; returns the
        vio_result (or None before gravity initialisation)."""
        if not self.is_gravity_set:
            return None
        if self.is_first_img:
            self.is_first_img = False
            self.imu_timestamp = feature_msg.timestamp
        yield from self._batch_imu_processing(feature_msg.timestamp)
        yield from self._state_augmentation()
        self._add_feature_observations(feature_msg)
        yield from self._remove_lost_features()
        yield from self._prune_cam_state_buffer()
        # publish and online_reset's position variances in one read
        thr = self.config.position_std_threshold
        st = yield (("states", 12, 3) if thr > 0 else ("states",))
        self._settle()
        res = self._publish_from(feature_msg.timestamp, _lib.unpack_imu(st[0]))
        self._n_published += 1
        yield from self._online_reset(st[2] if thr > 0 else None)
        return res

    # ---------------------------------------------------------- propagation --
    def _batch_imu_processing(self, time_bound):
        """msckf.py:262-287: host walks the buffer, the device applies the samples."""
        used = 0
        dts, ws, accs = [], [], []
        t_state = self.imu_timestamp
        for m in self.imu_msg_buffer:
            t = m.vio_timestamp__
            if t < t_state:
                used += 1
                continue
            if t > time_bound:
                break
            dts.append(t - t_state)
            ws.append(m.angular_velocity)
            accs.append(m.linear_acceleration)
            used += 1
            t_state = t
        if dts:
            yield ("propagate", np.array(dts), np.array(ws).reshape(-1, 3), np.array(accs).reshape(-1, 3))
        self.imu_timestamp = t_state
        self.imu_id = self._next_id
        self._next_id += 1
        self.imu_msg_buffer = self.imu_msg_buffer[used:]

    def _state_augmentation(self):
        """msckf.py:385-407"""
        yield ("augment",)
        self.cam_ids.append(self.imu_id)

    def _add_feature_observations(self, feature_msg):
        """msckf.py:409-427"""
        sid = self.imu_id
        ms = self.map_server
        get = ms.get
        cur = len(ms)
        tracked = 0
        for f in feature_msg.vio_features:
            z = (float(f.u0), float(f.v0), float(f.u1), float(f.v1))   # packed into arrays once per request (_pack)
            feat = get(f.id)
            if feat is None:
                feat = Feature(f.id)
                ms[f.id] = feat
            else:
                tracked += 1
            feat.observations[sid] = z
        self.tracking_rate = tracked / (cur + 1e-5)

    # -------------------------------------------------------------- updates --
    def _pack(self, feats, cam_lists):
        slot = {cid: i for i, cid in enumerate(self.cam_ids)}
        off = [0]
        cams, zs = [], []
        for feat, cl in zip(feats, cam_lists):
            obs = feat.observations
            cams.extend([slot[cid] for cid in cl])
            zs.extend([obs[cid] for cid in cl])
            off.append(len(cams))
        return (np.array(off, np.int32), np.array(cams, np.int32),
                np.array(zs, float).reshape(-1, 4))

    def _triangulate(self, feats):
        """Feature.initialize_position (feature.py:167-295) for a batch of
        features, one wavefront each on the device."""
        if not feats:
            return
        off, cams, zs = self._pack(feats, [list(f.observations.keys()) for f in feats])
        p, ok = yield ("triangulate", off, cams, zs)
        for f, pi, oki in zip(feats, p, ok):
            f.position = pi
            f.is_initialized = bool(oki)

    def _update(self, feats, cam_lists, dofs, row_cap, to_init=()):
        """Stacked update over ``feats`` in order (device: jacobian, gating,
        stacking with the row cap, QR, Kalman), enqueued without a wait.
        Features in ``to_init`` are triangulated in the same device chain from
        the observations passed (their p_w rows go down as NaN); those whose
        triangulation fails take no part, exactly as if the host had dropped
        them (msckf.py:640-652).  The decision log and the new positions are
        applied at the next synchronisation point (``_settle``)."""
        if not feats:
            return
        off, cams, zs = self._pack(feats, cam_lists)
        chi2 = np.array([chi2_threshold(d) for d in dofs])
        init = set(id(f) for f in to_init)
        pw = np.array([np.full(3, np.nan) if id(f) in init else f.position for f in feats])
        pend = yield ("update", off, cams, zs, pw, chi2, row_cap)
        frame, D = self._n_published, 21 + 6 * len(self.cam_ids)

        def apply(acc, gam, p, valid, rows):
            # reproduce the reference's decision log: features after the row-cap
            # break are never gated (msckf.py:678-679); failed triangulations
            # never reach measurement_update
            for i, f in enumerate(feats):
                if id(f) in init:
                    f.is_initialized = bool(valid[i])
                    f.position = p[i]
            count = 0
            for i, f in enumerate(feats):
                if not valid[i]:
                    continue
                k = 4 * len(cam_lists[i]) - 3
                ok = bool(gam[i] < chi2[i])
                self.gate_log.append((frame, dofs[i], k, int(ok)))
                self.gamma_log.append((f.id, float(gam[i])))
                if ok:
                    count += k
                if row_cap and count > row_cap:
                    break
            # no processed feature (every triangulation failed): the reference
            # returns before measurement_update and logs no shape (msckf.py:652-654)
            if np.any(valid):
                self.shape_log.append((frame, rows, D))
        self._deferred.append((pend, apply))

    def _remove_lost_features(self):
        """msckf.py:616-689"""
        sid = self.imu_id
        invalid, candidates = [], []
        for feat in self.map_server.values():
            if sid in feat.observations:
                continue
            if len(feat.observations) < 3:
                invalid.append(feat.id)
                continue
            candidates.append(feat)
        # check_motion (always True with the EuRoC config's threshold -1,
        # config.py:10) needs the cam poses; the triangulations are independent
        # of each other, so they are batched into one launch.
        # The triangulations of the new features ride in the update's device
        # chain (their observations are the update's own): no wait here.
        thr = self.config.optimization.translation_threshold
        lost = candidates
        to_init = [f for f in candidates if not f.is_initialized]
        if thr >= 0 and to_init:
            _, cams_arr = yield ("states",)
            self._settle()
            cams = self._cam_dict(cams_arr)
            moved = set(id(f) for f in to_init if check_motion(f.observations, cams, thr))
            to_init = [f for f in to_init if id(f) in moved]
            candidates = [f for f in candidates if f.is_initialized or id(f) in moved]
        for fid in invalid:
            del self.map_server[fid]
        for feat in lost:   # gone from the map whether or not it initialises
            del self.map_server[feat.id]
        if not candidates:
            return
        cam_lists = [list(f.observations.keys()) for f in candidates]
        dofs = [len(cl) - 1 for cl in cam_lists]
        yield from self._update(candidates, cam_lists, dofs, self.ROW_CAP, to_init)

    def _find_redundant_cam_states(self, cams_arr):
        """msckf.py:691-727 (host; needs the cam poses)."""
        cams = list(self._cam_dict(cams_arr).items())
        key = len(cams) - 4
        ci = key + 1
        first = 0
        kp = cams[key][1]["p"]
        kR = to_rotation(cams[key][1]["q"])
        rm = []
        for _ in range(2):
            pos = cams[ci][1]["p"]
            Rc = to_rotation(cams[ci][1]["q"])
            dist = np.linalg.norm(pos - kp)
            ang = 2 * np.arccos(to_quaternion(Rc @ kR.T)[-1])
            if ang < 0.2618 and dist < 0.4 and self.tracking_rate > 0.5:
                rm.append(cams[ci][0])
                ci += 1
            else:
                rm.append(cams[first][0])
                first += 1
                ci += 1
        return sorted(rm)

    def _prune_cam_state_buffer(self):
        """msckf.py:730-818"""
        if len(self.cam_ids) < self.config.max_cam_state_size:
            return
        _, cams_arr = yield ("states",)
        self._settle()
        rm = self._find_redundant_cam_states(cams_arr)
        thr = self.config.optimization.translation_threshold
        cams = self._cam_dict(cams_arr)
        to_init, involved = [], []   # (feature, its observations of removed cams), map order
        for feat in self.map_server.values():
            obs = feat.observations
            inv = [c for c in rm if c in obs]
            if not inv:
                continue
            if len(inv) == 1:
                del obs[inv[0]]
                continue
            involved.append((feat, inv))
            if not feat.is_initialized:
                to_init.append(feat)
        # features that fail check_motion stay uninitialized: their involved
        # observations are dropped below like those of a failed triangulation
        yield from self._triangulate([f for f in to_init if check_motion(f.observations, cams, thr)])
        feats, cam_lists = [], []
        for feat, inv in involved:
            if feat.is_initialized:
                feats.append(feat)
                cam_lists.append(inv)
            else:
                for c in inv:
                    del feat.observations[c]
        if feats:
            yield from self._update(feats, cam_lists, [len(cl) for cl in cam_lists], 0)
        else:   # the reference still calls measurement_update with an empty H
            self.shape_log.append((self._n_published, 0, 21 + 6 * len(self.cam_ids)))
        for feat, cl in zip(feats, cam_lists):
            for c in cl:
                del feat.observations[c]
        slots = [self.cam_ids.index(c) for c in rm]
        yield ("prune", np.array(slots, np.int32))
        for c in rm:
            self.cam_ids.remove(c)

    # ------------------------------------------------------ output / reset --
    def publish(self, time):
        """msckf.py:888-908"""
        return self._publish_from(time, self.imu_state())

    def _publish_from(self, time, s):
        T_i_w = Isometry3d(to_rotation(s["q"]).T, s["p"])
        Tb = self._T_imu_body
        T_b_w = Tb * T_i_w * Tb.inverse()
        body_velocity = Tb._vio_R__ @ s["v"]
        R_w_c = s["R_imu_cam0"] @ T_i_w._vio_R__.T
        t_c_w = s["p"] + T_i_w._vio_R__ @ s["t_cam0_imu"]
        return VioResult(time, T_b_w, body_velocity, Isometry3d(R_w_c.T, t_c_w))

    def _online_reset(self, d):
        """msckf.py:859-886 (``d``: P's position-block diagonal, read with the
        publish state)"""
        thr = self.config.position_std_threshold
        if thr <= 0:
            return
        if np.max(np.sqrt(d)) < thr:
            return
        self.cam_ids.clear()
        self.map_server.clear()
        self.reset_log.append(self._n_published - 1)   # the frame just published
        imu, _ = yield ("states",)
        yield ("set_state", imu, None, self._initial_cov())

    def close(self):
        if self._own_ctx:
            self.ctx.close()
