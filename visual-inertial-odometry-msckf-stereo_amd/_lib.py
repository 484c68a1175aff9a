"""ctypes binding of libmsckf_hip.so (C-ABI in include/msckf_hip.h).

Fails loudly: if the shared library is missing, or no HIP device is usable,
constructing a context raises -- there is no CPU fallback anywhere in the
product path.
"""
from __future__ import annotations

import ctypes as C
import os
import threading

import numpy as np

from .config import FilterConfig

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(_HERE, "libmsckf_hip.so")

IMU_LEN = 42
CAM_LEN = 11
TRIANGULATE = 1

# IMU record field offsets (msckf_hip.h)
I_Q, I_P, I_V, I_BG, I_BA, I_QN, I_PN, I_VN, I_RIC, I_TCI, I_G, I_ALIAS = 0, 4, 7, 10, 13, 16, 20, 23, 26, 35, 38, 41


class MsckfConfigT(C.Structure):
    _fields_ = [
        ("gyro_noise", C.c_double), ("acc_noise", C.c_double),
        ("gyro_bias_noise", C.c_double), ("acc_bias_noise", C.c_double),
        ("observation_noise", C.c_double),
        ("R_cam0_cam1", C.c_double * 9), ("t_cam0_cam1", C.c_double * 3),
        ("huber_epsilon", C.c_double), ("estimation_precision", C.c_double),
        ("initial_damping", C.c_double),
        ("outer_loop_max_iteration", C.c_int32), ("inner_loop_max_iteration", C.c_int32),
    ]


class MsckfError(RuntimeError):
    pass


_lib = None
_lib_lock = threading.Lock()

_P = C.c_void_p
_D = C.POINTER(C.c_double)
_I = C.POINTER(C.c_int32)
_U8 = C.POINTER(C.c_uint8)

_SIGS = {
    "msckf_create": (C.c_int, [C.POINTER(MsckfConfigT), C.c_int, C.c_int, C.c_int, C.c_int, C.POINTER(_P)]),
    "msckf_destroy": (C.c_int, [_P]),
    "msckf_last_error": (C.c_char_p, []),
    "msckf_scalar_bytes": (C.c_int, [_P]),
    "msckf_device_info": (C.c_int, [_P, _I, C.c_char_p, C.c_int]),
    "msckf_set_state": (C.c_int, [_P, C.c_int, _D, C.c_int, _D, _D]),
    "msckf_get_state": (C.c_int, [_P, C.c_int, _D, _D, _D, _I]),
    "msckf_get_cov_diag": (C.c_int, [_P, C.c_int, C.c_int, C.c_int, _D]),
    "msckf_propagate": (C.c_int, [_P, C.c_int, C.c_int, _D, _D, _D]),
    "msckf_augment": (C.c_int, [_P, C.c_int]),
    "msckf_triangulate": (C.c_int, [_P, C.c_int, C.c_int, _I, _I, _D, _D, _U8]),
    "msckf_update": (C.c_int, [_P, C.c_int, C.c_int, _I, _I, _D, _D, _D, C.c_int, _U8, _D, _I]),
    "msckf_prune": (C.c_int, [_P, C.c_int, C.c_int, _I]),
    "msckf_propagate_batch": (C.c_int, [_P, C.c_int, _I, _I, _D, _D, _D]),
    "msckf_augment_batch": (C.c_int, [_P, C.c_int, _I]),
    "msckf_prune_batch": (C.c_int, [_P, C.c_int, _I, _I, _I]),
    "msckf_get_states_batch": (C.c_int, [_P, C.c_int, _I, _D, _D, _I]),
    "msckf_get_cov_diag_batch": (C.c_int, [_P, C.c_int, _I, C.c_int, C.c_int, _D]),
    "msckf_readback": (C.c_int, [_P, C.c_int, _I, _D, _D, _I, C.c_int, C.c_int, _D, _U8, _D, _D, _U8, _I]),
    "msckf_batch_triangulate": (C.c_int, [_P]),
    "msckf_batch_load": (C.c_int, [_P, _I, _I, _I, _D, _D, _D]),
    "msckf_batch_update": (C.c_int, [_P, C.c_int, C.c_int]),
    "msckf_batch_results": (C.c_int, [_P, _U8, _D, _D, _U8, _I]),
    "msckf_snapshot": (C.c_int, [_P]),
    "msckf_restore": (C.c_int, [_P]),
    "msckf_sync": (C.c_int, [_P]),
    "msckf_set_profiling": (C.c_int, [_P, C.c_int]),
    "msckf_set_profiling_stage": (C.c_int, [_P, C.c_char_p]),
    "msckf_kernel_times": (C.c_int, [_P, C.c_int, _D, _I, C.c_char_p, C.c_int]),
}

EXPORTED = tuple(_SIGS)

_F = C.POINTER(C.c_float)
# GPU stereo front-end (include/msckf_frontend.h), same library
FRONTEND_SIGS = {
    "mfe_create": (C.c_int, [C.c_int, C.c_int, C.c_int, C.c_int, C.c_int, C.c_int, C.POINTER(_P)]),
    "mfe_destroy": (C.c_int, [_P]),
    "mfe_last_error": (C.c_char_p, []),
    "mfe_upload": (C.c_int, [_P, C.c_int, _U8]),
    "mfe_fast": (C.c_int, [_P, C.c_int, C.c_int, _U8, C.c_int, _F, _F, _I]),
    "mfe_lk": (C.c_int, [_P, C.c_int, C.c_int, C.c_int, _F, _F, _U8, C.c_int, C.c_int, C.c_int, C.c_double]),
    "mfe_undistort": (C.c_int, [_P, C.c_int, _D, _D, _D, C.c_int, _D, _D, _D]),
    "mfe_distort": (C.c_int, [_P, C.c_int, _D, _D, _D, C.c_int, _D]),
}
FRONTEND_EXPORTED = tuple(FRONTEND_SIGS)

# multi-GPU replica transport, RCCL (include/msckf_replicas.h), same library
REPLICA_SIGS = {
    "msckf_rccl_unique_id": (C.c_int, [_U8]),
    "msckf_rccl_init": (C.c_int, [_U8, C.c_int, C.c_int, C.c_int, C.c_double, C.POINTER(_P)]),
    "msckf_rccl_allreduce": (C.c_int, [_P, _D, C.c_int, C.c_int]),
    "msckf_rccl_allgather": (C.c_int, [_P, C.c_void_p, C.c_int, C.c_void_p]),
    "msckf_rccl_set_timeout": (C.c_int, [_P, C.c_double]),
    "msckf_rccl_count": (C.c_int, [_P, _I, _I]),
    "msckf_rccl_destroy": (C.c_int, [_P]),
    "msckf_rccl_last_error": (C.c_char_p, []),
}
REPLICA_EXPORTED = tuple(REPLICA_SIGS)
RCCL_ID_BYTES = 128


def load_library(path: str = LIB_PATH):
    """Load and type the shared library (no device work)."""
    global _lib
    with _lib_lock:
        if _lib is not None:
            return _lib
        if not os.path.exists(path):
            raise MsckfError("HIP extension %s is missing -- build it with `make` "
                             "(or __graft_entry__.build()); there is no CPU fallback" % path)
        lib = C.CDLL(path)
        for name, (res, args) in list(_SIGS.items()) + list(FRONTEND_SIGS.items()) + list(REPLICA_SIGS.items()):
            fn = getattr(lib, name)
            fn.restype = res
            fn.argtypes = args
        _lib = lib
        return lib


def _ptr(a, t):
    return a.ctypes.data_as(C.POINTER(t)) if a is not None else None


def _f64(a, shape=None):
    a = np.ascontiguousarray(a, dtype=np.float64)
    if shape is not None:
        a = a.reshape(shape)
    return a


def _i32(a):
    return np.ascontiguousarray(a, dtype=np.int32)


def make_config(cfg: FilterConfig) -> MsckfConfigT:
    c = MsckfConfigT()
    c.gyro_noise, c.acc_noise = cfg.gyro_noise, cfg.acc_noise
    c.gyro_bias_noise, c.acc_bias_noise = cfg.gyro_bias_noise, cfg.acc_bias_noise
    c.observation_noise = cfg.observation_noise
    R01 = np.asarray(cfg.T_cn_cnm1, float)[:3, :3].ravel()
    t01 = np.asarray(cfg.T_cn_cnm1, float)[:3, 3]
    for i in range(9):
        c.R_cam0_cam1[i] = R01[i]
    for i in range(3):
        c.t_cam0_cam1[i] = t01[i]
    oc = cfg.optimization
    c.huber_epsilon, c.estimation_precision = oc.huber_epsilon, oc.estimation_precision
    c.initial_damping = oc.initial_damping
    c.outer_loop_max_iteration = oc.outer_loop_max_iteration
    c.inner_loop_max_iteration = oc.inner_loop_max_iteration
    return c


class Context:
    """One device context = ``n_filters`` independent filter slots of one
    scalar type on one HIP device.  Methods mirror the C-ABI one to one."""

    def __init__(self, cfg: FilterConfig, n_filters=1, n_cam_capacity=32, dtype=np.float64, device=0):
        self.lib = load_library()
        self.cfg = cfg
        self.dtype = np.dtype(dtype)
        self.B = n_filters
        self.Nmax = n_cam_capacity
        self._ccfg = make_config(cfg)
        h = _P()
        self._check(self.lib.msckf_create(C.byref(self._ccfg), device, self.dtype.itemsize,
                                          n_filters, n_cam_capacity, C.byref(h)))
        self.h = h
        self.lock = threading.RLock()
        self._pending = None   # the loaded batch's results, not read back yet (Pending)

    def _check(self, rc):
        if rc < 0:
            raise MsckfError("msckf: %s (rc=%d)" % (self.lib.msckf_last_error().decode(), rc))
        return rc

    def close(self):
        if getattr(self, "h", None):
            self.lib.msckf_destroy(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    # ---- state ----
    def set_state(self, f, imu, cams, P):
        imu = _f64(imu)
        n = 0 if cams is None else len(cams)
        cams_a = _f64(cams).reshape(n, CAM_LEN) if n else None
        P_a = _f64(P) if P is not None else None
        with self.lock:
            self._check(self.lib.msckf_set_state(self.h, f, _ptr(imu, C.c_double), n,
                                                 _ptr(cams_a, C.c_double), _ptr(P_a, C.c_double)))

    def get_state(self, f, want_P=True):
        imu = np.zeros(IMU_LEN)
        cams = np.zeros((self.Nmax, CAM_LEN))
        n = C.c_int32(0)
        with self.lock:
            self._check(self.lib.msckf_get_state(self.h, f, _ptr(imu, C.c_double), None, None, C.byref(n)))
            D = 21 + 6 * n.value
            P = np.zeros((D, D)) if want_P else None
            self._check(self.lib.msckf_get_state(self.h, f, _ptr(imu, C.c_double), _ptr(cams, C.c_double),
                                                 _ptr(P, C.c_double), C.byref(n)))
        return imu, cams[:n.value].copy(), P

    def cov_diag(self, f, i0, n):
        out = np.zeros(n)
        with self.lock:
            self._check(self.lib.msckf_get_cov_diag(self.h, f, i0, n, _ptr(out, C.c_double)))
        return out

    # ---- hot path ----
    def propagate(self, f, dt, gyro, acc):
        dt = _f64(dt)
        n = len(dt)
        if n == 0:
            return
        gyro = _f64(gyro, (n, 3))
        acc = _f64(acc, (n, 3))
        with self.lock:
            self._check(self.lib.msckf_propagate(self.h, f, n, _ptr(dt, C.c_double), _ptr(gyro, C.c_double),
                                                 _ptr(acc, C.c_double)))

    def augment(self, f):
        with self.lock:
            self._check(self.lib.msckf_augment(self.h, f))

    def triangulate(self, f, obs_off, obs_cam, obs_z):
        self.settle()
        obs_off, obs_cam = _i32(obs_off), _i32(obs_cam)
        nf = len(obs_off) - 1
        obs_z = _f64(obs_z, (len(obs_cam), 4))
        p = np.zeros((nf, 3))
        v = np.zeros(nf, np.uint8)
        with self.lock:
            self._check(self.lib.msckf_triangulate(self.h, f, nf, _ptr(obs_off, C.c_int32), _ptr(obs_cam, C.c_int32),
                                                   _ptr(obs_z, C.c_double), _ptr(p, C.c_double),
                                                   _ptr(v, C.c_uint8)))
        return p, v.astype(bool)

    def update(self, f, obs_off, obs_cam, obs_z, p_w, chi2, row_cap=0):
        self.settle()
        obs_off, obs_cam = _i32(obs_off), _i32(obs_cam)
        nf = len(obs_off) - 1
        obs_z = _f64(obs_z, (len(obs_cam), 4))
        p_w = _f64(p_w, (nf, 3))
        chi2 = _f64(chi2)
        acc = np.zeros(nf, np.uint8)
        gam = np.zeros(nf)
        rows = C.c_int32(0)
        with self.lock:
            self._check(self.lib.msckf_update(self.h, f, nf, _ptr(obs_off, C.c_int32), _ptr(obs_cam, C.c_int32),
                                              _ptr(obs_z, C.c_double), _ptr(p_w, C.c_double),
                                              _ptr(chi2, C.c_double), int(row_cap), _ptr(acc, C.c_uint8),
                                              _ptr(gam, C.c_double), C.byref(rows)))
        return acc.astype(bool), gam, rows.value

    def update_async(self, f, obs_off, obs_cam, obs_z, p_w, chi2, row_cap=0):
        """msckf_update without the wait: the batch of filter ``f`` is loaded
        and its chain (triangulation of the NaN rows of ``p_w`` fused in front,
        msckf_hip.h) enqueued; the returned Pending reads (accepted, gamma,
        p_w, valid, rows) on first use -- or when the next batch is loaded."""
        nf = len(obs_off) - 1
        feat_off = np.where(np.arange(self.B + 1) <= f, 0, nf).astype(np.int32)
        p_w = _f64(p_w, (nf, 3))
        self.batch_load(feat_off, obs_off, obs_cam, obs_z, p_w, chi2)
        self.batch_update(row_cap=row_cap, triangulate=not bool(np.isfinite(p_w).all()))
        return self.pending([(f, 0, nf)])[0]

    def pending(self, ranges):
        """Deferred results of the loaded batch, one view per (slot, first,
        end) feature range; the batch is read back once, for all of them."""
        self.settle()
        grp = _PendingBatch(self)
        self._pending = grp
        return [Pending(grp, s, a, b) for s, a, b in ranges]

    def settle(self):
        """Reads back the outstanding deferred batch (before its arena is
        reused by the next load)."""
        p, self._pending = self._pending, None
        if p is not None:
            p.read()

    def prune(self, f, slots):
        slots = _i32(slots)
        with self.lock:
            self._check(self.lib.msckf_prune(self.h, f, len(slots), _ptr(slots, C.c_int32)))

    # ---- multi-filter forms (one launch for a list of filter slots) ----
    def propagate_batch(self, filters, sample_off, dt, gyro, acc):
        filters, sample_off = _i32(filters), _i32(sample_off)
        n = int(sample_off[-1]) if len(sample_off) else 0
        dt = _f64(dt).reshape(n)
        gyro = _f64(gyro, (n, 3))
        acc = _f64(acc, (n, 3))
        with self.lock:
            self._check(self.lib.msckf_propagate_batch(self.h, len(filters), _ptr(filters, C.c_int32),
                                                       _ptr(sample_off, C.c_int32), _ptr(dt, C.c_double),
                                                       _ptr(gyro, C.c_double), _ptr(acc, C.c_double)))

    def augment_batch(self, filters):
        filters = _i32(filters)
        with self.lock:
            self._check(self.lib.msckf_augment_batch(self.h, len(filters), _ptr(filters, C.c_int32)))

    def prune_batch(self, filters, slot_off, slots):
        filters, slot_off, slots = _i32(filters), _i32(slot_off), _i32(slots)
        with self.lock:
            self._check(self.lib.msckf_prune_batch(self.h, len(filters), _ptr(filters, C.c_int32),
                                                   _ptr(slot_off, C.c_int32), _ptr(slots, C.c_int32)))

    def get_states_batch(self, filters, want_cams=True):
        """(imu records (n, IMU_LEN), list of cam arrays (n_cams_w, CAM_LEN))."""
        filters = _i32(filters)
        n = len(filters)
        imu = np.zeros((n, IMU_LEN))
        cams = np.zeros((n, self.Nmax, CAM_LEN)) if want_cams else None
        nc = np.zeros(n, np.int32)
        with self.lock:
            self._check(self.lib.msckf_get_states_batch(self.h, n, _ptr(filters, C.c_int32), _ptr(imu, C.c_double),
                                                        _ptr(cams, C.c_double), _ptr(nc, C.c_int32)))
        cl = [cams[w, :nc[w]].copy() for w in range(n)] if want_cams else [None] * n
        return imu, cl

    def cov_diag_batch(self, filters, i0, n):
        filters = _i32(filters)
        out = np.zeros((len(filters), n))
        with self.lock:
            self._check(self.lib.msckf_get_cov_diag_batch(self.h, len(filters), _ptr(filters, C.c_int32), i0, n,
                                                           _ptr(out, C.c_double)))
        return out

    def readback(self, filters, want_cams=True, cov=None):
        """A frame's sync point with ONE stream synchronisation (msckf_readback):
        (imu records (n, IMU_LEN), list of cam arrays, covariance diagonals
        (n, cov[1]) of [cov[0], cov[0] + cov[1]) or None).  An outstanding
        deferred batch (Pending) is read back in the same copy."""
        filters = _i32(filters)
        n = len(filters)
        imu = np.zeros((n, IMU_LEN))
        cams = np.zeros((n, self.Nmax, CAM_LEN)) if want_cams else None
        nc = np.zeros(n, np.int32)
        i0, ncv = cov if cov else (0, 0)
        cv = np.zeros((n, ncv)) if ncv else None
        pend = self._pending if self._pending is not None and self._pending.res is None else None
        if pend is not None:
            nf = self._nf
            acc, gam, p, v = np.zeros(nf, np.uint8), np.zeros(nf), np.zeros((nf, 3)), np.zeros(nf, np.uint8)
            rows = np.zeros(self.B, np.int32)
        else:
            acc = gam = p = v = rows = None
        with self.lock:
            self._check(self.lib.msckf_readback(
                self.h, n, _ptr(filters, C.c_int32), _ptr(imu, C.c_double), _ptr(cams, C.c_double),
                _ptr(nc, C.c_int32), int(i0), int(ncv), _ptr(cv, C.c_double), _ptr(acc, C.c_uint8),
                _ptr(gam, C.c_double), _ptr(p, C.c_double), _ptr(v, C.c_uint8), _ptr(rows, C.c_int32)))
        if pend is not None:
            pend.res = (acc.astype(bool), gam, p, v.astype(bool), rows)
            self._pending = None
        cl = [cams[w, :nc[w]].copy() for w in range(n)] if want_cams else [None] * n
        return imu, cl, cv

    def batch_triangulate(self):
        self._check(self.lib.msckf_batch_triangulate(self.h))

    # ---- throughput mode ----
    def batch_load(self, feat_off, obs_off, obs_cam, obs_z, p_w=None, chi2=None):
        self.settle()
        feat_off, obs_off, obs_cam = _i32(feat_off), _i32(obs_off), _i32(obs_cam)
        obs_z = _f64(obs_z, (len(obs_cam), 4))
        p_w = _f64(p_w) if p_w is not None else None
        chi2 = _f64(chi2) if chi2 is not None else None
        self._nf = int(feat_off[-1])
        with self.lock:
            self._check(self.lib.msckf_batch_load(self.h, _ptr(feat_off, C.c_int32), _ptr(obs_off, C.c_int32),
                                                  _ptr(obs_cam, C.c_int32), _ptr(obs_z, C.c_double),
                                                  _ptr(p_w, C.c_double), _ptr(chi2, C.c_double)))

    def batch_update(self, row_cap=0, triangulate=True):
        self._check(self.lib.msckf_batch_update(self.h, int(row_cap), TRIANGULATE if triangulate else 0))

    def batch_results(self):
        nf = self._nf
        acc = np.zeros(nf, np.uint8)
        gam = np.zeros(nf)
        p = np.zeros((nf, 3))
        v = np.zeros(nf, np.uint8)
        rows = np.zeros(self.B, np.int32)
        self._check(self.lib.msckf_batch_results(self.h, _ptr(acc, C.c_uint8), _ptr(gam, C.c_double),
                                                 _ptr(p, C.c_double), _ptr(v, C.c_uint8), _ptr(rows, C.c_int32)))
        return acc.astype(bool), gam, p, v.astype(bool), rows

    def device_info(self):
        """(HIP device index, PCI bus id) this context runs on."""
        dev = np.zeros(1, np.int32)
        buf = C.create_string_buffer(64)
        with self.lock:
            self._check(self.lib.msckf_device_info(self.h, _ptr(dev, C.c_int32), buf, 64))
        return int(dev[0]), buf.value.decode()

    def snapshot(self):
        self._check(self.lib.msckf_snapshot(self.h))

    def restore(self):
        self._check(self.lib.msckf_restore(self.h))

    def sync(self):
        self._check(self.lib.msckf_sync(self.h))

    def set_profiling(self, on=True):
        self._check(self.lib.msckf_set_profiling(self.h, 1 if on else 0))

    def set_profiling_stage(self, stage):
        """Time one stage only (None: profiling off)."""
        self._check(self.lib.msckf_set_profiling_stage(self.h, None if stage is None else stage.encode()))

    def kernel_times(self):
        ms = np.zeros(64)
        cnt = np.zeros(64, np.int32)
        buf = C.create_string_buffer(4096)
        k = self._check(self.lib.msckf_kernel_times(self.h, 64, _ptr(ms, C.c_double), _ptr(cnt, C.c_int32),
                                                    buf, 4096))
        names = buf.raw.split(b"\0")[:k]
        return {n.decode(): (float(ms[i]), int(cnt[i])) for i, n in enumerate(names)}


class _PendingBatch:
    """The results of one loaded batch, read back (one synchronisation) on demand."""
    __slots__ = ("ctx", "res")

    def __init__(self, ctx):
        self.ctx, self.res = ctx, None

    def read(self):
        if self.res is None:
            self.res = self.ctx.batch_results()
            if self.ctx._pending is self:
                self.ctx._pending = None
        return self.res


class Pending:
    """Deferred (accepted, gamma, p_w, valid, rows) of one filter's features."""
    __slots__ = ("grp", "slot", "a", "b")

    def __init__(self, grp, slot, a, b):
        self.grp, self.slot, self.a, self.b = grp, slot, a, b

    def get(self):
        acc, gam, p, v, rows = self.grp.read()
        a, b = self.a, self.b
        return acc[a:b].copy(), gam[a:b].copy(), p[a:b].copy(), v[a:b].copy(), int(rows[self.slot])


def pack_imu(q, p, v, bg, ba, q_null, p_null, v_null, R_imu_cam0, t_cam0_imu, gravity, alias):
    r = np.zeros(IMU_LEN)
    r[I_Q:I_Q + 4] = q
    r[I_P:I_P + 3] = p
    r[I_V:I_V + 3] = v
    r[I_BG:I_BG + 3] = bg
    r[I_BA:I_BA + 3] = ba
    r[I_QN:I_QN + 4] = q_null
    r[I_PN:I_PN + 3] = p_null
    r[I_VN:I_VN + 3] = v_null
    r[I_RIC:I_RIC + 9] = np.asarray(R_imu_cam0).ravel()
    r[I_TCI:I_TCI + 3] = t_cam0_imu
    r[I_G:I_G + 3] = gravity
    r[I_ALIAS] = 1.0 if alias else 0.0
    return r


def unpack_imu(r):
    return dict(q=r[I_Q:I_Q + 4].copy(), p=r[I_P:I_P + 3].copy(), v=r[I_V:I_V + 3].copy(),
                bg=r[I_BG:I_BG + 3].copy(), ba=r[I_BA:I_BA + 3].copy(), q_null=r[I_QN:I_QN + 4].copy(),
                p_null=r[I_PN:I_PN + 3].copy(), v_null=r[I_VN:I_VN + 3].copy(),
                R_imu_cam0=r[I_RIC:I_RIC + 9].reshape(3, 3).copy(), t_cam0_imu=r[I_TCI:I_TCI + 3].copy(),
                gravity=r[I_G:I_G + 3].copy(), alias=bool(r[I_ALIAS] != 0))


def pack_cams(q, p, q_null):
    q = np.atleast_2d(q)
    n = len(q)
    out = np.zeros((n, CAM_LEN))
    out[:, 0:4] = q
    out[:, 4:7] = np.atleast_2d(p)
    out[:, 7:11] = np.atleast_2d(q_null)
    return out
