"""CPU-only checks of the drop-in boundary: the C-ABI library loads and
exports every entry point include/msckf_hip.h declares; the ctypes binding
types exactly those; host-side packing helpers round-trip.  No compute calls
(there is no GPU here)."""
import ctypes
import os
import re

import numpy as np
import pytest

import msckf_amd
from msckf_amd import _lib

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def header_symbols(header="msckf_hip.h", prefix="msckf_"):
    src = open(os.path.join(ROOT, "include", header)).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"\b(%s[a-z_]+)\s*\(" % prefix, src)))


def test_library_exports_every_declared_symbol():
    if not os.path.exists(_lib.LIB_PATH):
        pytest.skip("libmsckf_hip.so not built (run `make`)")
    lib = ctypes.CDLL(_lib.LIB_PATH)
    syms = header_symbols()
    assert len(syms) >= 20
    for s in syms:
        assert hasattr(lib, s), s


def test_binding_matches_header():
    assert sorted(_lib.EXPORTED) == header_symbols()


def test_frontend_exports_and_binding():
    """include/msckf_frontend.h (GPU stereo front-end) is exported by the same
    library and typed one to one by the binding."""
    syms = header_symbols("msckf_frontend.h", "mfe_")
    assert sorted(_lib.FRONTEND_EXPORTED) == syms and len(syms) == 8
    if not os.path.exists(_lib.LIB_PATH):
        pytest.skip("libmsckf_hip.so not built")
    lib = ctypes.CDLL(_lib.LIB_PATH)
    for s in syms:
        assert hasattr(lib, s), s


def test_replica_transport_exports_and_binding():
    """include/msckf_replicas.h (RCCL replica transport) is exported by the
    same library and typed one to one by the binding; librccl itself is opened
    only when a communicator is made (dlopen), so loading needs no RCCL."""
    syms = header_symbols("msckf_replicas.h", "msckf_rccl_")
    assert sorted(_lib.REPLICA_EXPORTED) == syms and len(syms) == 8
    if not os.path.exists(_lib.LIB_PATH):
        pytest.skip("libmsckf_hip.so not built")
    lib = ctypes.CDLL(_lib.LIB_PATH)
    for s in syms:
        assert hasattr(lib, s), s


def test_load_library_types_functions():
    if not os.path.exists(_lib.LIB_PATH):
        pytest.skip("libmsckf_hip.so not built")
    lib = _lib.load_library()
    assert lib.msckf_create.restype is ctypes.c_int
    assert lib.msckf_last_error.restype is ctypes.c_char_p


def test_config_struct_layout():
    # 5 + 9 + 3 + 3 doubles, then 2 int32
    assert ctypes.sizeof(_lib.MsckfConfigT) == 20 * 8 + 2 * 4
    c = _lib.make_config(msckf_amd.FilterConfig())
    assert c.observation_noise == pytest.approx(0.035 ** 2)
    assert c.outer_loop_max_iteration == 5
    assert c.t_cam0_cam1[0] == pytest.approx(-0.110073808127187)


def test_imu_pack_roundtrip():
    rng = np.random.default_rng(0)
    vals = dict(q=rng.standard_normal(4), p=rng.standard_normal(3), v=rng.standard_normal(3),
                bg=rng.standard_normal(3), ba=rng.standard_normal(3), q_null=rng.standard_normal(4),
                p_null=rng.standard_normal(3), v_null=rng.standard_normal(3),
                R_imu_cam0=rng.standard_normal((3, 3)), t_cam0_imu=rng.standard_normal(3),
                gravity=rng.standard_normal(3), alias=True)
    r = _lib.pack_imu(**vals)
    assert r.shape == (_lib.IMU_LEN,)
    u = _lib.unpack_imu(r)
    for k, v in vals.items():
        np.testing.assert_array_equal(u[k], v)


def test_config_from_reference_object():
    """A reference-style ConfigEuRoC object (attribute names of config.py)
    converts without loss."""
    class O:
        pass
    cfg = msckf_amd.FilterConfig()
    ref = O()
    oc = O()
    for k, v in vars(cfg.optimization).items():
        setattr(oc, "_vio_%s__" % k, v)
    ref._vio_optimization_config__ = oc
    for k, v in vars(cfg).items():
        if k != "optimization":
            setattr(ref, "_vio_%s__" % k, v)
    c2 = msckf_amd.FilterConfig.from_reference(ref)
    assert c2.observation_noise == cfg.observation_noise
    np.testing.assert_array_equal(c2.T_cn_cnm1, cfg.T_cn_cnm1)
    assert c2.optimization.outer_loop_max_iteration == 5


def test_no_oracle_import_in_product():
    pkg = os.path.join(ROOT, "visual-inertial-odometry-msckf-stereo_amd")
    for dirpath, _, files in os.walk(pkg):
        for f in files:
            if f.endswith(".py"):
                src = open(os.path.join(dirpath, f)).read()
                assert not re.search(r"^\s*(from|import)\s+oracle", src, re.M), f
