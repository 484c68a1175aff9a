"""Debug: the degenerate-gate fixture's update with a given library -- the
assembled [A | b] (H_thin), T, and stage-A status -- to find non-finite values."""
import ctypes as C
import os, sys
import numpy as np
ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT); sys.path.insert(0, os.path.join(ROOT, "tests"))
import msckf_pkg  # noqa
from msckf_amd import _lib, FilterConfig
if len(sys.argv) > 1:
    _lib.load_library(os.path.abspath(sys.argv[1]))
from msckf_amd._lib import Context
from conftest import golden

g = golden("degenerate_gate")
n = (g["P"].shape[0] - 21) // 6
ctx = Context(FilterConfig(), n_filters=1, n_cam_capacity=n + 2, dtype=np.float64)
ctx.set_state(0, g["imu"], g["cams"], g["P"])
try:
    acc, gam, rows = ctx.update(0, g["obs_off"], g["obs_cam"], g["obs_z"], g["p_w"], g["chi2"])
    print("update ok", acc, gam, rows)
except Exception as e:
    print("update failed:", e)
fn = ctx.lib.msckf_debug_workspace
fn.argtypes = [C.c_void_p, C.c_int, C.POINTER(C.c_double), C.c_size_t]
Cmax = 6 * (n + 2)
def read(which, cnt):
    out = np.zeros(cnt)
    assert fn(ctx.h, which, out.ctypes.data_as(C.POINTER(C.c_double)), cnt) == 0
    return out
H = read(6, Cmax * (Cmax + 1)).reshape(Cmax, Cmax + 1)
Cn = 6 * n
A, b = H[:Cn, :Cn], H[:Cn, Cmax]
print("A finite", np.isfinite(A).all(), "b finite", np.isfinite(b).all(), "|A|", np.abs(A).max(), "sym", np.abs(A - A.T).max())
ev = np.linalg.eigvalsh((A + A.T) / 2) if np.isfinite(A).all() else None
print("A eig min/max", None if ev is None else (ev.min(), ev.max()))
T = read(4, Cmax * (Cmax + 1)).reshape(Cmax, Cmax + 1)[:Cn, :Cn]
print("T finite", np.isfinite(np.tril(T)).all(), "diag", np.diag(T)[:8])
af = read(7, 1).view(np.int32)
print("afail", af[:2])
