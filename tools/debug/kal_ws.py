"""Debug: Kalman stage-A workspace (Lc, Vi, S_ii) after one golden update,
against a numpy partial Cholesky of the input covariance."""
import ctypes as C
import os, sys
import numpy as np
ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT); sys.path.insert(0, os.path.join(ROOT, "tests"))
import msckf_pkg  # noqa
from conftest import golden
from test_gpu_parity import make_ctx, chi2_for


def read(ctx, which, n):
    out = np.zeros(n)
    fn = ctx.lib.msckf_debug_workspace
    fn.argtypes = [C.c_void_p, C.c_int, C.POINTER(C.c_double), C.c_size_t]
    rc = fn(ctx.h, which, out.ctypes.data_as(C.POINTER(C.c_double)), n)
    assert rc == 0, rc
    return out


for name in ("update_n10_f40", "update_n20_f100"):
    d = golden(name)
    for cap in (None, int(d["N"])):
        ctx = make_ctx(d, cap=cap)
        N = int(d["N"]); Cn = 6 * N
        capn = cap or N + 2
        Cmax = 6 * capn; Cp = (Cmax + 15) & ~15
        F = int(d["F"])
        sel = [f for f in range(F) if d["tri_ok"][f]]
        off, cams, zs = [0], [], []
        for f in sel:
            a, b = int(d["obs_off"][f]), int(d["obs_off"][f + 1])
            cams.extend(d["obs_cam"][a:b]); zs.extend(d["obs_z"][a:b]); off.append(len(cams))
        ctx.update(0, off, cams, zs, d["tri_p"][sel], chi2_for(np.diff(off)), row_cap=0)
        Lc = read(ctx, 0, Cp * Cp).reshape(Cp, Cp)[:Cn, :Cn]
        Vi = read(ctx, 1, 24 * Cp).reshape(24, Cp)[:21, :Cn]
        Sii = read(ctx, 2, 24 * 24).reshape(24, 24)[:21, :21]
        ctx.close()
        P = d["P"]
        Pcc, Pic, Pii = P[21:, 21:], P[:21, 21:], P[:21, :21]
        L = np.linalg.cholesky(Pcc)
        V = np.linalg.solve(L, Pic.T).T
        S = Pii - V @ V.T
        lo = np.tril_indices(21)
        print(name, "cap", cap, "Lc %.2e  Vi %.2e  Sii(lower) %.2e  Sii upper-only %.2e" % (
            np.abs(np.tril(Lc) - L).max() / np.abs(L).max(), np.abs(Vi - V).max() / np.abs(V).max(),
            np.abs(Sii[lo] - S[lo]).max() / np.abs(S).max(),
            np.abs(np.triu(Sii, 1) - np.triu(S, 1)).max() / np.abs(S).max()))
        E = np.abs(Sii - S) / np.abs(S).max()
        bad = np.argwhere(np.tril(E) > 1e-8)
        print("   bad lower entries:", len(bad), bad[:12].tolist())
