"""Debug: block structure of the covariance error of one golden update."""
import os, sys
import numpy as np
ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT); sys.path.insert(0, os.path.join(ROOT, "tests"))
import msckf_pkg  # noqa
from conftest import golden
from test_gpu_parity import make_ctx, chi2_for
for name in ("update_n10_f40", "update_n20_f100"):
    d = golden(name)
    for cap in (None, int(d["N"])):
        ctx = make_ctx(d, cap=cap)
        F = int(d["F"])
        sel = [f for f in range(F) if d["tri_ok"][f]]
        off, cams, zs = [0], [], []
        for f in sel:
            a, b = int(d["obs_off"][f]), int(d["obs_off"][f + 1])
            cams.extend(d["obs_cam"][a:b]); zs.extend(d["obs_z"][a:b]); off.append(len(cams))
        acc, gam, rows = ctx.update(0, off, cams, zs, d["tri_p"][sel], chi2_for(np.diff(off)), row_cap=0)
        _, _, P = ctx.get_state(0)
        ctx.close()
        E = np.abs(P - d["P_out"]) / np.abs(d["P_out"]).max()
        n = (P.shape[0] - 21) // 6
        print(name, "cap", cap, "rel err total %.3e" % (np.linalg.norm(P - d["P_out"]) / np.linalg.norm(d["P_out"])),
              "imu-imu %.2e imu-cam %.2e cam-cam %.2e" % (E[:21, :21].max(), E[21:, :21].max(), E[21:, 21:].max()))
        cb = [E[21 + 6 * i:27 + 6 * i, 21:].max() for i in range(n)]
        print("   per cam row block:", " ".join("%.1e" % x for x in cb))
