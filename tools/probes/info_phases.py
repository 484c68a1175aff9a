"""Phase cycles of the fused information assembly (k_info_fused) from the
probe build (`make probe`, -DMSCKF_GATE_PROBE): per filter and per chunk
iteration, one producer wave's load issue / build / barrier wait and one
tile-owner wave's MFMA phase / barrier wait (s_memtime cycles).  GPU only.
    python tools/probes/info_phases.py [bench args]
"""
import ctypes as C
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
import msckf_pkg  # noqa: E402,F401
import bench  # noqa: E402
from msckf_amd import _lib  # noqa: E402


def main():
    lib = _lib.load_library(os.path.join(ROOT, "tools", "probes", "libmsckf_probe.so"))
    read = lib.msckf_info_probe_read
    read.restype = C.c_int
    read.argtypes = [C.POINTER(C.c_ulonglong)]
    sys.argv = [sys.argv[0], "--no-cpu"] + sys.argv[1:]
    args = bench.parse()
    dtype = np.float32 if args.dtype == "fp32" else np.float64
    probs = bench.make_problems(args, 0, min(args.unique, args.batch))
    ctx, _ = bench.build_batch(args, probs, dtype, 0)
    buf = (C.c_ulonglong * 8)()
    ctx.restore(); ctx.batch_update(row_cap=0, triangulate=True); ctx.sync()
    read(buf)
    ctx.restore(); ctx.batch_update(row_cap=0, triangulate=True); ctx.sync()
    read(buf)
    a = np.frombuffer(buf, dtype=np.uint64).astype(float)
    nf, it = a[7], a[6]
    names = ["prologue", "prod_load_issue", "prod_build", "prod_barrier", "owner_mfma", "owner_barrier"]
    out = {"filters": int(nf), "iterations_per_filter": it / max(nf, 1),
           "cycles_per_filter": {n: round(a[i] / max(nf, 1)) for i, n in enumerate(names)},
           "cycles_per_iteration": {n: round(a[i] / max(it, 1)) for i, n in enumerate(names) if i > 0}}
    print(json.dumps(out, indent=1))
    ctx.close()


if __name__ == "__main__":
    main()
