"""Phase timing of the one-wave MFMA gate (k_gate_mfma) per size class:
wave-cycle sums of record fetch / Y pair blocks / assembly / elimination /
finish, from the probe build (`make probe`, -DMSCKF_GATE_PROBE).  GPU only.
Caveat: the probe's own device-scope atomics sit in each wave's in-order
vmcnt queue, so a phase that waits on a later load also waits for them --
read the split as indicative only (SQ counters are the clean measurement).

    python tools/probes/gate_phases.py [--dtype fp32|fp64] [--batch 2048]
"""
import ctypes as C
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
import bench  # noqa: E402
from msckf_amd import _lib  # noqa: E402

PH = ["fetch", "y_pairs", "assemble", "eliminate", "finish", "total"]


def main():
    lib = _lib.load_library(os.path.join(ROOT, "tools", "probes", "libmsckf_probe.so"))
    read = lib.msckf_gate_probe_read
    read.restype = C.c_int
    read.argtypes = [C.POINTER(C.c_ulonglong)]
    sys.argv = [sys.argv[0], "--no-cpu"] + sys.argv[1:]
    args = bench.parse()
    dtype = np.float32 if args.dtype == "fp32" else np.float64
    probs = bench.make_problems(args, 0, min(args.unique, args.batch))
    ctx, _ = bench.build_batch(args, probs, dtype, 0)
    buf = (C.c_ulonglong * (2 * 9 * 8))()
    ctx.restore(); ctx.batch_update(row_cap=0, triangulate=True); ctx.sync()
    read(buf)   # reset after the warm-up
    ctx.restore(); ctx.batch_update(row_cap=0, triangulate=True); ctx.sync()
    read(buf)
    a = np.frombuffer(buf, dtype=np.uint64).reshape(2, 9, 8).astype(float)
    out = {}
    for t, kind in ((0, "per_feature_f32"), (1, "per_feature_f64")):
        for nb in range(1, 9):
            w = a[t, nb, 6]
            if w == 0:
                continue
            ph = PH if t < 2 else ["scatter_prefetch", "y_pairs", "assemble", "eliminate", "finish", "total"]
            row = dict({"features": int(w)}, **{p: round(a[t, nb, i] / w) for i, p in enumerate(ph)})
            out["%s NB%d" % (kind, nb)] = row
    print(json.dumps({"dtype": args.dtype, "cycles_per_wave": out}, indent=1))
    ctx.close()


if __name__ == "__main__":
    main()
