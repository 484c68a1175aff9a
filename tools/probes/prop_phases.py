"""Phase timing of the IMU propagation kernel (k_propagate): wave-cycle sums
of its start (P11 load, cross-block prefetch), the chunk scalars (phases
A..B4), the per-sample Phi (C1..C3b), the Q term (C4..C5), D1, D2, D3 and the
end (write-back, cross blocks), from the probe build (`make probe`,
-DMSCKF_GATE_PROBE), on the bench's propagation shape (2048 filters x 10
samples, 30 cams).  GPU only.  The probe's own atomics perturb the timing a
little: read the split as indicative.

    python tools/probes/prop_phases.py [--dtype fp32|fp64] [--batch 2048] [--samples 10]
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

PH = ["start", "chunk_scalars", "phi_C1_C3b", "q_C4_C5", "D1", "D2", "D3", "end_cross_block", "total"]


def main():
    lib = _lib.load_library(os.path.join(ROOT, "tools", "probes", "libmsckf_probe.so"))
    read = lib.msckf_prop_probe_read
    read.restype = C.c_int
    read.argtypes = [C.POINTER(C.c_ulonglong)]
    ns = 10
    if "--samples" in sys.argv:
        i = sys.argv.index("--samples")
        ns = int(sys.argv[i + 1])
        del sys.argv[i:i + 2]
    sys.argv = [sys.argv[0], "--no-cpu"] + sys.argv[1:]
    args = bench.parse()
    dtype = np.float32 if args.dtype == "fp32" else np.float64
    probs = bench.make_problems(args, 0, min(args.unique, args.batch))
    ctx, _ = bench.build_batch(args, probs, dtype, 0)
    B = args.batch
    rng = np.random.default_rng(5)
    n = B * ns
    dt = np.full(n, 0.005)
    gyro = 0.2 * rng.standard_normal((n, 3))
    acc = rng.standard_normal((n, 3)) + np.array([0.0, 0.0, 9.81])
    filters = np.arange(B, dtype=np.int32)
    off = (np.arange(B + 1) * ns).astype(np.int32)
    buf = (C.c_ulonglong * 20)()
    ctx.restore(); ctx.propagate_batch(filters, off, dt, gyro, acc); ctx.sync()
    read(buf)   # reset after the warm-up
    reps = 5
    for _ in range(reps):
        ctx.restore(); ctx.propagate_batch(filters, off, dt, gyro, acc)
    ctx.sync()
    read(buf)
    a = np.frombuffer(buf, dtype=np.uint64).reshape(2, 10).astype(float)
    k = 1 if dtype == np.float64 else 0
    waves = max(a[k, 9], 1.0)
    per = {PH[i]: round(a[k, i] / waves, 1) for i in range(9)}
    tot = per["total"]
    print(json.dumps({"dtype": args.dtype, "filters": B, "samples": ns, "waves": int(waves),
                      "cycles_per_wave": per,
                      "fraction": {p: round(v / tot, 3) for p, v in per.items() if p != "total"}}))
    ctx.close()


if __name__ == "__main__":
    main()
