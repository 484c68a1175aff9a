"""Propagation kernel sweep: device time of msckf_propagate_batch against the
number of filters in the launch and the IMU samples per filter (separates the
per-sample serial chain from the occupancy/tail effects).  GPU only.

    python tools/prop_sweep.py [--dtype fp32|fp64] [--N 30]
"""
import json
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402


def run(ctx, B, n_samples, steps=5):
    rng = np.random.default_rng(5)
    n = B * n_samples
    dt = np.full(n, 0.005)
    gyro = 0.2 * rng.standard_normal((n, 3))
    acc = rng.standard_normal((n, 3)) + np.array([0.0, 0.0, 9.81])
    filters = np.arange(B, dtype=np.int32)
    off = (np.arange(B + 1) * n_samples).astype(np.int32)
    ctx.restore()
    ctx.propagate_batch(filters, off, dt, gyro, acc)
    ctx.sync()
    ctx.set_profiling(True)
    for _ in range(steps):
        ctx.restore()
        ctx.propagate_batch(filters, off, dt, gyro, acc)
    ctx.sync()
    kms = ctx.kernel_times()["propagate"][0] / steps
    ctx.set_profiling(False)
    return kms


def main():
    sys.argv = [sys.argv[0], "--no-cpu"] + sys.argv[1:]
    args = bench.parse()
    dtype = np.float32 if args.dtype == "fp32" else np.float64
    probs = bench.make_problems(args, 0, min(args.unique, args.batch))
    ctx, _ = bench.build_batch(args, probs, dtype, 0)
    out = []
    one = os.environ.get("PROP_ONE")
    if one:
        B, ns = map(int, one.split(","))
        run(ctx, B, ns, steps=1)
        ctx.close()
        return
    for B in (256, 1024, args.batch):
        for ns in (1, 2, 5, 10, 20):
            kms = run(ctx, B, ns)
            out.append({"filters": B, "samples": ns, "kernel_ms": round(kms, 4),
                        "us_per_sample_round": round(kms * 1e3 / ns, 2)})
            print(json.dumps(out[-1]), flush=True)
    ctx.close()


if __name__ == "__main__":
    main()
