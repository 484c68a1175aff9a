"""Experiment: the headline batch (2048 filters) split over K contexts, each
with its own HIP streams, their update chains enqueued back to back so the
GPU can overlap one sub-batch's Kalman stages with another's gating.

    python tools/exp_two_ctx.py [--k 1 2 4] [--steps 20]
"""
import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402


def run(k, steps, warmup):
    sys.argv = [sys.argv[0], "--no-cpu"]
    args = bench.parse()
    B = args.batch
    probs = bench.make_problems(args, 0, min(args.unique, B))
    sub = B // k
    ctxs = []
    for i in range(k):
        a = argparse.Namespace(**vars(args))
        a.batch = sub
        ctx, _ = bench.build_batch(a, probs[i:] + probs[:i], np.float32, 0)
        ctxs.append(ctx)
    for _ in range(warmup):
        for c in ctxs:
            c.restore()
            c.batch_update(row_cap=0, triangulate=True)
    for c in ctxs:
        c.sync()
    t0 = time.perf_counter()
    for _ in range(steps):
        for c in ctxs:
            c.restore()
            c.batch_update(row_cap=0, triangulate=True)
    for c in ctxs:
        c.sync()
    el = time.perf_counter() - t0
    for c in ctxs:
        c.close()
    return {"k": k, "filters": sub * k, "ms_per_step": round(el / steps * 1e3, 3),
            "updates_per_s": round(sub * k * steps / el, 1)}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--k", type=int, nargs="+", default=[1, 2, 4])
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    a = ap.parse_args()
    for k in a.k:
        print(json.dumps(run(k, a.steps, a.warmup)), flush=True)


if __name__ == "__main__":
    main()
