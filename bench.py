"""Throughput bench: EKF measurement updates/s at N cam-states x F features
(default 30 x 200, BASELINE.json's metric).

One "step" = one batched EKF measurement update of B independent filters
(SURVEY.md 8(d) unit of work): triangulation of every feature, per-feature
Jacobian + nullspace projection + chi2 gating, stacking (no row cap), the
compression of the stacked rows (information assembly) and the
Kalman / covariance update -- on inputs already resident in HBM.  Each step
first restores the filters' pristine state on the device (a D2D copy that is
counted inside the timed region) so every step does identical work.

  python bench.py [--gpus N --steps K --warmup W --batch B --N 30 --F 200 --dtype fp32]

The JSON line carries the headline (fp32 context, BASELINE config 2) and,
unless --no-fp64, the same workload in the fp64 context (the precision the
north-star's 1e-6 tolerance is stated at) as ``fp64``; ``accuracy`` compares
the GPU's updated filters with the CPU oracle's (computed in the
cpu_baseline leg, as the checker).

--gpus N > 1: N ranks, one process per GPU -- spawned by this script (its
parent process never touches the GPU) or by an external launcher
(torch.distributed.run sets WORLD_SIZE).  Ranks are independent replicas
(the filter does not shard): disjoint problem seeds, no data
exchange.  RCCL (msckf_amd.replicas, include/msckf_replicas.h) carries only
the start/stop barriers, the max-over-ranks of the elapsed time and the device
gather; a host TCP hub hands out its unique id (and carries the control
messages itself if RCCL cannot come up -- ``replicas`` in the line says which).
"""
import argparse
import json
import os
import platform
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)
import msckf_pkg  # noqa: E402,F401
from msckf_amd import synth, replicas, FilterConfig, CHI2_05  # noqa: E402

BASE_METRIC = "EKF measurement updates/sec at 30 cam-states x 200 features; ATE RMSE vs ref"
HBM_PEAK_GBS = 8000.0
FP32_PEAK_TFLOPS = 157.3      # MI355X dense FP32 (vector = MFMA f32 rate), MI355X_MICROARCH.md
FP64_PEAK_TFLOPS = 78.6
N_CHECK = 4                   # distinct problems the accuracy block compares with the oracle


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=50)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--batch", type=int, default=2048, help="independent filters per GPU per step")
    ap.add_argument("--N", type=int, default=30)
    ap.add_argument("--F", type=int, default=200)
    ap.add_argument("--dtype", default="fp32", choices=["fp32", "fp64"])
    ap.add_argument("--unique", type=int, default=32, help="distinct synthetic problems tiled over the batch")
    ap.add_argument("--cpu-seconds", type=float, default=15.0, help="budget of the CPU-baseline sample")
    ap.add_argument("--rccl-timeout", type=float, default=1800.0,
                    help="deadline (s) of every replica collective once RCCL is up (rank 0 runs the accuracy / "
                         "ATE legs while the others wait in a barrier)")
    ap.add_argument("--no-cpu", action="store_true")
    ap.add_argument("--no-fp64", action="store_true", help="skip the fp64-context leg")
    ap.add_argument("--no-ate", action="store_true", help="skip the ATE replay leg")
    ap.add_argument("--no-prop", action="store_true", help="skip the IMU-propagation leg")
    ap.add_argument("--stub", action="store_true",
                    help="TESTS ONLY: a CPU stand-in for the device context (exercises the multi-rank launch, "
                         "barriers and max-over-ranks without a GPU; the line it prints is not a measurement)")
    return ap.parse_args()


def metric_name(args):
    if (args.N, args.F) == (30, 200):
        return BASE_METRIC
    return "EKF measurement updates/sec at %d cam-states x %d features" % (args.N, args.F)


def make_problems(args, rank, unique):
    return [synth.make_update_problem(args.N, args.F, seed=sd) for sd in replicas.problem_seeds(rank, unique)]


def build_batch(args, probs, dtype, device):
    from msckf_amd._lib import Context, pack_imu, pack_cams
    B = args.batch
    ctx = Context(FilterConfig(), n_filters=B, n_cam_capacity=args.N, dtype=dtype, device=device)
    feat_off, obs_off, cams, zs, chi = [0], [0], [], [], []
    for b in range(B):
        p = probs[b % len(probs)]
        imu = pack_imu(q=p.imu["q"], p=p.imu["p"], v=p.imu["v"], bg=p.imu["bg"], ba=p.imu["ba"],
                       q_null=p.imu["q_null"], p_null=p.imu["p_null"], v_null=p.imu["v_null"],
                       R_imu_cam0=p.imu["R_imu_cam0"], t_cam0_imu=p.imu["t_cam0_imu"], gravity=p.gravity,
                       alias=True)
        ctx.set_state(b, imu, pack_cams(p.cam_q, p.cam_p, p.cam_q_null), p.P)
        feat_off.append(feat_off[-1] + p.F)
        obs_off.extend(list(obs_off[-1] + p.obs_off[1:]))
        cams.append(p.obs_cam)
        zs.append(p.obs_z)
        chi.extend(CHI2_05[m - 2] for m in p.track_lengths())
    ctx.batch_load(np.array(feat_off), np.array(obs_off), np.concatenate(cams), np.concatenate(zs),
                   None, np.array(chi))
    ctx.snapshot()
    return ctx, np.array(feat_off)


def flops_model(probs, B, accepted, valid, feat_off):
    """Algorithmic flops of one step, per kernel-timer stage, from the realised
    shapes (FMA = 2 flops; DESIGN.md 'Kernels' states each formula), plus
    'canonical' = SURVEY.md 8(d)'s per-update formula (dense Householder QR of
    the stacked R x C matrix, rows-space gating)."""
    tot = {"canonical": 0.0, "gate": 0.0, "compress": 0.0, "kalman_a": 0.0, "kalman_b": 0.0,
           "kalman_c": 0.0, "kalman_e": 0.0}
    for b in range(B):
        p = probs[b % len(probs)]
        C = 6 * p.N
        D = 21 + C
        M = p.track_lengths().astype(float)
        acc = accepted[feat_off[b]:feat_off[b + 1]].astype(float)
        val = valid[feat_off[b]:feat_off[b + 1]].astype(float)
        k = 4 * M - 3
        # gating (rank-3 reduced saddle point): 3x3 observation-pair blocks Ht_a P_ab Ht_b^T
        # (3x6 . 6x6 . 6x3 = 162 FMA per pair) + LDL^T of the (3M+4)^2 matrix
        tot["gate"] += 2 * float(np.sum(val * (162.0 * M * (M + 1) / 2 + (3 * M + 4) ** 3 / 6)))
        # information assembly: per included feature, every observed cam pair takes G_i^T G_j (3 x 6 x 6)
        tot["compress"] += 2 * float(np.sum(acc * (54.0 * M * (M + 1) + 27 * M)))
        if acc.sum() > 0:
            # algorithmic (implementation-independent) counts: partial Cholesky over the
            # C cam pivots of the (C+21)^2 [P_cc P_ci; P_ic P_ii]; G = A Lc and Lc^T G;
            # Cholesky of T plus the forward substitution of the E = 22 + C extra rows
            N = C + 21
            tot["kalman_a"] += 2 * (N ** 3 - (N - C) ** 3) / 6
            tot["kalman_b"] += 2 * (C ** 3 / 2 + C ** 3 / 6 + C * C / 2)
            tot["kalman_c"] += 2 * (C ** 3 / 6 + (22 + C) * C * C / 2)
            tot["kalman_e"] += 2 * (D * (D + 1) / 2 * C + D * C)
        R = float(np.sum(k * acc))
        n = min(R, C)
        F_proj = float(np.sum(48.0 * M * (6 * M + 1)))
        F_gate = float(np.sum(2 * k * (6 * M) ** 2 + 2 * k ** 2 * (6 * M) + k ** 3 / 3 + 2 * k ** 2))
        F_qr = 2 * C * C * (R - C / 3) + 4 * R * C if R > C else 0.0
        F_kal = 2 * n * C * D + 2 * n * n * C + n ** 3 / 3 + 2 * n * n * D + 2 * n * D + 2 * n * D * D + D * D
        tot["canonical"] += F_proj + F_gate + F_qr + F_kal
    return tot


def pmc_traffic(stage, dtype, workload):
    """HBM bytes per step of a stage's kernels from the committed rocprofv3 PMC
    summary (tools/pmc_summary.py; FETCH_SIZE and WRITE_SIZE from separate
    passes, FETCH_SIZE doubled as MI355X_MICROARCH.md prescribes for gfx950),
    or None if no summary covers them."""
    # the headline workload's summary, or one per (workload, dtype) for the other
    # configs (tools/profile_round.sh writes profiles/pmc_summary_<workload>_<dtype>.json)
    for name in ("pmc_summary.json", "pmc_summary_%s_%s.json" % (workload, dtype)):
        path = os.path.join(ROOT, "profiles", name)
        if not os.path.exists(path):
            continue
        with open(path) as fh:
            summ = json.load(fh)
        if summ.get("dtype") != dtype or summ.get("workload", "N30xF200xB2048") != workload:
            continue
        return summ.get("stages", {}).get(stage, {}).get("fetch_x2_bytes_per_step")
    return None


# ------------------------------------------------------------ cpu_baseline --
def _oracle_worker(payload):
    """One CPU worker of the baseline: oracle updates on 1 BLAS thread for
    about ``seconds``; returns (updates, elapsed, outputs of the first
    ``keep`` distinct problems)."""
    probs, seconds, tests_dir, keep = payload
    sys.path.insert(0, tests_dir)
    from helpers import problem_to_dict, oracle_update
    try:
        from threadpoolctl import threadpool_limits
        threadpool_limits(1)
    except Exception:
        pass
    oracle_update(problem_to_dict(probs[0]))          # warm-up
    done, outs, t0 = 0, [], time.perf_counter()
    while True:
        st, acc, _, _, _ = oracle_update(problem_to_dict(probs[done % len(probs)]))
        if done < keep:
            outs.append((st, acc))
        done += 1
        el = time.perf_counter() - t0
        if el > seconds and done >= keep:
            return done, el, outs


def cpu_model():
    try:
        with open("/proc/cpuinfo") as fh:
            for line in fh:
                if line.startswith("model name"):
                    return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return platform.processor() or platform.machine()


def cpu_baseline(args, probs):
    """Oracle (numpy restatement of the reference) on a bounded sample of the
    same workload: 1 BLAS thread in this process, and -- SURVEY.md 8(d) asks
    for both -- one single-threaded worker per host core of this job's CPU
    share (forked before this process touches the GPU).  The first N_CHECK
    distinct problems' oracle outputs are kept for the accuracy block."""
    tests_dir = os.path.join(ROOT, "tests")
    done, el, outs = _oracle_worker((probs, args.cpu_seconds, tests_dir, min(N_CHECK, len(probs))))
    out = {"value": done / el, "unit": "updates/s", "cores": 1, "kind": "port", "cpu": cpu_model(),
           "sample": "%d synthetic %dx%d updates (triangulation + jacobian + gating + QR + Kalman as in the reference), "
                     "numpy/OpenBLAS 1 thread, oracle/msckf_oracle.py" % (done, args.N, args.F)}
    try:
        ncpu = len(os.sched_getaffinity(0))
    except Exception:
        ncpu = os.cpu_count() or 1
    workers = max(1, min(16, ncpu))
    if workers > 1 and args.cpu_seconds > 0:
        import multiprocessing as mp
        with mp.get_context("fork").Pool(workers) as pool:
            res = pool.map(_oracle_worker, [(probs[w % len(probs):] + probs[:w % len(probs)],
                                             args.cpu_seconds / 2, tests_dir, 0) for w in range(workers)])
        out["all_cores"] = {"value": sum(r[0] for r in res) / max(r[1] for r in res), "unit": "updates/s",
                            "cores": workers, "sample": "%d updates over %d single-threaded worker processes"
                                                        % (sum(r[0] for r in res), workers)}
    return out, outs


def _state_vector(imu, cams):
    return np.concatenate([imu["q"], imu["p"], imu["v"], imu["bg"], imu["ba"],
                           np.asarray(cams)[:, 0:7].ravel()])


def accuracy(ctx, refs, acc, feat_off):
    """Checker: the GPU's updated filters 0..len(refs)-1 against the oracle's
    outputs for the same problems (from the cpu_baseline leg): chi2 decision
    agreement, relative deviation of the state vector (IMU q, p, v, bg, ba and
    every cam's q, p) and of the covariance (Frobenius), the north-star
    quantities (<= 1e-6 relative)."""
    from msckf_amd._lib import unpack_imu
    agree, sdev, pdev = [], [], []
    for b, (st, acc_o) in enumerate(refs):
        sl = slice(feat_off[b], feat_off[b + 1])
        agree.append(float(np.mean(acc[sl].astype(bool) == acc_o)))
        imu, cams, P = ctx.get_state(b)
        x = _state_vector(unpack_imu(imu), cams)
        xo = np.concatenate([st.imu.q, st.imu.p, st.imu.v, st.imu.bg, st.imu.ba] +
                            [np.concatenate([c.q, c.p]) for c in st.cams.values()])
        sdev.append(float(np.linalg.norm(x - xo) / np.linalg.norm(xo)))
        pdev.append(float(np.linalg.norm(P - st.P) / np.linalg.norm(st.P)))
    return {"filters_checked": len(refs), "decision_agreement": min(agree),
            "state_rel_dev_max": max(sdev), "cov_frobenius_rel_dev_max": max(pdev),
            "within_1e-6": bool(max(sdev) <= 1e-6 and max(pdev) <= 1e-6),
            "reference": "oracle/msckf_oracle.py (fp64 numpy restatement of the reference, pinned to its fixtures) "
                         "on the same problems, its own triangulation and decisions"}


# ------------------------------------------------------------------- legs --
def timed_update(ctx, args, grp):
    """Warm-up; a profiled pass of args.steps steps (every stage timed with HIP
    events, outside the timed region: the per-stage breakdown and the dominant
    stage); then exactly args.steps timed steps between barriers, the device
    synchronised on both sides, with HIP events around the dominant stage only
    (two event packets per step instead of two per stage).  Returns
    (max-over-ranks seconds, per-stage times of the profiled pass, the
    dominant stage's times from the timed region)."""
    for _ in range(args.warmup):
        ctx.restore()
        ctx.batch_update(row_cap=0, triangulate=True)
    ctx.sync()
    ctx.set_profiling(True)
    for _ in range(args.steps):
        ctx.restore()
        ctx.batch_update(row_cap=0, triangulate=True)
    ctx.sync()
    stages = ctx.kernel_times()
    ctx.set_profiling(False)
    dom = max((k for k in stages if k != "restore"), key=lambda k: stages[k][0])
    ctx.set_profiling_stage(dom)
    grp.barrier()
    ctx.sync()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        ctx.restore()
        ctx.batch_update(row_cap=0, triangulate=True)
    ctx.sync()
    grp.barrier()
    el = time.perf_counter() - t0
    timed = ctx.kernel_times()
    ctx.set_profiling(False)
    return grp.max_over_ranks(el), stages, timed


def roofline_of(times, fl, args, dtype):
    """Dominant stage by device time (HIP events on the launch stream around
    that stage, inside the timed region) against the peak of its arithmetic
    type."""
    kern = {k: v for k, v in times.items() if k != "restore"}
    dom = max(kern, key=lambda k: kern[k][0])
    dom_ms = kern[dom][0] / args.steps
    dom_flops = fl.get(dom)
    # gating computes in the context's scalar type; projection, assembly and Kalman stages in fp64
    peak = (FP32_PEAK_TFLOPS if dtype == "fp32" else FP64_PEAK_TFLOPS) if dom == "gate" else FP64_PEAK_TFLOPS
    if not dom_flops:
        return None
    ach = dom_flops / (dom_ms * 1e-3) / 1e12
    traffic = pmc_traffic(dom, dtype, "N%dxF%dxB%d" % (args.N, args.F, args.batch))
    return {"bound": "mfma", "kernel": dom, "achieved": round(ach, 3), "peak": peak, "unit": "TFLOP/s",
            "frac": round(ach / peak, 5), "traffic": traffic, "ms_per_step": round(dom_ms, 4),
            "flops_per_step": dom_flops,
            "note": "peak of the stage's arithmetic type (fp32 vector = fp32 MFMA, fp64 vector = fp64 MFMA on "
                    "MI355X); achieved = algorithmic flops (DESIGN.md section 5) / HIP-event device time; traffic = "
                    "PMC 2 x FETCH_SIZE + WRITE_SIZE bytes per step (profiles/pmc_summary.json)"}


def no_triangulation_leg(ctx, args, grp):
    """updates/s without the triangulation (positions from
    the previous triangulating step stay resident), the quantity the survey's
    CPU probe numbers are quoted on."""
    ctx.restore()
    ctx.batch_update(row_cap=0, triangulate=False)
    ctx.sync()
    grp.barrier()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        ctx.restore()
        ctx.batch_update(row_cap=0, triangulate=False)
    ctx.sync()
    grp.barrier()
    el = grp.max_over_ranks(time.perf_counter() - t0)
    return {"value": round(replicas.whole_job_rate(args.batch, grp.world, args.steps, el), 2),
            "unit": "updates/s", "ms_per_step": round(el / args.steps * 1e3, 3)}


def fp64_leg(args, grp, probs, refs):
    ctx, feat_off = build_batch(args, probs, np.float64, grp.local_rank)
    el, times, timed = timed_update(ctx, args, grp)
    acc, gam, pw, valid, rows = ctx.batch_results()
    fl = flops_model(probs, args.batch, acc, valid, feat_off)
    out = {"value": round(replicas.whole_job_rate(args.batch, grp.world, args.steps, el), 2),
           "unit": "updates/s", "dtype": "f64", "ms_per_step": round(el / args.steps * 1e3, 3),
           "roofline": roofline_of(timed, fl, args, "fp64"),
           "kernel_ms_per_step": {k: round(v[0] / args.steps, 3)
                                  for k, v in sorted(times.items(), key=lambda kv: -kv[1][0])}}
    if refs:
        out["accuracy"] = accuracy(ctx, refs, acc, feat_off)
    ctx.close()
    return out


def propagation_leg(ctx, args, n_samples=10, steps=5):
    """IMU propagation (A2-A4) reported separately, at the same
    D, as IMU samples/s: every filter of the batch takes n_samples samples
    (one frame's worth at 200 Hz IMU / 20 Hz camera) in ONE launch of
    msckf_propagate_batch.  It is HBM/latency-class work, so its roofline is
    HBM: algorithmic bytes per filter = read P[0:21, :] (21 D) + write P11
    (441) and both IMU x cam cross blocks (2 * 21 C), in the context's
    scalar type.  Device time from HIP events on the launch stream; the
    host->device copy of the samples is outside it."""
    B, N = args.batch, args.N
    rng = np.random.default_rng(5)
    n = B * n_samples
    dt = np.full(n, 0.005)
    gyro = 0.2 * rng.standard_normal((n, 3))
    acc = rng.standard_normal((n, 3)) + np.array([0.0, 0.0, 9.81])
    filters = np.arange(B, dtype=np.int32)
    off = (np.arange(B + 1) * n_samples).astype(np.int32)
    ctx.restore()
    ctx.propagate_batch(filters, off, dt, gyro, acc)          # warm-up
    ctx.set_profiling(True)
    t0 = time.perf_counter()
    for _ in range(steps):
        ctx.restore()
        ctx.propagate_batch(filters, off, dt, gyro, acc)
    ctx.sync()
    el = time.perf_counter() - t0
    kms = ctx.kernel_times()["propagate"][0] / steps
    ctx.set_profiling(False)
    ts = 4 if args.dtype == "fp32" else 8
    D, C = 21 + 6 * N, 6 * N
    nbytes = B * (21 * D + 441 + 2 * 21 * C) * ts
    gbs = nbytes / (kms * 1e-3) / 1e9
    return {"value": round(n / (kms * 1e-3), 1), "unit": "IMU samples/s (device time)",
            "wall_samples_per_s": round(n * steps / el, 1), "filters": B, "samples_per_filter": n_samples,
            "D": D, "kernel_ms": round(kms, 4),
            "roofline": {"bound": "hbm", "achieved": round(gbs, 2), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                         "frac": round(gbs / HBM_PEAK_GBS, 5), "bytes_per_launch": nbytes,
                         "traffic": prop_traffic(args.dtype, B, n_samples, D)}}


def prop_traffic(dtype, B, n_samples, D):
    """HBM bytes of one propagation launch (2 x FETCH_SIZE + WRITE_SIZE) from the
    committed rocprofv3 passes (profiles/pmc_propagation.json, tools/gpu/prop_pmc.sh),
    or None if they were taken on another shape."""
    path = os.path.join(ROOT, "profiles", "pmc_propagation.json")
    if not os.path.exists(path):
        return None
    with open(path) as fh:
        d = json.load(fh)
    if (d.get("dtype"), d.get("filters"), d.get("samples_per_filter"), d.get("D")) != (dtype, B, n_samples, D):
        return None
    return d.get("fetch_x2_bytes_per_launch")


def ate_leg():
    """The metric's second half, "ATE RMSE vs ref": the deterministic replay
    (msckf_amd.replay) of the 200-frame synthetic stereo+IMU stream through the
    drop-in MSCKF class (fp64, batch of one), against the reference filter's
    own trajectory on the same stream (tests/golden/sequence_s1.npz, written by
    tools/gen_golden.py from the reference) and against the stream's ground
    truth (SE(3)-aligned)."""
    import msckf_amd
    from msckf_amd.replay import FeatureStream, replay
    from msckf_amd.trajectory import Trajectory, ate
    g = np.load(os.path.join(ROOT, "tests", "golden", "sequence_s1.npz"), allow_pickle=False)
    st = FeatureStream.from_synthetic(synth.make_sequence(int(g["n_frames"]), int(g["seed"])))
    warm = msckf_amd.MSCKF()   # first launches of every kernel outside the timed replay
    replay(warm, FeatureStream.from_synthetic(synth.make_sequence(30, int(g["seed"]))))
    warm.close()
    ev = st.events()           # the front-end's messages, built before the timed region
    flt = msckf_amd.MSCKF()
    t0 = time.perf_counter()
    traj = replay(flt, st, events=ev)
    el = time.perf_counter() - t0
    flt.close()
    ref = Trajectory(g["rec"][:, 0], g["rec"][:, 5:8])
    return {"ate_vs_ref_m": ate(traj, ref, align="none"), "ate_vs_gt_m": round(ate(traj, st.gt), 5),
            "frames": len(traj), "frames_per_s": round(len(traj) / el, 1),
            "sequence": "synthetic stereo+IMU stream s1 (%d frames, 200 Hz IMU), reference trajectory from "
                        "tests/golden/sequence_s1.npz; fp64, host loop + one filter per call; frames_per_s: the filter's "
                        "imu/feature callbacks on prebuilt messages, after a 30-frame warm-up" % len(traj)}


def gather_devices(grp, mine):
    """Every rank's (device index, PCI bus id), in rank order; the replicas
    must sit on distinct GPUs (one process per GPU)."""
    devs = grp.all_gather({"rank": grp.rank, "local_rank": grp.local_rank, "device": mine[0], "pci_bus_id": mine[1]})
    if grp.rank == 0 and len({d["pci_bus_id"] for d in devs}) != len(devs):
        raise SystemExit("bench.py: replicas share a GPU: %s" % devs)
    return devs


def stub_main(args, grp):
    """--stub (tests only): the launch / barrier / max-over-ranks path with a
    CPU stand-in for a step (rank r sleeps 2 (r + 1) ms per step) and for the
    device (index = local rank, bus id 'stub:<local rank>')."""
    devs = gather_devices(grp, (grp.local_rank, "stub:%d" % grp.local_rank))
    cpu = None
    if grp.rank == 0 and not args.no_cpu:
        cpu = {"value": None, "unit": "updates/s", "cores": 1, "kind": "port", "sample": "stub (not a measurement)"}
    grp.barrier()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        time.sleep(0.002 * (grp.rank + 1))
    grp.barrier()
    el = grp.max_over_ranks(time.perf_counter() - t0)
    if grp.rank == 0:
        print(json.dumps({"metric": metric_name(args), "value": replicas.whole_job_rate(args.batch, grp.world,
                                                                                      args.steps, el),
                          "unit": "updates/s", "n_gpus": grp.world, "steps": args.steps, "warmup": args.warmup,
                          "ms_per_step": round(el / args.steps * 1e3, 3), "data": "stub (no GPU, not a measurement)",
                          "ranks_seconds_max": el, "devices": devs, "cpu_baseline": cpu}), flush=True)


def main():
    args = parse()
    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        # one process per GPU; this parent never initialises the GPU
        sys.exit(replicas.spawn([os.path.abspath(__file__)] + sys.argv[1:], args.gpus))
    grp = replicas.init()
    if grp.world != args.gpus:
        raise SystemExit("bench.py: --gpus %d but the launcher started %d rank(s)" % (args.gpus, grp.world))
    if args.stub:
        stub_main(args, grp)
        grp.close()
        return
    rank = grp.rank
    dtype = np.float32 if args.dtype == "fp32" else np.float64
    probs = make_problems(args, rank, min(args.unique, args.batch))
    cpu, refs = None, []
    if rank == 0 and not args.no_cpu:   # before this process initialises the GPU (any world size)
        cpu, refs = cpu_baseline(args, probs[:N_CHECK])

    ctx, feat_off = build_batch(args, probs, dtype, grp.local_rank)
    transport = grp.attach_rccl(ctx.device_info()[0], collective_timeout_s=args.rccl_timeout)   # barriers / max / gathers over RCCL from here on
    devs = gather_devices(grp, ctx.device_info())
    el, times, timed = timed_update(ctx, args, grp)
    value = replicas.whole_job_rate(args.batch, grp.world, args.steps, el)
    acc, gam, pw, valid, rows = ctx.batch_results()
    fl = flops_model(probs, args.batch, acc, valid, feat_off)
    out = {
        "metric": metric_name(args), "value": round(value, 2), "unit": "updates/s", "n_gpus": grp.world,
        "steps": args.steps, "warmup": args.warmup, "ms_per_step": round(el / args.steps * 1e3, 3),
        "higher_is_better": True, "scaling": "weak", "vs_baseline": None,
        "dtype": "f32/f64" if args.dtype == "fp32" else "f64",
        "data": "synthetic (SURVEY.md 8(d) generator: %d distinct problems tiled over %d filters per GPU)"
                % (len(probs), args.batch),
        "config": {"workload": "batched EKF measurement update, %d cam-states x %d features, %d filters/GPU, "
                               "triangulation + jacobian + gating + information assembly + Kalman, no row cap"
                               % (args.N, args.F, args.batch),
                   "cam_states": args.N, "features": args.F, "filters_per_gpu": args.batch,
                   "stacked_rows_mean": float(np.mean(rows)), "parallelism": "replicas%d" % grp.world},
        "devices": devs,
        "replicas": transport,
        "roofline": roofline_of(timed, fl, args, args.dtype),
        # per-stage HIP-event times of the profiled pass before the timed region
        "kernel_ms_per_step": {k: round(v[0] / args.steps, 3) for k, v in sorted(times.items(), key=lambda kv: -kv[1][0])},
        "canonical_gflop_per_update": round(fl["canonical"] / args.batch / 1e9, 4),
    }
    if refs:
        out["accuracy"] = accuracy(ctx, refs, acc, feat_off)
    if cpu is not None:
        out["cpu_baseline"] = cpu
    out["without_triangulation"] = no_triangulation_leg(ctx, args, grp)
    if not args.no_prop:
        out["propagation"] = propagation_leg(ctx, args)
    ctx.close()
    if args.dtype == "fp32" and not args.no_fp64:
        out["fp64"] = fp64_leg(args, grp, probs, refs)
    if rank == 0 and not args.no_ate:
        out["ate"] = ate_leg()
    if rank == 0:
        print(json.dumps(out), flush=True)
    grp.close()


if __name__ == "__main__":
    main()
