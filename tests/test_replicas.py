"""N > 1 path of bench.py: independent replicas, one process per GPU, with a
host TCP hub for the control messages (msckf_amd/replicas.py, no PyTorch).

CPU only: the hub's barrier / MAX / SUM at world size 2, bench.py spawning two
ranks itself (``--gpus 2``) and the same bench.py under the driver's external
launcher (torch.distributed.run, rendezvous through the hub file), both with
``--stub`` in place of the device context."""
import json
import os
import socket
import subprocess
import sys
import textwrap

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import msckf_pkg  # noqa: E402,F401
from msckf_amd import replicas  # noqa: E402

PKG_DIR = os.path.join(ROOT, "visual-inertial-odometry-msckf-stereo_amd")


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _json_line(stdout):
    lines = [l for l in stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, stdout
    return json.loads(lines[0])


def test_single_process_needs_no_hub(monkeypatch):
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK", replicas.HUB_ENV):
        monkeypatch.delenv(k, raising=False)
    grp = replicas.init()      # world 1: no hub, no socket
    assert grp.world == 1 and grp._sock is None
    assert grp.max_over_ranks(1.25) == 1.25
    grp.barrier()
    grp.close()


def test_problem_seeds_disjoint():
    a, b = set(replicas.problem_seeds(0, 32)), set(replicas.problem_seeds(1, 32))
    assert len(a) == 32 and not (a & b)


def test_shard_round_robin():
    parts = [replicas.shard(list(range(11)), r, 8) for r in range(8)]
    assert sorted(sum(parts, [])) == list(range(11))
    assert [len(p) for p in parts] == [2, 2, 2, 1, 1, 1, 1, 1]


def test_whole_job_rate():
    assert replicas.whole_job_rate(2048, 8, 10, 0.2) == pytest.approx(2048 * 8 * 10 / 0.2)


_WORKER = textwrap.dedent("""
    import json, sys
    sys.path.insert(0, %r)
    import msckf_pkg
    from msckf_amd import replicas
    grp = replicas.init()
    grp.barrier()
    mx = grp.max_over_ranks(0.5 + grp.rank)          # rank 1 is the slow one
    mine = replicas.shard(list(range(11)), grp.rank, grp.world)
    total = grp.sum_over_ranks(len(mine))
    grp.barrier()
    print(json.dumps({"rank": grp.rank, "world": grp.world, "max": mx, "total": total, "mine": mine}))
    grp.close()
""") % ROOT


@pytest.mark.timeout(120)
def test_hub_world2_collectives():
    """replicas.spawn: two ranks, the parent hosting the hub."""
    script = os.path.join(ROOT, "tests", "_replica_worker.py")
    with open(script, "w") as fh:
        fh.write(_WORKER)
    try:
        out = subprocess.run([sys.executable, "-c",
                              "import sys; sys.path.insert(0, %r); import msckf_pkg; from msckf_amd import replicas; "
                              "sys.exit(replicas.spawn([%r], 2))" % (ROOT, script)],
                             capture_output=True, text=True, timeout=100)
    finally:
        os.unlink(script)
    assert out.returncode == 0, out.stderr
    res = sorted((json.loads(l) for l in out.stdout.splitlines() if l.startswith("{")), key=lambda r: r["rank"])
    assert [r["rank"] for r in res] == [0, 1] and all(r["world"] == 2 for r in res)
    assert all(r["max"] == pytest.approx(1.5) for r in res)       # both see the slowest rank's value
    assert all(r["total"] == 11 for r in res)
    assert sorted(res[0]["mine"] + res[1]["mine"]) == list(range(11))


@pytest.mark.timeout(120)
def test_bench_spawns_ranks():
    """bench.py --gpus 2 starts its own two ranks (the parent never touches a
    GPU) and reports n_gpus = 2 with the slowest rank's time."""
    out = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--no-cpu", "--stub",
                          "--steps", "5"], capture_output=True, text=True, timeout=100,
                         env={k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")})
    assert out.returncode == 0, out.stderr
    line = _json_line(out.stdout)
    assert line["n_gpus"] == 2
    assert line["ms_per_step"] >= 4.0              # rank 1 sleeps 4 ms per step
    assert line["value"] == pytest.approx(2048 * 2 * 5 / line["ranks_seconds_max"])
    # every replica's device is in the line, one per rank, all distinct
    assert [d["rank"] for d in line["devices"]] == [0, 1]
    assert [d["pci_bus_id"] for d in line["devices"]] == ["stub:0", "stub:1"]


@pytest.mark.timeout(120)
def test_bench_keeps_cpu_baseline_at_world2():
    """Rank 0 computes the CPU baseline before it touches the GPU whatever
    the world size, so an N > 1 line carries it too."""
    out = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--stub", "--steps", "2"],
                         capture_output=True, text=True, timeout=100,
                         env={k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")})
    assert out.returncode == 0, out.stderr
    line = _json_line(out.stdout)
    assert line["n_gpus"] == 2 and line["cpu_baseline"] is not None


_FAILING = textwrap.dedent("""
    import sys, time
    sys.path.insert(0, %r)
    import msckf_pkg
    from msckf_amd import replicas
    grp = replicas.init()
    if grp.rank == 1:
        sys.exit(3)          # dies before its first collective
    grp.barrier()            # rank 0 would wait here for the hub's whole timeout
""") % ROOT


@pytest.mark.timeout(60)
def test_spawn_fails_fast_when_a_rank_dies():
    script = os.path.join(ROOT, "tests", "_replica_failing.py")
    with open(script, "w") as fh:
        fh.write(_FAILING)
    try:
        import time
        t0 = time.time()
        out = subprocess.run([sys.executable, "-c",
                              "import sys; sys.path.insert(0, %r); import msckf_pkg; from msckf_amd import replicas; "
                              "sys.exit(replicas.spawn([%r], 2))" % (ROOT, script)],
                             capture_output=True, text=True, timeout=50)
        el = time.time() - t0
    finally:
        os.unlink(script)
    assert out.returncode != 0      # rank 1's 3, or rank 0's error once the hub drops it
    assert el < 30


@pytest.mark.timeout(180)
def test_bench_under_external_launcher():
    """The driver's launch: torch.distributed.run starts the ranks with
    WORLD_SIZE set; rank 0 hosts the hub and the others find it through the
    rendezvous file."""
    port = _free_port()
    out = subprocess.run([sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
                          "--master-addr", "127.0.0.1", "--master-port", str(port),
                          os.path.join(ROOT, "bench.py"), "--gpus", "2", "--no-cpu", "--stub", "--steps", "5"],
                         capture_output=True, text=True, timeout=170)
    assert out.returncode == 0, out.stderr[-3000:]
    line = _json_line(out.stdout)
    assert line["n_gpus"] == 2 and line["ms_per_step"] >= 4.0
    assert sorted(d["local_rank"] for d in line["devices"]) == [0, 1]


def test_bench_rejects_gpus_mismatch():
    env = dict(os.environ, WORLD_SIZE="1", RANK="0", LOCAL_RANK="0")
    out = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--stub"],
                         capture_output=True, text=True, timeout=60, env=env)
    assert out.returncode != 0 and "--gpus 2" in out.stderr


def test_package_has_no_torch():
    """north_star: no PyTorch in the product -- not even in the replica layer."""
    for dirpath, _, files in os.walk(PKG_DIR):
        for f in files:
            if f.endswith(".py"):
                src = open(os.path.join(dirpath, f)).read()
                assert "import torch" not in src and "from torch" not in src, f
