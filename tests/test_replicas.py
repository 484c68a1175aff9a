"""N > 1 path of bench.py: independent replicas over torch.distributed.

Runs the replica helpers (msckf_amd/replicas.py) at world size 2 over gloo on
CPU: the barrier, the MAX all-reduce of the timing, disjoint problem seeds and
the whole-job rate -- the same code bench.py runs over RCCL on the GPUs."""
import os
import socket
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import msckf_pkg  # noqa: E402,F401
from msckf_amd import replicas  # noqa: E402


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank),
                      LOCAL_RANK=str(rank), WORLD_SIZE=str(world))
    try:
        from msckf_amd import synth
        grp = replicas.init("gloo")
        seeds = replicas.problem_seeds(grp.rank, 3)
        # a replica's work is its own batch of synthetic problems
        prob = synth.make_update_problem(6, 12, seed=seeds[0])
        grp.barrier()
        el = 0.5 + grp.rank            # rank 1 is the slow one
        mx = grp.max_over_ranks(el)
        rate = replicas.whole_job_rate(64, grp.world, 10, mx)
        mine = replicas.shard(list(range(11)), grp.rank, grp.world)   # 11 sequences over the ranks
        total = grp.sum_over_ranks(len(mine))
        grp.barrier()
        q.put((grp.rank, grp.world, seeds, float(prob.P.sum()), mx, rate, mine, total))
        grp.close()
    except Exception as e:   # surface the failure in the parent
        q.put((rank, "error", repr(e)))


def test_single_process_needs_no_group(monkeypatch):
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK"):
        monkeypatch.delenv(k, raising=False)
    grp = replicas.init("nccl")      # world 1: no process group, no GPU touched
    assert grp.world == 1 and grp.dist is None
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


@pytest.mark.timeout(120)
def test_gloo_world2_replicas():
    import torch.multiprocessing as mp
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = [q.get(timeout=100) for _ in procs]
    for p in procs:
        p.join(timeout=30)
        assert p.exitcode == 0
    for r in res:
        assert r[1] != "error", r
    res.sort()
    (r0, w0, s0, p0, m0, v0, sh0, t0), (r1, w1, s1, p1, m1, v1, sh1, t1) = res
    assert sorted(sh0 + sh1) == list(range(11)) and not (set(sh0) & set(sh1))   # each sequence on one rank
    assert t0 == t1 == 11
    assert (r0, r1) == (0, 1) and w0 == w1 == 2
    assert not (set(s0) & set(s1))          # different problems per replica
    assert p0 != p1
    assert m0 == m1 == pytest.approx(1.5)   # both ranks see the slowest rank's time
    assert v0 == v1 == pytest.approx(64 * 2 * 10 / 1.5)
