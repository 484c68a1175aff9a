"""Multi-GPU layout of the throughput path: independent replicas.

The EKF update does not shard: one filter's covariance is a
few hundred KB and every stage of its update is a chain of small dependent
factorisations, so there is no data-parallel exchange to make.  N GPUs run N
independent batches of filters, one process per GPU.  The ranks exchange only
control: the start / stop barriers of the timed region and the max (or sum)
of a float.  No collective touches the data path.  On GPUs the control
messages travel over RCCL (xGMI between the node's GPUs; include/
msckf_replicas.h, librccl opened at run time, no PyTorch): ``attach_rccl``
makes one communicator per rank, its unique id handed out over a host TCP
hub (stdlib sockets) that also carries everything when there is no GPU (the
--stub tests) or when RCCL cannot be brought up (then every rank falls back
together and the bench line says why).

Launch modes (both one process per GPU, RANK / LOCAL_RANK / WORLD_SIZE in the
environment):
* ``spawn(argv, n)`` -- the parent process (which never touches the GPU)
  starts n children, hosts the hub and passes its address in MSCKF_HUB;
* an external launcher (``python -m torch.distributed.run --nproc-per-node N``
  on one node, as the driver runs bench.py) -- rank 0 hosts the hub and
  publishes its port in a rendezvous file keyed by MASTER_PORT and the
  launcher's pid (every rank's parent), under the temp directory.
"""
import json
import os
import socket
import subprocess
import sys
import tempfile
import threading
import time
from dataclasses import dataclass
from typing import List, Optional

HUB_ENV = "MSCKF_HUB"
TIMEOUT_S = 900.0


def _send(sock, obj):
    sock.sendall((json.dumps(obj) + "\n").encode())


class _Lines:
    """Newline-delimited JSON reader over a socket."""

    def __init__(self, sock):
        self.sock, self.buf = sock, b""

    def read(self):
        while b"\n" not in self.buf:
            chunk = self.sock.recv(65536)
            if not chunk:
                raise ConnectionError("replica hub: peer closed the connection")
            self.buf += chunk
        line, self.buf = self.buf.split(b"\n", 1)
        return json.loads(line)


class Hub:
    """Serves ``world`` ranks: each round every rank sends {op, v}; once all
    have arrived the hub replies to each with the reduction (max / sum /
    barrier).  All ranks issue the same collectives in the same order."""

    def __init__(self, world: int, host: str = "127.0.0.1", port: int = 0):
        self.world = world
        self.srv = socket.socket(socket.AF_INET, socket.SOCK_STREAM)
        self.srv.setsockopt(socket.SOL_SOCKET, socket.SO_REUSEADDR, 1)
        self.srv.bind((host, port))
        self.srv.listen(world)
        self.srv.settimeout(TIMEOUT_S)
        self.address = "%s:%d" % self.srv.getsockname()[:2]
        self.error: Optional[BaseException] = None
        self.thread = threading.Thread(target=self._run, daemon=True)
        self.thread.start()

    def _run(self):
        conns = {}
        try:
            while len(conns) < self.world:
                c, _ = self.srv.accept()
                c.settimeout(TIMEOUT_S)
                r = _Lines(c)
                hello = r.read()
                conns[int(hello["rank"])] = (c, r)
            order = [conns[k] for k in sorted(conns)]
            while True:
                msgs = [r.read() for _, r in order]
                ops = {m["op"] for m in msgs}
                if len(ops) != 1:
                    raise RuntimeError("replica hub: ranks disagree on the collective: %s" % sorted(ops))
                op = ops.pop()
                if op == "gather":   # every rank's JSON value, in rank order
                    res = [m.get("v") for m in msgs]
                else:
                    vals = [float(m.get("v", 0.0)) for m in msgs]
                    res = {"max": max(vals), "sum": sum(vals)}.get(op, 0.0)
                for c, _ in order:
                    _send(c, {"v": res})
                if op == "close":
                    break
        except BaseException as e:   # surfaced to the ranks as a closed connection
            self.error = e
        finally:
            for c, _ in conns.values():
                c.close()
            self.srv.close()


class RcclComm:
    """One RCCL communicator of this rank (msckf_rccl_*, include/
    msckf_replicas.h): all-reduce of doubles (sum / max, a barrier when the
    caller needs one) and all-gather of bytes, on the device the rank runs on."""

    def __init__(self, uid: bytes, world: int, rank: int, device: int, timeout_s: float = 60.0):
        import ctypes as C
        from . import _lib
        self._C, self._L = C, _lib.load_library()
        self.world, self.rank = world, rank
        h = C.c_void_p()
        buf = (C.c_uint8 * _lib.RCCL_ID_BYTES).from_buffer_copy(uid)
        rc = self._L.msckf_rccl_init(buf, world, rank, device, timeout_s, C.byref(h))
        if rc != 0:
            raise RuntimeError("msckf_rccl_init: %s (rc=%d)" % (self._L.msckf_rccl_last_error().decode(), rc))
        self._h = h

    @staticmethod
    def unique_id() -> bytes:
        import ctypes as C
        from . import _lib
        L = _lib.load_library()
        buf = (C.c_uint8 * _lib.RCCL_ID_BYTES)()
        rc = L.msckf_rccl_unique_id(buf)
        if rc != 0:
            raise RuntimeError("msckf_rccl_unique_id: %s (rc=%d)" % (L.msckf_rccl_last_error().decode(), rc))
        return bytes(buf)

    def _check(self, rc, what):
        if rc != 0:
            raise RuntimeError("%s: %s (rc=%d)" % (what, self._L.msckf_rccl_last_error().decode(), rc))

    def allreduce(self, x: float, op: str) -> float:
        C = self._C
        v = (C.c_double * 1)(float(x))
        self._check(self._L.msckf_rccl_allreduce(self._h, v, 1, 1 if op == "max" else 0), "msckf_rccl_allreduce")
        return float(v[0])

    def allgather_bytes(self, b: bytes) -> List[bytes]:
        C = self._C
        n = len(b)
        src = C.create_string_buffer(b, n)
        dst = C.create_string_buffer(n * self.world)
        self._check(self._L.msckf_rccl_allgather(self._h, src, n, dst), "msckf_rccl_allgather")
        raw = dst.raw
        return [raw[k * n:(k + 1) * n] for k in range(self.world)]

    def set_timeout(self, seconds: float):
        self._check(self._L.msckf_rccl_set_timeout(self._h, float(seconds)), "msckf_rccl_set_timeout")

    def count(self):
        C = self._C
        n, r = C.c_int32(), C.c_int32()
        self._check(self._L.msckf_rccl_count(self._h, C.byref(n), C.byref(r)), "msckf_rccl_count")
        return n.value, r.value

    def close(self):
        if self._h is not None:
            h, self._h = self._h, None
            self._check(self._L.msckf_rccl_destroy(h), "msckf_rccl_destroy")


@dataclass
class ReplicaGroup:
    rank: int
    world: int
    local_rank: int
    _sock: Optional[socket.socket] = None
    _lines: Optional[_Lines] = None
    _hub: Optional[Hub] = None
    _rdzv: Optional[str] = None
    _rccl: Optional[RcclComm] = None
    transport: str = "none (one rank)"

    def _hub_call(self, op, v=0.0):
        if self._sock is None:
            return float(v)
        _send(self._sock, {"op": op, "v": float(v)})
        return float(self._lines.read()["v"])

    def _hub_gather(self, obj):
        if self._sock is None:
            return [obj]
        _send(self._sock, {"op": "gather", "v": obj})
        return list(self._lines.read()["v"])

    def _rccl_do(self, what, fn, *a):
        # A collective that fails after the communicator came up ends the job
        # with the transport named: the ranks cannot agree to fall back to the
        # hub without a working collective, and a half-finished timed region
        # must not print a line.
        try:
            return fn(*a)
        except RuntimeError as e:
            raise RuntimeError("replica %s over rccl failed on rank %d of %d: %s"
                               % (what, self.rank, self.world, e)) from e

    def _call(self, op, v=0.0):
        if self._rccl is not None:
            return self._rccl_do(op, self._rccl.allreduce, v, "max" if op == "max" else "sum")
        return self._hub_call(op, v)

    def attach_rccl(self, device: int, timeout_s: float = 60.0, collective_timeout_s: float = 1800.0) -> dict:
        """Brings up RCCL on ``device`` for this group's collectives (the
        north star's multi-GPU transport).  Rank 0 makes the unique id and
        hands it out over the hub; every rank then reports over the hub
        whether its communicator came up, and unless all did, all of them stay
        on the hub.  ``timeout_s`` bounds the bring-up; ``collective_timeout_s``
        every later collective (generous: the ranks wait in a barrier while
        rank 0 runs its accuracy and ATE legs).  Returns the transport record
        for the bench line: the transport used and each rank's ncclCommCount
        (or the reason)."""
        uid, err = None, None
        if self.rank == 0:
            try:
                uid = RcclComm.unique_id().hex()
            except Exception as e:   # noqa: BLE001 -- reported, then the hub carries on
                err = str(e)
        uid = self._hub_gather(uid)[0]
        comm = None
        if uid is not None:
            try:
                comm = RcclComm(bytes.fromhex(uid), self.world, self.rank, device, timeout_s)
            except Exception as e:   # noqa: BLE001
                err = str(e)
        oks = self._hub_gather(comm is not None)
        errs = self._hub_gather(err)
        if not all(oks):
            if comm is not None:
                try:   # this rank came up but another did not: the hub carries on for all of them
                    comm.close()
                except RuntimeError as e:   # an aborted teardown is recorded, not raised
                    errs = errs + ["rank %d teardown: %s" % (self.rank, e)]
            self.transport = "tcp-hub (rccl unavailable: %s)" % next(e for e in errs if e)
            return {"transport": self.transport}
        comm.set_timeout(collective_timeout_s)
        self._rccl = comm
        self.transport = "rccl"
        counts = [json.loads(b.rstrip(b"\0").decode()) for b in
                  self._rccl_do("gather", self._rccl.allgather_bytes,
                                json.dumps(list(comm.count())).encode().ljust(32, b"\0"))]
        rec = {"transport": "rccl", "rccl_comm_count": [c[0] for c in counts],
               "rccl_ranks": [c[1] for c in counts], "collective_timeout_s": collective_timeout_s}
        if self.world > 1:
            rec["note"] = ("world > 1 over RCCL runs only in the driver's multi-GPU bench; "
                           "this repo's own tests cover world 1 on the GPU and world 2 over the hub")
        return rec

    def barrier(self):
        self._call("barrier")

    def max_over_ranks(self, x: float) -> float:
        """MAX over ranks of one float (the timed region's elapsed seconds)."""
        return self._call("max", x)

    def sum_over_ranks(self, x: float) -> float:
        """SUM over ranks of one float (e.g. frames processed by every rank)."""
        return self._call("sum", x)

    def all_gather(self, obj):
        """Every rank's JSON-serialisable ``obj``, in rank order (control
        data only: e.g. the device each replica ran on)."""
        if self._rccl is not None:
            b = json.dumps(obj).encode()
            n = int(self._rccl_do("gather", self._rccl.allreduce, len(b), "max"))
            return [json.loads(x.rstrip(b"\0").decode())
                    for x in self._rccl_do("gather", self._rccl.allgather_bytes, b.ljust(n, b"\0"))]
        return self._hub_gather(obj)

    def close(self):
        # the hub, the socket and the rendezvous file are released even when the
        # RCCL teardown raises (an aborted ncclCommFinalize, rc -4): a stale
        # rendezvous file keyed by MASTER_PORT and ppid would be picked up by a
        # later run
        try:
            if self._rccl is not None:
                comm, self._rccl = self._rccl, None
                comm.close()
        finally:
            try:
                if self._sock is not None:
                    self._hub_call("close")
            finally:
                if self._sock is not None:
                    self._sock.close()
                    self._sock = None
                if self._hub is not None:
                    self._hub.thread.join(timeout=30)
                if self._rdzv and os.path.exists(self._rdzv):
                    os.unlink(self._rdzv)


def _rdzv_path():
    key = "%s_%d" % (os.environ.get("MASTER_PORT", "0"), os.getppid())
    return os.path.join(tempfile.gettempdir(), "msckf_replicas_%s.hub" % key)


def _connect(address: str, rank: int):
    host, port = address.rsplit(":", 1)
    deadline = time.time() + 120
    while True:
        try:
            s = socket.create_connection((host, int(port)), timeout=TIMEOUT_S)
            break
        except OSError:
            if time.time() > deadline:
                raise
            time.sleep(0.1)
    _send(s, {"rank": rank})
    return s


def init() -> ReplicaGroup:
    """One process per GPU; RANK / LOCAL_RANK / WORLD_SIZE from the
    environment.  World size 1 needs no hub."""
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", str(rank)))
    grp = ReplicaGroup(rank, world, local)
    if world <= 1:
        return grp
    address = os.environ.get(HUB_ENV)
    if not address:   # external launcher: rank 0 hosts the hub, the others find it on disk
        path = _rdzv_path()
        if rank == 0:
            grp._hub = Hub(world, os.environ.get("MASTER_ADDR", "127.0.0.1"))
            address = grp._hub.address
            tmp = path + ".%d.tmp" % os.getpid()
            with open(tmp, "w") as fh:
                fh.write(address)
            os.replace(tmp, path)
            grp._rdzv = path
        else:   # wait for a file written by THIS job's rank 0 (not a stale one of a dead job)
            t0 = time.time()
            while not (os.path.exists(path) and os.path.getmtime(path) > t0 - 60):
                if time.time() > t0 + 120:
                    raise TimeoutError("replica hub rendezvous file %s never appeared" % path)
                time.sleep(0.05)
            with open(path) as fh:
                address = fh.read().strip()
    grp._sock = _connect(address, rank)
    grp._lines = _Lines(grp._sock)
    return grp


def spawn(argv: List[str], n: int, env_extra: Optional[dict] = None) -> int:
    """Runs ``python argv...`` as n ranks (one per GPU) from a parent that
    never initialises the GPU; the parent hosts the hub.  Returns the first
    non-zero exit code of the ranks (0 if all succeed).  The children are
    polled: the first one to fail ends the job -- the others (blocked in a
    hub read or its accept) are terminated instead of waiting out the hub's
    timeout."""
    hub = Hub(n)
    procs = []
    for r in range(n):
        env = dict(os.environ)
        env.update(env_extra or {})
        env.update(RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n), LOCAL_WORLD_SIZE=str(n),
                   MASTER_ADDR="127.0.0.1")
        env[HUB_ENV] = hub.address
        procs.append(subprocess.Popen([sys.executable] + list(argv), env=env))
    first_bad = 0
    while True:
        codes = [p.poll() for p in procs]
        bad = [c for c in codes if c not in (None, 0)]
        if bad and not first_bad:
            first_bad = bad[0]
            for p in procs:
                if p.poll() is None:
                    p.terminate()
            try:
                hub.srv.close()
            except OSError:
                pass
        if all(c is not None for c in codes):
            break
        time.sleep(0.05)
    for p in procs:
        p.wait()
    hub.thread.join(timeout=5 if first_bad else 30)
    return first_bad or next((c for c in codes if c != 0), 0)


def problem_seeds(rank: int, unique: int) -> List[int]:
    """Seeds of the distinct synthetic problems a replica tiles over its
    batch: disjoint across ranks, so N replicas process N different batches."""
    return [1000 * rank + u for u in range(unique)]


def shard(items: list, rank: int, world: int) -> list:
    """The independent units (sequences, filter batches) a rank owns:
    round-robin, so every unit runs on exactly one rank (SURVEY config 4:
    sequences one per GPU, no cross-GPU state)."""
    return list(items[rank::world])


def whole_job_rate(filters_per_rank: int, world: int, steps: int, max_elapsed_s: float) -> float:
    """Updates/s of the whole job: every rank's updates over the slowest rank's time."""
    return filters_per_rank * world * steps / max_elapsed_s
