"""GPU: the replica transport over RCCL (include/msckf_replicas.h), world
size 1 on the box's one GPU -- communicator bring-up, all-reduce (sum / max),
all-gather and ncclCommCount through the C-ABI, and a ReplicaGroup routing its
barrier / max / gather over it.  (World sizes > 1 run in the driver's
multi-GPU bench; the launch logic is covered on CPU by test_replicas.py.)"""
import numpy as np
import pytest

from msckf_amd import replicas
from msckf_amd._lib import Context
from msckf_amd import FilterConfig

pytestmark = pytest.mark.gpu


def test_rccl_world1_collectives():
    ctx = Context(FilterConfig(), n_filters=1, n_cam_capacity=4)   # selects the device, as bench.py does
    dev = ctx.device_info()[0]
    comm = replicas.RcclComm(replicas.RcclComm.unique_id(), 1, 0, dev, timeout_s=60.0)
    try:
        assert comm.count() == (1, 0)
        assert comm.allreduce(2.5, "sum") == 2.5
        assert comm.allreduce(-7.0, "max") == -7.0
        assert comm.allgather_bytes(b"abc\x00xyz") == [b"abc\x00xyz"]
        comm.set_timeout(5.0)
        assert comm.allreduce(1.0, "sum") == 1.0
        with pytest.raises(RuntimeError):
            comm.set_timeout(0.0)
    finally:
        comm.close()   # finalize polled to completion, then destroy (raises if the teardown was aborted)
        ctx.close()


def test_replica_group_over_rccl():
    ctx = Context(FilterConfig(), n_filters=1, n_cam_capacity=4)
    grp = replicas.ReplicaGroup(rank=0, world=1, local_rank=0)
    try:
        tr = grp.attach_rccl(ctx.device_info()[0], collective_timeout_s=120.0)
        assert tr == {"transport": "rccl", "rccl_comm_count": [1], "rccl_ranks": [0],
                      "collective_timeout_s": 120.0}, tr
        grp.barrier()
        assert grp.max_over_ranks(3.25) == 3.25
        assert grp.sum_over_ranks(1.5) == 1.5
        assert grp.all_gather({"rank": 0, "pci_bus_id": "0000:05:00.0"}) == [{"rank": 0, "pci_bus_id": "0000:05:00.0"}]
    finally:
        grp.close()
        ctx.close()
