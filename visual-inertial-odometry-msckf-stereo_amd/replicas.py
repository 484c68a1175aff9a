"""Multi-GPU layout of the throughput path: independent replicas.

The EKF update does not shard: one filter's covariance is a
few hundred KB and every stage of its update is a chain of small dependent
factorisations, so there is no data-parallel exchange to make.  N GPUs run N
independent batches of filters, one process per GPU (torch.distributed.run);
the process group is used only for the start/stop barriers of the timed
region and for the max-over-ranks of the elapsed time.  No collective touches
the data path.

The helpers take the backend as a parameter so the same code runs over RCCL
("nccl") on the GPU box and over gloo on CPU in the tests.
"""
import os
from dataclasses import dataclass
from typing import List, Optional


@dataclass
class ReplicaGroup:
    rank: int
    world: int
    local_rank: int
    dist: Optional[object]   # torch.distributed when world > 1
    device: str              # tensor device used for the reductions

    def barrier(self):
        if self.dist is not None:
            self.dist.barrier()

    def max_over_ranks(self, x: float) -> float:
        """MAX all-reduce of one float (the timed region's elapsed seconds)."""
        if self.dist is None:
            return float(x)
        import torch
        t = torch.tensor([float(x)], dtype=torch.float64, device=self.device)
        self.dist.all_reduce(t, op=self.dist.ReduceOp.MAX)
        return float(t.item())

    def sum_over_ranks(self, x: float) -> float:
        """SUM all-reduce of one float (e.g. frames processed by every rank)."""
        if self.dist is None:
            return float(x)
        import torch
        t = torch.tensor([float(x)], dtype=torch.float64, device=self.device)
        self.dist.all_reduce(t, op=self.dist.ReduceOp.SUM)
        return float(t.item())

    def close(self):
        if self.dist is not None:
            self.dist.destroy_process_group()


def init(backend: str = "nccl") -> ReplicaGroup:
    """One process per GPU; RANK / LOCAL_RANK / WORLD_SIZE / MASTER_* from the
    environment (torch.distributed.run sets them).  World size 1 needs no
    process group."""
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", str(rank)))
    if world <= 1:
        return ReplicaGroup(rank, 1, local, None, "cpu")
    import torch
    import torch.distributed as dist
    device = "cpu"
    if backend == "nccl":
        torch.cuda.set_device(local)
        device = "cuda"
    dist.init_process_group(backend)
    return ReplicaGroup(rank, world, local, dist, device)


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
