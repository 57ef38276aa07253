"""One-process-per-GPU helpers (torch.distributed: RCCL on GPUs, gloo on CPU).

The reference's only parallelism is an R PSOCK pool over the outer cluster
index (R/reclusterDEConsensusFast.R:61-65,384).  Here each rank owns one
MI355X.  The benchmark shards whole jobs across ranks (weak scaling, no
data-path collective); RCCL carries only the barrier and the max of the step
time.  ``shard_range`` is the gene row-block split used when one job is
sharded across ranks.
"""
from __future__ import annotations

import os
from dataclasses import dataclass


@dataclass
class Dist:
    rank: int = 0
    world: int = 1
    local_rank: int = 0
    torch: object = None
    dist: object = None
    device: object = None

    @property
    def active(self) -> bool:
        return self.world > 1

    def barrier(self):
        if self.active:
            self.dist.barrier()

    def max_over_ranks(self, value: float) -> float:
        if not self.active:
            return float(value)
        t = self.torch.tensor([float(value)], dtype=self.torch.float64, device=self.device)
        self.dist.all_reduce(t, op=self.dist.ReduceOp.MAX)
        return float(t.item())

    def sum_over_ranks(self, value: float) -> float:
        if not self.active:
            return float(value)
        t = self.torch.tensor([float(value)], dtype=self.torch.float64, device=self.device)
        self.dist.all_reduce(t, op=self.dist.ReduceOp.SUM)
        return float(t.item())

    def all_reduce_sum_(self, tensor):
        """In-place sum over ranks (RCCL over xGMI on GPU tensors, gloo on CPU)."""
        if self.active:
            self.dist.all_reduce(tensor, op=self.dist.ReduceOp.SUM)
        return tensor

    def close(self):
        if self.active:
            self.dist.destroy_process_group()


def init(backend: str | None = None) -> Dist:
    """Read RANK/WORLD_SIZE/LOCAL_RANK (torchrun) and join the process group.
    backend None: "nccl" (RCCL over xGMI) when GPUs are visible, else "gloo"."""
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world <= 1:
        return Dist(rank, world, local)
    os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
    import torch
    import torch.distributed as tdist
    if backend is None:
        backend = "nccl" if torch.cuda.device_count() > 0 else "gloo"
    device = torch.device("cpu")
    if backend == "nccl":
        torch.cuda.set_device(local)
        device = torch.device(f"cuda:{local}")
    elif os.environ.get("SCC_SHARE_GPU"):  # ranks rehearsed on one GPU over gloo
        torch.cuda.set_device(0)
    tdist.init_process_group(backend)
    return Dist(rank, world, local, torch, tdist, device)


def shard_range(n: int, rank: int, world: int) -> tuple[int, int]:
    """Contiguous balanced block [lo, hi) of n items for ``rank``."""
    base, rem = divmod(n, world)
    lo = rank * base + min(rank, rem)
    return lo, lo + base + (1 if rank < rem else 0)


def job_seed(base_seed: int, rank: int) -> int:
    """Weak scaling: every rank runs its own job of the benchmark shape."""
    return base_seed + 1000 * rank
