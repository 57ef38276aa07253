"""One-process-per-GPU helpers (torch.distributed: RCCL on GPUs, gloo on CPU).

The reference's only parallelism is an R PSOCK pool over the outer cluster
index (R/reclusterDEConsensusFast.R:61-65,384).  Here each rank owns one
MI355X and ONE job is sharded over the ranks (``sharded.py``):
gene row-blocks for the DE, cell blocks for the PCA, packed-column slices for
the distance.  ``shard_range`` / ``weighted_range`` are the contiguous splits.
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
    backend: str = ""

    @property
    def active(self) -> bool:
        return self.world > 1

    def barrier(self):
        if self.active:
            self.dist.barrier()

    def _host_staged(self, tensor) -> bool:
        # gloo runs its collectives on host memory: device tensors go through a copy
        return self.backend == "gloo" and getattr(tensor, "is_cuda", False)

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
            if self._host_staged(tensor):
                h = tensor.cpu()
                self.dist.all_reduce(h, op=self.dist.ReduceOp.SUM)
                tensor.copy_(h)
            else:
                self.dist.all_reduce(tensor, op=self.dist.ReduceOp.SUM)
        return tensor

    def all_reduce_min_(self, tensor):
        """In-place element-wise minimum over ranks."""
        if self.active:
            if self._host_staged(tensor):
                h = tensor.cpu()
                self.dist.all_reduce(h, op=self.dist.ReduceOp.MIN)
                tensor.copy_(h)
            else:
                self.dist.all_reduce(tensor, op=self.dist.ReduceOp.MIN)
        return tensor

    def broadcast_(self, tensor, src: int = 0):
        """In-place copy of rank ``src``'s tensor to every rank."""
        if self.active:
            if self._host_staged(tensor):
                h = tensor.cpu()
                self.dist.broadcast(h, src=src)
                tensor.copy_(h)
            else:
                self.dist.broadcast(tensor, src=src)
        return tensor

    def all_gather_cat(self, tensor):
        """The ranks' equal-sized 1-D tensors concatenated in rank order."""
        if not self.active:
            return tensor
        torch = self.torch
        src = tensor.cpu() if self._host_staged(tensor) else tensor
        if self.backend == "nccl":
            out = torch.empty(self.world * src.numel(), dtype=src.dtype, device=src.device)
            self.dist.all_gather_into_tensor(out, src)
        else:
            parts = [torch.empty_like(src) for _ in range(self.world)]
            self.dist.all_gather(parts, src)
            out = torch.cat(parts)
        return out.to(tensor.device) if out.device != tensor.device else out

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
    return Dist(rank, world, local, torch, tdist, device, backend)


def shard_range(n: int, rank: int, world: int) -> tuple[int, int]:
    """Contiguous balanced block [lo, hi) of n items for ``rank``."""
    base, rem = divmod(n, world)
    lo = rank * base + min(rank, rem)
    return lo, lo + base + (1 if rank < rem else 0)


def weighted_range(weights, rank: int, world: int) -> tuple[int, int]:
    """Contiguous block [lo, hi) of the items whose cumulative weight falls in
    rank's equal share (e.g. genes balanced by their stored values)."""
    import numpy as np
    w = np.asarray(weights, np.float64)
    n = len(w)
    if n == 0 or world <= 1:
        return (0, n) if rank == 0 else (n, n)
    c = np.concatenate([[0.0], np.cumsum(w)])
    tot = c[-1]
    if tot <= 0:
        return shard_range(n, rank, world)

    def cut(r):
        if r <= 0:
            return 0
        if r >= world:
            return n
        return int(np.searchsorted(c, tot * r / world, side="left"))

    return cut(rank), cut(rank + 1)


def job_seed(base_seed: int, rank: int) -> int:
    """--mode jobs (weak scaling): every rank runs its own job of the benchmark shape."""
    return base_seed + 1000 * rank
