"""One DE job sharded over the ranks of a process group.

The reference parallelises the pair loop with a PSOCK foreach over the outer
cluster index (R/reclusterDEConsensusFast.R:61-65,359,384).  Here each rank
(one MI355X) holds the whole dataset and runs the per-(pair, gene) stage —
per-cluster statistics, filters, ranks, exact U / ties / p — on its block of
gene rows (``scc_de_run_shard``).  The only exchange is one all-reduce (RCCL
over xGMI) of the shard buffers: they are disjoint and zero elsewhere, so the
int64 sum is the exact union of every rank's cells.  Every rank then runs the
per-pair selection (BH over all genes of the pair, filters, top-N, union) on
the same bits (``scc_de_finish``) and gets the result ``scc_de_run`` gives.
"""
from __future__ import annotations

from . import parallel

_SHARD_KEYS = ("mode", "q_val_thrs", "log_fc_thrs", "min_per_cent", "top_n", "fc_thrs", "mean_scaling_factor",
               "test_all")


def gene_shard(G: int, rank: int, world: int) -> tuple[int, int]:
    """Gene rows of ``rank``: contiguous, equal-sized blocks."""
    return parallel.shard_range(G, rank, world)


def de_sharded(eng, ds, code, K, dist: parallel.Dist, device, fetch="rows", **params):
    """The DE of one job over all ranks of ``dist``; every rank returns the same
    DeResult.  ``device``: the torch device of this rank's engine."""
    import torch

    shard_kw = {k: v for k, v in params.items() if k in _SHARD_KEYS}
    lo, hi = gene_shard(ds.G, dist.rank, dist.world)
    nbytes = eng.de_shard_bytes(K, ds.G)
    buf = torch.empty(nbytes // 8, dtype=torch.int64, device=device)
    eng.de_run_shard(ds, code, K, lo, hi, buf.data_ptr(), **shard_kw)
    eng.synchronize()  # the engine's streams -> the collective's stream
    dist.all_reduce_sum_(buf)
    torch.cuda.synchronize(device)
    return eng.de_finish(ds, code, K, buf.data_ptr(), fetch=fetch, **shard_kw)
