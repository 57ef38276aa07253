"""One DE + distance job sharded over the ranks of a process group.

The reference parallelises the pair loop with a PSOCK foreach over the outer
cluster index (R/reclusterDEConsensusFast.R:61-65,359,384).  Here each rank
(one MI355X) holds the whole dataset and runs the per-(pair, gene) stage —
per-cluster statistics, filters, ranks, exact U / ties / p — on its block of
gene rows (``scc_de_run_shard``).  The only exchange is one all-reduce (RCCL
over xGMI) of the shard buffers: they are disjoint and zero elsewhere, so the
int64 sum is the exact union of every rank's cells.  Every rank then runs the
per-pair selection (BH over all genes of the pair, filters, top-N, union) on
the same bits (``scc_de_finish``) and gets the result ``scc_de_run`` gives.

The shard buffers are torch tensors: import torch (and let it load its HIP
runtime) before ``scconsensus_amd._native`` loads ``libscc.so``.
"""
from __future__ import annotations

from . import parallel

_SHARD_KEYS = ("mode", "q_val_thrs", "log_fc_thrs", "min_per_cent", "top_n", "fc_thrs", "mean_scaling_factor",
               "test_all", "test")


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
    if buf.is_cuda:
        torch.cuda.synchronize(buf.device)
    return eng.de_finish(ds, code, K, buf.data_ptr(), fetch=fetch, **shard_kw)


def column_shard(N: int, rank: int, world: int) -> tuple[int, int]:
    """Columns [lo, hi) of the packed N x N lower triangle for ``rank``: column
    j holds N - 1 - j entries, the ranks get (nearly) equal entry counts."""
    import math

    total = N * (N - 1) // 2

    def col_at(share):  # first column whose packed start is >= share
        # start(j) = j (2N - j - 1) / 2 = share  ->  j = ((2N - 1) - sqrt((2N - 1)^2 - 8 share)) / 2
        b = 2 * N - 1
        j = int((b - math.sqrt(max(b * b - 8 * share, 0))) / 2)
        start = lambda c: c * (2 * N - c - 1) // 2  # noqa: E731
        while j > 0 and start(j) > share:
            j -= 1
        while j < N and start(j) < share:
            j += 1
        return j

    lo = 0 if rank == 0 else col_at(total * rank // world)
    hi = N if rank == world - 1 else col_at(total * (rank + 1) // world)
    return lo, hi


def distance_sharded(eng, ds, genes, dist: parallel.Dist, metric=None, f32=False, device_out_ptr=0):
    """This rank's column slice of the job's packed distance vector, kept in
    HBM (device_out_ptr 0: the engine's workspace) or copied to a host array
    (device_out_ptr None).  Returns (col_lo, col_hi, host array or None)."""
    from . import _native as nat

    lo, hi = column_shard(ds.N, dist.rank, dist.world)
    m = nat.SCC_DIST_PCA_EUCLID if metric is None else metric
    out = eng.distance_cols(ds, genes, lo, hi, metric=m, f32=f32, device_out_ptr=device_out_ptr)
    return lo, hi, out
