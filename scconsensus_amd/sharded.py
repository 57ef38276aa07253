"""One DE + distance job sharded over the ranks of a process group.

The reference parallelises the pair loop with a PSOCK foreach over the outer
cluster index (R/reclusterDEConsensusFast.R:61-65,359,384) and rbind()s the
workers' data frames.  Here every rank (one MI355X) holds the whole dataset
and owns:

* DE: a gene row-block, balanced by stored values (``gene_shard``).  It runs
  the per-(pair, gene) stage -- statistics, filters, ranks, exact U / ties / p
  -- on its genes only and packs the tested cells as 64-byte records
  (``scc_de_run_shard_records``).  ONE all-gather of the records (RCCL over
  xGMI; a few MB instead of the dense P x G arrays) gives every rank every
  tested cell, and ``scc_de_finish_records`` runs the per-pair selection (BH
  over all genes of the pair, filters, top-N, union) identically everywhere.
* PCA (Fast:398): a block of cells.  Column sums of X[U, block] (all-gather,
  combined in rank order), the centred partial Gram (all-reduce of |U| x |U|
  fp64), the eigensolve of the summed Gram on rank 0 (its vectors broadcast),
  the block's scores (all-gather of the ranks' N/world x 16 row blocks).
* dist (Fast:400): a packed-column slice of equal entry count, kept in its HBM
  (or streamed to pinned host memory).

Every engine call's status is agreed over the ranks before the collective that
follows it, so an error one rank alone sees (an R stop() on its genes, an
OOM) raises on every rank instead of leaving the others blocked.

The buffers are torch tensors: import torch (and let it load its HIP runtime)
before ``scconsensus_amd._native`` loads ``libscc.so``.  The engine launches on
torch's current stream while a sharded stage runs (``scc_ctx_set_stream``), so
torch's fills and copies, the RCCL collectives and the engine's kernels are
ordered by the stream alone, with no host synchronisation between them.
"""
from __future__ import annotations

import math

import numpy as np

from . import parallel

_SHARD_KEYS = ("mode", "q_val_thrs", "log_fc_thrs", "min_per_cent", "top_n", "fc_thrs", "mean_scaling_factor",
               "test_all", "test")
REC_WORDS = 8  # scc_de_record: 64 bytes = 8 int64 words
_I64_MAX = (1 << 63) - 1


class ShardError(RuntimeError):
    """An engine call failed on some rank; raised on every rank."""

    def __init__(self, code, msg):
        super().__init__(f"sharded job failed (scc error {code}): {msg}")
        self.code = code


def gene_shard(G: int, rank: int, world: int, weights=None) -> tuple[int, int]:
    """Gene rows of ``rank``: contiguous blocks, balanced by ``weights`` (the
    stored values per gene) when given, else by gene count."""
    if weights is None:
        return parallel.shard_range(G, rank, world)
    return parallel.weighted_range(weights, rank, world)


def cell_shard(N: int, rank: int, world: int) -> tuple[int, int]:
    """Cells of ``rank`` for the sharded PCA (equal blocks)."""
    return parallel.shard_range(N, rank, world)


def _call(fn, *a, **kw):
    """(result, status code, message) of an engine call."""
    from . import _native as nat
    try:
        return fn(*a, **kw), 0, ""
    except nat.SccError as e:
        return None, int(e.code), str(e)


def _on_stream(eng, device):
    """The engine's work on torch's current stream of ``device`` (a GPU
    engine; the CPU stand-ins of the gloo tests have no streams)."""
    import contextlib

    import torch
    if getattr(device, "type", "cpu") != "cuda" or not hasattr(eng, "on_stream"):
        return contextlib.nullcontext()
    return eng.on_stream(torch.cuda.current_stream(device).cuda_stream)


def _raise_if(codes, msg=""):
    codes = [int(c) for c in codes]
    if any(codes):
        bad = max(codes)
        raise ShardError(bad, msg or f"rank {codes.index(bad)} reported scc error {bad}")


def _stage_to_host(t):
    """An asynchronous copy of device tensor ``t`` into pinned host memory,
    ordered on the current stream (valid once that stream has been
    synchronised); CPU tensors are returned as they are."""
    import torch
    if getattr(t, "is_cuda", False):
        h = torch.empty(t.shape, dtype=t.dtype, pin_memory=True)
        h.copy_(t, non_blocking=True)
        return h
    return t


def de_sharded(eng, ds, code, K, dist: parallel.Dist, device, fetch="rows", weights=None, exchange="records",
               pair_split=True, **params):
    """The DE of one job over all ranks of ``dist``; every rank returns the same
    DeResult.  ``device``: the torch device of this rank's engine.
    ``exchange`` "records" (compact, default) or "dense" (the [P][G] int64 sum).
    FAST with fetch="union" over > 1 rank (``pair_split``): each rank runs the
    selection of a block of pairs and the union comes from the MIN-combined
    first-occurrence keys (the result then carries the union only)."""
    with _on_stream(eng, device):
        return _de_sharded(eng, ds, code, K, dist, device, fetch, weights, exchange, pair_split, **params)


def _de_sharded(eng, ds, code, K, dist, device, fetch, weights, exchange, pair_split, **params):
    import torch

    shard_kw = {k: v for k, v in params.items() if k in _SHARD_KEYS}
    lo, hi = gene_shard(ds.G, dist.rank, dist.world, weights)
    P = K * (K - 1) // 2
    if exchange == "dense":
        nbytes = eng.de_shard_bytes(K, ds.G)
        buf = torch.empty(nbytes // 8 + 1, dtype=torch.int64, device=device)
        _, st, msg = _call(eng.de_run_shard, ds, code, K, lo, hi, buf.data_ptr(), **shard_kw)
        buf[-1] = st  # the status rides in the last word: summed, nonzero iff some rank failed
        dist.all_reduce_sum_(buf)
        st_all = int(buf[-1].item())
        _raise_if([st_all], msg)
        return eng.de_finish(ds, code, K, buf.data_ptr(), fetch=fetch, **shard_kw)
    cap = max(1, P * (hi - lo))
    buf = torch.empty(cap * REC_WORDS, dtype=torch.int64, device=device)
    n, st, msg = _call(eng.de_run_shard_records, ds, code, K, lo, hi, buf.data_ptr(), cap, **shard_kw)
    n = n or 0
    # the one host read of the records exchange: RCCL sizes a gather on the
    # host, and the gather's stride is the ranks' largest record count
    info = dist.all_gather_cat(torch.tensor([st, n], dtype=torch.int64, device=device)).view(-1, 2).cpu().numpy()
    _raise_if(info[:, 0], msg)
    counts = info[:, 1].astype(np.int64)
    stride = int(max(1, counts.max()))
    if stride > cap:  # this rank sends a block of the common stride
        big = torch.zeros(stride * REC_WORDS, dtype=torch.int64, device=device)
        big[: cap * REC_WORDS] = buf
        buf = big
    recs = dist.all_gather_cat(buf[: stride * REC_WORDS])
    if fetch == "union" and params.get("mode", 0) == 0 and dist.world > 1 and pair_split:
        # the pairs are independent until the union: each rank selects its
        # pairs; the genes' first-occurrence keys are combined by MIN
        from . import _native as nat
        plo, phi = parallel.shard_range(P, dist.rank, dist.world)
        first = torch.empty(ds.G + 1, dtype=torch.int64, device=device)
        _, st, msg = _call(eng.de_finish_records_pairs, ds, code, K, recs.data_ptr(), counts, stride, plo, phi,
                           first.data_ptr(), **shard_kw)
        keys = first[: ds.G]
        keys[keys == -1] = _I64_MAX  # unselected (all ones) sorts last under a signed MIN
        first[-1] = -st  # the status rides along: MIN = minus the largest error code
        dist.all_reduce_min_(first)
        keys[keys == _I64_MAX] = -1
        # the status word is copied behind the union's own read-back (same
        # stream), so checking it costs no extra host round trip
        st_host = _stage_to_host(first[-1:])
        try:
            union = eng.de_union_first_occ(keys.data_ptr(), ds.G)
        except Exception:
            # a failed rank's keys are garbage, so the union call may fail on them
            # first: the job's status word names the real failure
            if getattr(first, "is_cuda", False):
                torch.cuda.current_stream(device).synchronize()
            _raise_if([-int(st_host[0])], msg)
            raise
        _raise_if([-int(st_host[0])], msg)
        return nat.DeResult(nat.SCC_DE_FAST, K, P, union, np.zeros(0, np.int32))
    return eng.de_finish_records(ds, code, K, recs.data_ptr(), counts, stride, fetch=fetch, **shard_kw)


def pca_sharded(eng, ds, genes, dist: parallel.Dist, device, ncomp=0):
    """prcomp_irlba(t(X[genes, ]), n = min(|U|, 15), center = TRUE)$x (Fast:398)
    of one job over the ranks: returns the full N x 16 score matrix (torch,
    float64, on ``device``; columns >= ncomp zero), identical on every rank.
    Every stage's status word rides in its collective; they are read back
    once, at the end (one host round trip)."""
    with _on_stream(eng, device):
        full, status, msgs = _pca_sharded(eng, ds, genes, dist, device, ncomp)
        _raise_if(status.cpu().numpy(), msgs[0] if msgs else "another rank's PCA stage failed")
    return full


def _pca_sharded(eng, ds, genes, dist, device, ncomp):
    """(scores, status words on the device, messages): no host read."""
    import torch

    genes = np.ascontiguousarray(genes, np.int32)
    nu, N = len(genes), ds.N
    lo, hi = cell_shard(N, dist.rank, dist.world)
    f64 = dict(dtype=torch.float64, device=device)
    msgs = []

    def call(fn, *a):
        _, st, m = _call(fn, *a)
        if st:
            msgs.append(m)
        return st

    part = torch.zeros(2 * nu + 1, **f64)  # dd column sums + the status word
    part[-1] = call(eng.pca_shard_colsum, ds, genes, lo, hi, part.data_ptr())
    parts = dist.all_gather_cat(part).view(dist.world, 2 * nu + 1)
    pcs = parts[:, : 2 * nu].contiguous()
    gram = torch.zeros(nu * nu + 1, **f64)
    gram[-1] = call(eng.pca_shard_gram, pcs.data_ptr(), dist.world, gram.data_ptr())
    dist.all_reduce_sum_(gram)
    # the eigenvectors of rank 0, broadcast: ONE eigensolve, so every rank's
    # score block comes from the same vectors
    vecs = torch.zeros(nu * 16 + 1, **f64)
    if dist.rank == 0:
        vecs[-1] = call(eng.pca_shard_eigen, gram.data_ptr(), vecs.data_ptr(), ncomp)
    dist.broadcast_(vecs, src=0)
    # this rank's rows, then an all-gather of equal-size blocks (a block holds
    # at most `rows` cells: N / world rounded up) and the status word
    rows = -(-N // dist.world)
    full = torch.zeros(N * 16, **f64)
    st = call(eng.pca_shard_project, vecs.data_ptr(), full.data_ptr(), ncomp)
    blk = torch.zeros(rows * 16 + 1, **f64)
    blk[: (hi - lo) * 16] = full[lo * 16: hi * 16]
    blk[-1] = st
    allb = dist.all_gather_cat(blk).view(dist.world, rows * 16 + 1)
    status = torch.stack([parts[:, -1].max(), gram[-1], vecs[-1], allb[:, -1].max()])
    for r in range(dist.world):
        a, b = cell_shard(N, r, dist.world)
        full[a * 16: b * 16] = allb[r, : (b - a) * 16]
    return full, status, msgs


def column_shard(N: int, rank: int, world: int) -> tuple[int, int]:
    """Columns [lo, hi) of the packed N x N lower triangle for ``rank``: column
    j holds N - 1 - j entries, the ranks get (nearly) equal entry counts."""
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


def distance_sharded(eng, ds, genes, dist: parallel.Dist, device=None, f32=False, device_out_ptr=0, ncomp=0,
                     scores=None):
    """This rank's column slice of the job's packed PCA-Euclidean distance,
    from the sharded PCA (or given ``scores``), kept in HBM (device_out_ptr 0:
    the engine's workspace; or a device pointer) or streamed to a host array
    (device_out_ptr None).  Returns (col_lo, col_hi, host array or None).
    When the call fails (ShardError), the output may already have been
    overwritten with scores from the failed PCA."""
    import torch

    if device is None:
        device = torch.device(f"cuda:{torch.cuda.current_device()}")
    lo, hi = column_shard(ds.N, dist.rank, dist.world)
    with _on_stream(eng, device):
        status, msgs = None, []
        if scores is None:
            # the PCA's status words are checked after the distance is queued
            # behind them: the job's one host read
            scores, status, msgs = _pca_sharded(eng, ds, genes, dist, device, ncomp)
            st_host = _stage_to_host(status)
        try:
            out = eng.distance_scores(scores.data_ptr(), ds.N, lo, hi, f32=f32, device_out_ptr=device_out_ptr)
        except Exception:
            if status is not None:  # a failed PCA stage is the real error
                if getattr(status, "is_cuda", False):
                    torch.cuda.current_stream(device).synchronize()
                _raise_if(st_host.numpy(), msgs[0] if msgs else "another rank's PCA stage failed")
            raise
        if status is not None:
            if getattr(status, "is_cuda", False):
                torch.cuda.current_stream(device).synchronize()
            _raise_if(st_host.numpy(), msgs[0] if msgs else "another rank's PCA stage failed")
    return lo, hi, out
