"""GPU: the pieces of one job sharded over ranks, emulated in one
process on the test box's MI355X, and the streamed distance output.

* Compact records (scc_de_run_shard_records / scc_de_finish_records): any
  split of the genes into row-blocks, gathered block by block, gives the
  unsharded scc_de_run result bit for bit (FAST, FAST t-test, SLOW).
* Sharded PCA (scc_pca_shard_*): W engines (one per emulated rank) over cell
  blocks, their Grams summed in rank order; the distance equals the
  unsharded one (bit for bit at W = 1, within 1e-6 otherwise: the Gram's
  partial sums are added in a different order) and the exact SVD within 1e-5.
* Streamed output: scc_distance to a pageable host buffer (pinned staging
  ring) and to a pinned one (direct DMA), with tiny tiles/slots so many
  overlap, equals the device-resident result bit for bit.
"""
import numpy as np
import pytest
import torch

import oracle as O
from scconsensus_amd import _native as nat
from scconsensus_amd import api, sharded, synth

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def eng():
    return nat.Engine(0)


@pytest.fixture(scope="module")
def cfg_a():
    d = synth.generate("A")
    names, code = api.select_clusters(d.labels, 10)
    return d, names, code


def _same(a, b):
    for f in ["union", "nodg"]:
        np.testing.assert_array_equal(getattr(a, f), getattr(b, f))
    if a.rows is not None:
        for f in ["pair_tested", "gene", "p", "q", "avg_logfc", "pct1", "pct2", "u2", "ties", "de", "top"]:
            np.testing.assert_array_equal(getattr(a.rows, f), getattr(b.rows, f), err_msg=f)
    for f in ["p", "q", "logfc", "u2", "de"]:
        x, y = getattr(a, f), getattr(b, f)
        if x is not None and y is not None:
            np.testing.assert_array_equal(x, y, err_msg=f)


def _records(eng, ds, code, K, bounds, **kw):
    P = K * (K - 1) // 2
    blocks, counts = [], []
    for lo, hi in bounds:
        cap = max(1, P * (hi - lo))
        buf = torch.full((cap * 8,), -1, dtype=torch.int64, device="cuda:0")
        n = eng.de_run_shard_records(ds, code, K, lo, hi, buf.data_ptr(), cap, **kw)
        assert 0 <= n <= cap
        blocks.append(buf)
        counts.append(n)
    stride = max(1, max(counts))
    allr = torch.full((len(bounds) * stride * 8,), -7, dtype=torch.int64, device="cuda:0")
    for b, (buf, n) in enumerate(zip(blocks, counts)):
        allr[b * stride * 8: b * stride * 8 + n * 8] = buf[: n * 8]
    torch.cuda.synchronize()
    return allr, counts, stride


@pytest.mark.parametrize("bounds", [[(0, 700), (700, 1400), (1400, 2000)], [(0, 1), (1, 1999), (1999, 2000)],
                                    [(0, 2000)], [(0, 0), (0, 1000), (1000, 2000)]])
def test_records_fast_match_unsharded(eng, cfg_a, bounds):
    d, names, code = cfg_a
    K = len(names)
    ds = eng.dataset_csc(d.indptr, d.indices, d.data, d.G, d.N)
    ref = eng.de_run(ds, code, K, nat.SCC_DE_FAST, fetch="rows")
    allr, counts, stride = _records(eng, ds, code, K, bounds)
    assert sum(counts) == len(ref.rows.gene)  # one record per tested (pair, gene) cell
    got = eng.de_finish_records(ds, code, K, allr.data_ptr(), counts, stride, fetch="rows")
    _same(ref, got)


@pytest.mark.parametrize("bounds", [[(0, 300), (300, 1301), (1301, 2000)], [(0, 255), (255, 257), (257, 2000)],
                                    [(0, 1), (1, 1999), (1999, 2000)], [(0, 0), (0, 2000)]])
def test_records_range_ingest_matches_full(eng, cfg_a, bounds, monkeypatch):
    """Gene-shard ingest of a validated dataset (k_ing_hist rng: two wave-parallel
    binary searches per cell, only the shard's gene tiles read, nodg from the
    dataset's cache) gives the same records and nodg as reading every entry:
    first pass on a fresh dataset (full read, validates), second pass (range
    read), third with SCC_INGEST_FULL=1."""
    d, names, code = cfg_a
    K = len(names)
    ds = eng.dataset_csc(d.indptr, d.indices, d.data, d.G, d.N)
    runs = []
    for full in ("0", "0", "1"):
        monkeypatch.setenv("SCC_INGEST_FULL", full)
        allr, counts, stride = _records(eng, ds, code, K, bounds)
        got = eng.de_finish_records(ds, code, K, allr.data_ptr(), counts, stride, fetch="rows")
        runs.append((allr.cpu().numpy(), counts, got))
    for allr, counts, got in runs[1:]:
        assert counts == runs[0][1]
        np.testing.assert_array_equal(allr, runs[0][0])
        _same(runs[0][2], got)
    ref = eng.de_run(eng.dataset_csc(d.indptr, d.indices, d.data, d.G, d.N), code, K, nat.SCC_DE_FAST, fetch="rows")
    _same(ref, runs[1][2])


@pytest.mark.parametrize("pair_cuts", [[0, 28], [0, 10, 20, 28], [0, 0, 1, 27, 28]])
def test_pair_split_selection_union(eng, cfg_a, pair_cuts):
    """FAST selection split by pairs (scc_de_finish_records_pairs on each block
    of pairs, first-occurrence keys MIN-combined, scc_de_union_first_occ):
    deGeneUnion identical, in order, to the unsharded scc_de_run's."""
    d, names, code = cfg_a
    K = len(names)
    P = K * (K - 1) // 2
    assert pair_cuts[-1] == P
    ds = eng.dataset_csc(d.indptr, d.indices, d.data, d.G, d.N)
    ref = eng.de_run(ds, code, K, nat.SCC_DE_FAST, fetch="union")
    allr, counts, stride = _records(eng, ds, code, K, [(0, 900), (900, 2000)])
    big = (1 << 63) - 1
    comb = torch.full((d.G,), big, dtype=torch.int64, device="cuda:0")
    for lo, hi in zip(pair_cuts[:-1], pair_cuts[1:]):
        first = torch.empty(d.G, dtype=torch.int64, device="cuda:0")
        eng.de_finish_records_pairs(ds, code, K, allr.data_ptr(), counts, stride, lo, hi, first.data_ptr())
        torch.cuda.synchronize()
        first[first == -1] = big
        comb = torch.minimum(comb, first)
    comb[comb == big] = -1
    torch.cuda.synchronize()
    np.testing.assert_array_equal(eng.de_union_first_occ(comb.data_ptr(), d.G), ref.union)


def test_records_t_and_slow_match_unsharded(eng, cfg_a):
    d, names, code = cfg_a
    K = len(names)
    ds = eng.dataset_csc(d.indptr, d.indices, d.data, d.G, d.N)
    ref = eng.de_run(ds, code, K, nat.SCC_DE_FAST, fetch="rows", test="t")
    allr, counts, stride = _records(eng, ds, code, K, [(0, 900), (900, 2000)], test="t")
    _same(ref, eng.de_finish_records(ds, code, K, allr.data_ptr(), counts, stride, fetch="rows", test="t"))
    X = d.dense()[:400]
    ds2 = eng.dataset_dense(X)
    kw = dict(mode=nat.SCC_DE_SLOW)
    ref = eng.de_run(ds2, code, K, fetch="all", **kw)
    allr, counts, stride = _records(eng, ds2, code, K, [(0, 150), (150, 400)], **kw)
    assert sum(counts) == K * (K - 1) // 2 * 400  # SLOW tests every gene
    got = eng.de_finish_records(ds2, code, K, allr.data_ptr(), counts, stride, fetch="all", **kw)
    _same(ref, got)
    assert got.log_thr == ref.log_thr


def test_records_capacity_and_bad_records(eng, cfg_a):
    d, names, code = cfg_a
    K = len(names)
    ds = eng.dataset_csc(d.indptr, d.indices, d.data, d.G, d.N)
    buf = torch.zeros(8 * 4, dtype=torch.int64, device="cuda:0")
    with pytest.raises(nat.SccError) as e:
        eng.de_run_shard_records(ds, code, K, 0, d.G, buf.data_ptr(), 4)
    assert e.value.code == nat.SCC_ERR_INVALID
    allr, counts, stride = _records(eng, ds, code, K, [(0, d.G)])
    allr.view(-1, 8)[0, 0] = 10_000  # pair index out of range
    torch.cuda.synchronize()
    with pytest.raises(nat.SccError):
        eng.de_finish_records(ds, code, K, allr.data_ptr(), counts, stride, fetch="union")


@pytest.mark.parametrize("world", [1, 2, 3])
def test_sharded_pca_matches_unsharded(cfg_a, world):
    d, names, code = cfg_a
    e0 = nat.Engine(0)
    ds0 = e0.dataset_csc(d.indptr, d.indices, d.data, d.G, d.N)
    union = e0.de_run(ds0, code, len(names), nat.SCC_DE_FAST, fetch="union").union
    full = e0.distance(ds0, union)
    nu, N = len(union), d.N
    engs = [nat.Engine(0) for _ in range(world)]
    dss = [e.dataset_csc(d.indptr, d.indices, d.data, d.G, d.N) for e in engs]
    parts = []
    for r, (e, ds) in enumerate(zip(engs, dss)):
        lo, hi = sharded.cell_shard(N, r, world)
        part = torch.empty(2 * nu, dtype=torch.float64, device="cuda:0")
        e.pca_shard_colsum(ds, union, lo, hi, part.data_ptr())
        parts.append(part)
    parts = torch.cat(parts)
    grams = []
    for e in engs:
        g = torch.empty(nu * nu, dtype=torch.float64, device="cuda:0")
        e.pca_shard_gram(parts.data_ptr(), world, g.data_ptr())
        grams.append(g)
    gram = grams[0].clone()
    for g in grams[1:]:
        gram += g
    # as sharded.pca_sharded runs it: ONE eigensolve (rank 0), its vectors
    # broadcast, every rank projects its block.  (Separate eigensolves per rank
    # are not used: the hand-off solver's partial sums follow how many
    # workgroups joined, and at config A's sigma15 / sigma16 = 1.00035 a last-bit
    # difference can rotate PC 15 or flip a near-tied sign rule between blocks.)
    vecs = torch.zeros(nu * 16, dtype=torch.float64, device="cuda:0")
    engs[0].pca_shard_eigen(gram.data_ptr(), vecs.data_ptr())
    scores = torch.zeros(N * 16, dtype=torch.float64, device="cuda:0")
    for e in engs:
        e.pca_shard_project(vecs.data_ptr(), scores.data_ptr())
    torch.cuda.synchronize()
    got = engs[0].distance_scores(scores.data_ptr(), N, 0, N)
    if world == 1:
        # eigen + project == the one-call scc_pca_shard_scores == the unsharded distance
        scores1 = torch.zeros(N * 16, dtype=torch.float64, device="cuda:0")
        engs[0].pca_shard_scores(gram.data_ptr(), scores1.data_ptr())
        torch.cuda.synchronize()
        assert torch.equal(scores, scores1)
        np.testing.assert_array_equal(got, full)
    else:
        # the Gram's partial sums are added in another order: PC 15 moves by ~1e-8
        assert np.max(np.abs(got - full)) < 1e-6
    ref = O.dist_euclidean(O.pca_scores(d.dense(), union))
    assert np.max(np.abs(got - ref)) < 1e-5
    # a rank's slice from the same scores
    lo, hi = sharded.column_shard(N, world - 1, world)
    s0, s1 = lo * (2 * N - lo - 1) // 2, hi * (2 * N - hi - 1) // 2
    np.testing.assert_array_equal(engs[-1].distance_scores(scores.data_ptr(), N, lo, hi), got[s0:s1])
    for ds in dss:
        ds.close()
    for e in engs:
        e.close()
    e0.close()


@pytest.mark.parametrize("metric", [nat.SCC_DIST_PCA_EUCLID, nat.SCC_DIST_PEARSON])
@pytest.mark.parametrize("f32", [False, True])
@pytest.mark.parametrize("kernel_copy", ["1", "0"])
def test_streamed_output_matches_device(eng, cfg_a, metric, f32, kernel_copy, monkeypatch):
    monkeypatch.setenv("SCC_D2H_KERNEL", kernel_copy)  # k_d2h on the CUs, or hipMemcpyAsync
    monkeypatch.setenv("SCC_DIST_CHUNK_MB", "1")  # ~20 chunks into a pinned buffer at config A
    monkeypatch.setenv("SCC_DIST_STAGE_MB", "1")  # ~10-20 staging chunks through the 2-slot ring
    d, names, code = cfg_a
    ds = eng.dataset_csc(d.indptr, d.indices, d.data, d.G, d.N)
    union = eng.de_run(ds, code, len(names), nat.SCC_DE_FAST, fetch="union").union
    N = d.N
    n = N * (N - 1) // 2
    dt = torch.float32 if f32 else torch.float64
    dev = torch.empty(n, dtype=dt, device="cuda:0")
    eng.distance(ds, union, metric, f32=f32, device_out_ptr=dev.data_ptr())
    eng.synchronize()
    ref = dev.cpu().numpy()
    pageable = eng.distance(ds, union, metric, f32=f32)
    np.testing.assert_array_equal(pageable, ref)
    pinned = torch.empty(n, dtype=dt, pin_memory=True)
    eng.distance(ds, union, metric, f32=f32, out=pinned.numpy())
    np.testing.assert_array_equal(pinned.numpy(), ref)
    # a pinned destination one element off its 16-B alignment (the copy's head/tail path)
    off = torch.zeros(n + 2, dtype=dt, pin_memory=True)
    eng.distance(ds, union, metric, f32=f32, out=off.numpy()[1:n + 1])
    np.testing.assert_array_equal(off.numpy()[1:n + 1], ref)
    assert off[0].item() == 0 and off[n + 1].item() == 0
    # a column slice, streamed
    lo, hi = 100, 1700
    s0, s1 = lo * (2 * N - lo - 1) // 2, hi * (2 * N - hi - 1) // 2
    np.testing.assert_array_equal(eng.distance_cols(ds, union, lo, hi, metric, f32=f32), ref[s0:s1])


@pytest.mark.parametrize("register", ["1", "0"])
def test_large_pageable_output_registered(eng, register, monkeypatch):
    """A pageable output of >= 256 MB (R's allocVector at scale) through the
    staging ring (the default) or registered with the runtime for the call and
    written directly by k_d2h (SCC_DIST_REGISTER=1); both bit-identical to the
    device output, the buffer's neighbours untouched (one element off the
    16-B alignment, as inside an R vector)."""
    monkeypatch.setenv("SCC_DIST_REGISTER", register)
    d = synth.generate("A", G=600, N=8300, K=6, seed=21)
    names, code = api.select_clusters(d.labels, 10)
    ds = eng.dataset_csc(d.indptr, d.indices, d.data, d.G, d.N)
    union = eng.de_run(ds, code, len(names), nat.SCC_DE_FAST, fetch="union").union
    n = d.N * (d.N - 1) // 2
    assert 8 * n >= 256 << 20
    dev = torch.empty(n, dtype=torch.float64, device="cuda:0")
    eng.distance(ds, union, nat.SCC_DIST_PCA_EUCLID, device_out_ptr=dev.data_ptr())
    eng.synchronize()
    ref = dev.cpu().numpy()
    del dev
    buf = np.full(n + 2, -7.0)
    eng.distance(ds, union, nat.SCC_DIST_PCA_EUCLID, out=buf[1:n + 1])
    np.testing.assert_array_equal(buf[1:n + 1], ref)
    assert buf[0] == -7.0 and buf[n + 1] == -7.0
    ds.close()
