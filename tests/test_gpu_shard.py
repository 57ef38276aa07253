"""GPU: one DE job sharded over gene row-blocks gives exactly the
unsharded result.  The ranks are emulated in one process on one MI355X: each
shard is run in turn into its own device buffer, the buffers are summed as
int64 words (what the RCCL all-reduce does across ranks) and the sum is
finished.  Rows, U, ties, p, q, flags and the union must be bit-identical."""
import numpy as np
import pytest
import torch

from scconsensus_amd import _native as nat
from scconsensus_amd import api, parallel, sharded, synth

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def eng():
    return nat.Engine(0)


@pytest.fixture(scope="module")
def cfg_a():
    d = synth.generate("A")
    names, code = api.select_clusters(d.labels, 10)
    return d, names, code


def _run_shards(eng, ds, code, K, bounds, **kw):
    nbytes = eng.de_shard_bytes(K, ds.G)
    total = torch.zeros(nbytes // 8, dtype=torch.int64, device="cuda:0")
    for lo, hi in bounds:
        buf = torch.full((nbytes // 8,), -1, dtype=torch.int64, device="cuda:0")  # the engine must zero it
        eng.de_run_shard(ds, code, K, lo, hi, buf.data_ptr(), **kw)
        eng.synchronize()
        total += buf
    torch.cuda.synchronize()
    return total


def _same(a, b):
    for f in ["union", "nodg"]:
        np.testing.assert_array_equal(getattr(a, f), getattr(b, f))
    if a.rows is not None:
        for f in ["pair_tested", "gene", "p", "q", "avg_logfc", "pct1", "pct2", "u2", "ties", "de", "top"]:
            np.testing.assert_array_equal(getattr(a.rows, f), getattr(b.rows, f), err_msg=f)
    for f in ["p", "q", "logfc", "u2", "de"]:
        x, y = getattr(a, f), getattr(b, f)
        if x is not None:
            np.testing.assert_array_equal(x, y, err_msg=f)


@pytest.mark.parametrize("bounds", [[(0, 700), (700, 1400), (1400, 2000)], [(0, 1), (1, 1999), (1999, 2000)],
                                    [(0, 2000)], [(0, 0), (0, 1000), (1000, 2000)]])
def test_fast_shards_match_unsharded(eng, cfg_a, bounds):
    d, names, code = cfg_a
    K = len(names)
    ds = eng.dataset_csc(d.indptr, d.indices, d.data, d.G, d.N)
    ref = eng.de_run(ds, code, K, nat.SCC_DE_FAST, fetch="rows")
    tot = _run_shards(eng, ds, code, K, bounds)
    got = eng.de_finish(ds, code, K, tot.data_ptr(), fetch="rows")
    _same(ref, got)
    assert len(got.union) > 50


def test_fast_t_shards_match_unsharded(eng, cfg_a):
    d, names, code = cfg_a
    K = len(names)
    ds = eng.dataset_csc(d.indptr, d.indices, d.data, d.G, d.N)
    ref = eng.de_run(ds, code, K, nat.SCC_DE_FAST, fetch="rows", test="t")
    tot = _run_shards(eng, ds, code, K, [(0, 900), (900, 2000)], test="t")
    _same(ref, eng.de_finish(ds, code, K, tot.data_ptr(), fetch="rows", test="t"))


def test_slow_shards_match_unsharded(eng, cfg_a):
    d, names, code = cfg_a
    K = len(names)
    X = d.dense()[:400]
    ds = eng.dataset_dense(X)
    kw = dict(mode=nat.SCC_DE_SLOW)
    ref = eng.de_run(ds, code, K, fetch="all", **kw)
    tot = _run_shards(eng, ds, code, K, [(0, 150), (150, 400)], **kw)
    got = eng.de_finish(ds, code, K, tot.data_ptr(), fetch="all", **kw)
    _same(ref, got)
    assert got.log_thr == ref.log_thr


def test_de_sharded_single_rank(eng, cfg_a):
    d, names, code = cfg_a
    K = len(names)
    ds = eng.dataset_csc(d.indptr, d.indices, d.data, d.G, d.N)
    ref = eng.de_run(ds, code, K, nat.SCC_DE_FAST, fetch="rows", min_per_cent=10.0)
    got = sharded.de_sharded(eng, ds, code, K, parallel.Dist(), torch.device("cuda:0"), min_per_cent=10.0)
    _same(ref, got)


def test_finish_requires_a_shard_run(cfg_a):
    e2 = nat.Engine(0)
    d, names, code = cfg_a
    ds = e2.dataset_csc(d.indptr, d.indices, d.data, d.G, d.N)
    buf = torch.zeros(e2.de_shard_bytes(len(names), d.G) // 8, dtype=torch.int64, device="cuda:0")
    with pytest.raises(nat.SccError):
        e2.de_finish(ds, code, len(names), buf.data_ptr())


@pytest.mark.parametrize("metric,f32", [(nat.SCC_DIST_PCA_EUCLID, False), (nat.SCC_DIST_PCA_EUCLID, True),
                                        (nat.SCC_DIST_PEARSON, False)])
def test_distance_column_slices_match_full(eng, cfg_a, metric, f32):
    d, names, code = cfg_a
    ds = eng.dataset_csc(d.indptr, d.indices, d.data, d.G, d.N)
    union = eng.de_run(ds, code, len(names), nat.SCC_DE_FAST, fetch="union").union
    full = eng.distance(ds, union, metric=metric, f32=f32)
    for world in (2, 3, 8):
        parts = [eng.distance_cols(ds, union, *sharded.column_shard(d.N, r, world), metric=metric, f32=f32)
                 for r in range(world)]
        np.testing.assert_array_equal(np.concatenate(parts), full)
    # ragged slices: one column, the last column, an empty one, a block-unaligned middle
    N = d.N
    for lo, hi in [(0, 1), (N - 2, N), (5, 5), (63, 1000), (1000, N - 2)]:
        s0 = lo * (2 * N - lo - 1) // 2
        s1 = hi * (2 * N - hi - 1) // 2
        np.testing.assert_array_equal(eng.distance_cols(ds, union, lo, hi, metric=metric, f32=f32), full[s0:s1])


def test_distance_sharded_single_rank(eng, cfg_a):
    d, names, code = cfg_a
    ds = eng.dataset_csc(d.indptr, d.indices, d.data, d.G, d.N)
    union = eng.de_run(ds, code, len(names), nat.SCC_DE_FAST, fetch="union").union
    lo, hi, out = sharded.distance_sharded(eng, ds, union, parallel.Dist(), device_out_ptr=None)
    assert (lo, hi) == (0, d.N)
    np.testing.assert_array_equal(out, eng.distance(ds, union))
