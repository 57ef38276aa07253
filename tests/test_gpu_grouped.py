"""More than 64 clusters on the GPU in ONE engine run (7-bit cluster codes;
BASELINE config E has K = 100), against one oracle run over all K; and the
group-pair orchestration (grouped.py, for K > 128) against the native run.

Covered routes: the wave kernel's second mask register (clusters 64..127)
and its 1024-pair windows (genes tested by > 1024 pairs), the items'
tested-pair tables in HBM (K^2 and P too large for LDS), the re-split with
per-parent atomics (genes with > 2048 tested pairs), the gene-level cross
kernel in 2048-pair windows."""
import numpy as np
import pytest

import oracle as O
from scconsensus_amd import api, grouped, synth
from test_gpu_de import _dense_stretch_matrix, _fast_compare, _slow_compare

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def eng():
    from scconsensus_amd import _native
    return _native.Engine(0)


@pytest.mark.parametrize("kw", [dict(), dict(min_per_cent=1.0, log_fc_thrs=0.0)])
def test_fast_100_clusters_single_run(eng, kw):
    d = synth.generate("A", G=200, N=9000, K=100, seed=17)
    names, code = api.select_clusters(d.labels, 10)
    K = len(names)
    assert K == 100
    ds = eng.dataset_csc(d.indptr, d.indices, d.data, d.G, d.N)
    g, o = _fast_compare(eng, ds, d.dense(), code, K, **kw)
    if kw:  # nearly every pair tests every gene: > 4096 tested pairs per gene (5 wave windows)
        assert np.bincount(o.row_gene).max() > 4096


def test_slow_100_clusters_single_run(eng):
    d = synth.generate("A", G=50, N=7000, K=100, seed=19)
    names, code = api.select_clusters(d.labels, 10)
    assert len(names) == 100
    ds = eng.dataset_csc(d.indptr, d.indices, d.data, d.G, d.N)
    _slow_compare(eng, ds, d.dense(), code, len(names))


@pytest.mark.parametrize("frac", [0.9, 0.07])
def test_many_clusters_dense_value_stretch(eng, frac):
    """Re-split parents and LDS items with K = 80 (tables in HBM)."""
    d, X = _dense_stretch_matrix(seed=23, G=16, N=8000, K=80, frac=frac, nested=150)
    names, code = api.select_clusters(d.labels, 10)
    assert len(names) == 80
    ds = eng.dataset_csc(d.indptr, d.indices, d.data, d.G, d.N)
    _slow_compare(eng, ds, X, code, len(names))
    _fast_compare(eng, ds, X, code, len(names), min_per_cent=1.0, log_fc_thrs=0.0)


def test_128_clusters_and_the_limit(eng):
    from scconsensus_amd import _native as nat
    d = synth.generate("A", G=60, N=9000, K=129, seed=29)
    names, code = api.select_clusters(d.labels, 10)
    assert len(names) == 129
    ds = eng.dataset_csc(d.indptr, d.indices, d.data, d.G, d.N)
    with pytest.raises(nat.SccError) as e:
        eng.de_run(ds, code, 129, nat.SCC_DE_FAST, fetch="rows")
    assert e.value.code == nat.SCC_ERR_UNSUPPORTED
    c128 = np.where(code == 128, -1, code).astype(np.int32)  # drop the last cluster: K = 128
    _fast_compare(eng, ds, d.dense(), c128, 128, min_per_cent=5.0, log_fc_thrs=0.2)
    # K = 129 through the group-pair runs (3 runs of <= 128 clusters)
    g = grouped.de_fast_grouped(eng, ds, code, 129)
    o = O.de_fast(d.dense(), code, 129)
    np.testing.assert_array_equal(g.rows.gene, o.row_gene)
    np.testing.assert_array_equal(g.rows.u2, np.round(2 * o.row_W).astype(np.int64))
    np.testing.assert_array_equal(g.union, o.union)


def test_grouped_runs_equal_native(eng):
    d = synth.generate("A", G=160, N=5000, K=70, seed=17)
    names, code = api.select_clusters(d.labels, 10)
    K = len(names)
    ds = eng.dataset_csc(d.indptr, d.indices, d.data, d.G, d.N)
    from scconsensus_amd import _native as nat
    nat_r = eng.de_run(ds, code, K, nat.SCC_DE_FAST, fetch="rows")
    g = grouped.de_fast_grouped(eng, ds, code, K, group=32, min_k=0)
    for f in ("pair_tested", "gene", "p", "q", "u2", "ties", "top"):
        np.testing.assert_array_equal(getattr(g.rows, f), getattr(nat_r.rows, f), err_msg=f)
    np.testing.assert_array_equal(g.union, nat_r.union)
