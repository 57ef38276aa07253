"""Many clusters on the GPU, each through ONE scc_de_run call: up to 128 in
one engine run (7-bit cluster codes; BASELINE config E has K = 100), and any
K beyond that through the group-pair runs inside libscc (de_run_grouped),
against one oracle run over all K; plus gene counts past one LDS histogram
window (G = 50,000 and forced small windows).

Covered routes: the wave kernel's second mask register (clusters 64..127)
and its 1024-pair windows (genes tested by > 1024 pairs), the items'
tested-pair tables in HBM (K^2 and P too large for LDS), the re-split with
per-parent atomics (genes with > 2048 tested pairs), the gene-level cross
kernel in 2048-pair windows."""
import numpy as np
import pytest

import oracle as O
from scconsensus_amd import api, synth
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


def test_129_clusters_one_call(eng):
    """K = 129: the smallest K past one engine run (3 group-pair runs)."""
    d = synth.generate("A", G=60, N=9000, K=129, seed=29)
    names, code = api.select_clusters(d.labels, 10)
    assert len(names) == 129
    ds = eng.dataset_csc(d.indptr, d.indices, d.data, d.G, d.N)
    _fast_compare(eng, ds, d.dense(), code, 129)
    c128 = np.where(code == 128, -1, code).astype(np.int32)  # drop the last cluster: K = 128, one run
    _fast_compare(eng, ds, d.dense(), c128, 128, min_per_cent=5.0, log_fc_thrs=0.2)


def test_fast_150_clusters_one_call(eng):
    d = synth.generate("A", G=60, N=12000, K=150, seed=31)
    names, code = api.select_clusters(d.labels, 10)
    assert len(names) == 150
    ds = eng.dataset_csc(d.indptr, d.indices, d.data, d.G, d.N)
    g, o = _fast_compare(eng, ds, d.dense(), code, 150, min_per_cent=5.0, log_fc_thrs=0.2)
    assert len(o.row_gene) > 100_000 and len(o.union) > 30


def test_slow_150_clusters_one_call(eng):
    d = synth.generate("A", G=24, N=12000, K=150, seed=37)
    names, code = api.select_clusters(d.labels, 10)
    assert len(names) == 150
    ds = eng.dataset_csc(d.indptr, d.indices, d.data, d.G, d.N)
    g, o = _slow_compare(eng, ds, d.dense(), code, 150)
    assert g.p.shape == (150 * 149 // 2, 24) and len(o.union) > 0


@pytest.mark.parametrize("mode", ["fast", "slow"])
def test_grouped_runs_equal_native(eng, mode, monkeypatch):
    """SCC_GROUP_SIZE=32 forces group-pair runs at K = 70 (3 groups): bit for
    bit the one-run result."""
    from scconsensus_amd import _native as nat
    d = synth.generate("A", G=160 if mode == "fast" else 40, N=5000, K=70, seed=17)
    names, code = api.select_clusters(d.labels, 10)
    K = len(names)
    ds = eng.dataset_csc(d.indptr, d.indices, d.data, d.G, d.N)
    m = nat.SCC_DE_FAST if mode == "fast" else nat.SCC_DE_SLOW
    kw = dict(min_per_cent=5.0, log_fc_thrs=0.1) if mode == "fast" else dict(q_val_thrs=0.05, fc_thrs=1.5)
    one = eng.de_run(ds, code, K, m, fetch="all", **kw)
    monkeypatch.setenv("SCC_GROUP_SIZE", "32")
    grp = eng.de_run(ds, code, K, m, fetch="all", **kw)
    np.testing.assert_array_equal(grp.union, one.union)
    np.testing.assert_array_equal(grp.nodg, one.nodg)
    for f in ("p", "logfc", "u2") + (("q", "de") if mode == "slow" else ()):
        np.testing.assert_array_equal(getattr(grp, f), getattr(one, f), err_msg=f)
    if mode == "fast":
        for f in ("pair_tested", "gene", "p", "q", "avg_logfc", "pct1", "pct2", "u2", "ties", "de", "top"):
            np.testing.assert_array_equal(getattr(grp.rows, f), getattr(one.rows, f), err_msg=f)
        u = eng.de_run(ds, code, K, m, fetch="union", **kw)  # no per-pair vectors kept
        np.testing.assert_array_equal(u.union, one.union)
    else:
        assert grp.log_thr == one.log_thr


def test_50000_genes(eng):
    """G = 50,000 (was refused past 40,960: one LDS histogram window per
    chunk; now 8-bit counters, 163,840 genes per window)."""
    d = synth.generate("A", G=50_000, N=1200, K=6, seed=41)
    names, code = api.select_clusters(d.labels, 10)
    X = d.dense()
    ds = eng.dataset_csc(d.indptr, d.indices, d.data, d.G, d.N)
    g, o = _fast_compare(eng, ds, X, code, len(names))
    assert len(o.union) > 30
    np.testing.assert_array_equal(g.nodg, O.nodg(X))
    _slow_compare(eng, ds, X, code, len(names))


@pytest.mark.parametrize("window", ["100", "777"])
def test_histogram_windows(eng, window, monkeypatch):
    """Forced small gene windows (several histogram passes per count chunk),
    CSC and dense input, FAST and SLOW: the oracle's results."""
    monkeypatch.setenv("SCC_HIST_WINDOW", window)
    d = synth.generate("A", G=1000, N=1500, K=6, seed=43)
    names, code = api.select_clusters(d.labels, 10)
    X = d.dense()
    for ds in (eng.dataset_csc(d.indptr, d.indices, d.data, d.G, d.N), eng.dataset_dense(X)):
        g, _ = _fast_compare(eng, ds, X, code, len(names))
        np.testing.assert_array_equal(g.nodg, O.nodg(X))
        _slow_compare(eng, ds, X, code, len(names))
