"""GPU parity: the MI355X DE engine (through the C ABI) vs the CPU oracle.

Bar (BASELINE.json north_star): rank sums / U statistics and selected-gene
sets bit-exact; p/q within 1e-6 relative.  logFC is compared at 1e-12
relative or 5e-14 absolute (GPU expm1/log vs glibc: a few ulp of the two
log-means, which the subtraction m_i - m_j keeps in absolute terms when they
nearly cancel; documented in DESIGN.md)."""
import numpy as np
import pytest

import oracle as O
from scconsensus_amd import api, synth

pytestmark = pytest.mark.gpu

P_RTOL = 1e-6
LFC_RTOL = 1e-12
LFC_ATOL = 5e-14


@pytest.fixture(scope="module")
def eng():
    from scconsensus_amd import _native
    return _native.Engine(0)


@pytest.fixture(scope="module")
def cfg_a():
    d = synth.generate("A")
    names, code = api.select_clusters(d.labels, 10)
    return d, d.dense(), names, code


@pytest.fixture(scope="module")
def edge():
    d = synth.edge_fixture()
    names, code = api.select_clusters(d.labels, 10)
    return d, d.dense(), names, code


def _fast_compare(eng, ds, X, code, K, **kw):
    from scconsensus_amd import _native as nat
    g = eng.de_run(ds, code, K, nat.SCC_DE_FAST, fetch="rows", **kw)
    o = O.de_fast(X, code, K, **kw)
    r = g.rows
    np.testing.assert_array_equal(r.pair_tested, o.pair_tested)      # tested feature sets (sizes)
    np.testing.assert_array_equal(r.gene, o.row_gene)                 # sets AND R's row order
    np.testing.assert_array_equal(r.u2, np.round(2 * o.row_W).astype(np.int64))  # exact U
    np.testing.assert_array_equal(r.ties, np.round(o.row_ties).astype(np.int64))
    np.testing.assert_allclose(r.p, o.row_p, rtol=P_RTOL, atol=0)
    np.testing.assert_allclose(r.q, o.row_q, rtol=P_RTOL, atol=0)
    np.testing.assert_allclose(r.avg_logfc, o.row_lfc, rtol=LFC_RTOL, atol=LFC_ATOL)
    np.testing.assert_array_equal(r.pct1, o.row_pct1)
    np.testing.assert_array_equal(r.pct2, o.row_pct2)
    np.testing.assert_array_equal(r.de, o.row_de)
    np.testing.assert_array_equal(r.top, o.row_top)
    np.testing.assert_array_equal(g.union, o.union)                   # deGeneUnion, in order
    return g, o


def test_fast_config_a(eng, cfg_a):
    d, X, names, code = cfg_a
    ds = eng.dataset_csc(d.indptr, d.indices, d.data, d.G, d.N)
    g, o = _fast_compare(eng, ds, X, code, len(names))
    assert len(o.union) > 50
    # the p-values agree far tighter than the bar
    assert np.max(np.abs(g.rows.p - o.row_p) / np.maximum(o.row_p, 1e-300)) < 1e-12
    np.testing.assert_array_equal(g.nodg, O.nodg(X))


def test_fast_config_a_dense_input(eng, cfg_a):
    d, X, names, code = cfg_a
    ds = eng.dataset_dense(X)
    _fast_compare(eng, ds, X, code, len(names))


@pytest.mark.parametrize("kw", [dict(q_val_thrs=0.05, log_fc_thrs=0.25, min_per_cent=10.0, top_n=5),
                                dict(q_val_thrs=0.5, log_fc_thrs=1.0, min_per_cent=40.0, top_n=100)])
def test_fast_config_a_params(eng, cfg_a, kw):
    d, X, names, code = cfg_a
    ds = eng.dataset_csc(d.indptr, d.indices, d.data, d.G, d.N)
    _fast_compare(eng, ds, X, code, len(names), **kw)


@pytest.mark.parametrize("kw", [dict(), dict(min_per_cent=5.0, log_fc_thrs=0.1, top_n=10)])
def test_fast_t_test_config_a(eng, cfg_a, kw):
    """test.use = "t" (DiffTTest, Fast:185-196): Welch t.test p per tested
    feature, then the same BH / filters / union as the Wilcoxon path."""
    d, X, names, code = cfg_a
    ds = eng.dataset_csc(d.indptr, d.indices, d.data, d.G, d.N)
    g, o = _fast_compare(eng, ds, X, code, len(names), test="t", **kw)
    assert o.status == 0 and len(o.union) > 20
    assert np.max(np.abs(g.rows.p - o.row_p) / np.maximum(o.row_p, 1e-300)) < 1e-9
    assert (g.rows.u2 == 0).all()


def test_fast_t_test_constant_data_stops(eng):
    """R's t.test stops on "data are essentially constant": a tested gene
    constant within both clusters (different levels) makes the engine return
    SCC_ERR_RSTOP, like the oracle's status."""
    from scconsensus_amd import _native as nat
    rng = np.random.default_rng(5)
    N, G = 60, 5
    code = np.repeat(np.arange(3), 20).astype(np.int32)
    X = rng.gamma(1.0, 1.0, (G, N)) * (rng.random((G, N)) < 0.7)
    X[2] = np.where(code == 0, 1.0, 3.0)
    assert O.de_fast(X, code, 3, test="t").status == nat.SCC_ERR_RSTOP
    ds = eng.dataset_dense(X)
    with pytest.raises(nat.SccError) as e:
        eng.de_run(ds, code, 3, nat.SCC_DE_FAST, test="t", fetch="rows")
    assert e.value.code == nat.SCC_ERR_RSTOP


@pytest.mark.parametrize("K", [18, 26, 40])
def test_fast_many_clusters(eng, K):
    """More tested pairs per gene than the wave kernel's 2-slot variant holds
    (P = 153: 4 slots; P = 325: 8 slots; P = 780: 16 slots, config C/D-like)."""
    d = synth.generate("A", G=400, N=4000, K=K, seed=7)
    names, code = api.select_clusters(d.labels, 10)
    assert len(names) * (len(names) - 1) // 2 > 128
    ds = eng.dataset_csc(d.indptr, d.indices, d.data, d.G, d.N)
    _fast_compare(eng, ds, d.dense(), code, len(names), min_per_cent=5.0, log_fc_thrs=0.1)


def test_fast_edge_fixture(eng, edge):
    d, X, names, code = edge
    assert "grey" not in names and "grey60" not in names and "tiny" not in names
    ds = eng.dataset_csc(d.indptr, d.indices, d.data, d.G, d.N)
    g, o = _fast_compare(eng, ds, X, code, len(names), log_fc_thrs=0.1, min_per_cent=15.0)
    from scconsensus_amd import _native as nat
    full = eng.de_run(ds, code, len(names), nat.SCC_DE_FAST, log_fc_thrs=0.1, min_per_cent=15.0, fetch="rows")
    assert full.rows is not None


def test_exact_branch_is_exercised(eng, edge):
    """Tie-free genes between the 20- and 15-cell clusters use R's exact pwilcox."""
    from scconsensus_amd import _native as nat
    d, X, names, code = edge
    ds = eng.dataset_csc(d.indptr, d.indices, d.data, d.G, d.N)
    g = eng.de_run(ds, code, len(names), nat.SCC_DE_FAST, fetch="all")
    a, b = names.index("brown"), names.index("yellow")
    K = len(names)
    p = a * K - a * (a + 1) // 2 + (b - a - 1)
    for gene in range(30, 36):
        x = X[gene, code == a]
        y = X[gene, code == b]
        po, W, T, meth = O.wilcox_test(x, y)
        assert meth == "exact"
        assert g.u2[p, gene] == int(2 * W)
        assert g.p[p, gene] == pytest.approx(po, rel=1e-13)


def _slow_compare(eng, ds, X, code, K, qthr=0.05, fc=1.5, msf=5.0):
    from scconsensus_amd import _native as nat
    g = eng.de_run(ds, code, K, nat.SCC_DE_SLOW, q_val_thrs=qthr, fc_thrs=fc, mean_scaling_factor=msf, fetch="all")
    o = O.de_slow(X, code, K, qthr, fc, msf)
    assert g.log_thr == pytest.approx(o.log_thr, rel=1e-14)
    np.testing.assert_array_equal(g.u2, np.round(2 * o.W).astype(np.int64))
    np.testing.assert_allclose(g.p, o.p, rtol=P_RTOL, atol=0, equal_nan=True)
    np.testing.assert_allclose(g.q, o.q, rtol=P_RTOL, atol=0, equal_nan=True)
    np.testing.assert_allclose(g.logfc, o.lfc, rtol=LFC_RTOL, atol=LFC_ATOL)
    np.testing.assert_array_equal(g.de, o.de)
    np.testing.assert_array_equal(g.union, o.union)
    return g, o


def test_slow_config_a_subset(eng, cfg_a):
    d, X, names, code = cfg_a
    Xs = X[:600]
    sub = synth.from_dense(Xs, d.labels)
    ds = eng.dataset_csc(sub.indptr, sub.indices, sub.data, sub.G, sub.N)
    g, o = _slow_compare(eng, ds, Xs, code, len(names))
    assert len(o.union) > 0


def test_slow_many_clusters(eng):
    """SLOW tests every pair: P = 1225 (config D's K = 50) is past the wave
    kernel's 1024 tested pairs, so every bucket goes to the LDS items."""
    d = synth.generate("A", G=120, N=3000, K=50, seed=9)
    names, code = api.select_clusters(d.labels, 10)
    assert len(names) == 50
    ds = eng.dataset_csc(d.indptr, d.indices, d.data, d.G, d.N)
    _slow_compare(eng, ds, d.dense(), code, len(names))


def test_slow_edge_fixture(eng, edge):
    d, X, names, code = edge
    ds = eng.dataset_csc(d.indptr, d.indices, d.data, d.G, d.N)
    _slow_compare(eng, ds, X, code, len(names), qthr=0.2, fc=1.2, msf=0.5)


def test_repeat_is_bitwise_deterministic(eng, cfg_a):
    from scconsensus_amd import _native as nat
    d, X, names, code = cfg_a
    ds = eng.dataset_csc(d.indptr, d.indices, d.data, d.G, d.N)
    a = eng.de_run(ds, code, len(names), nat.SCC_DE_FAST, fetch="all")
    b = eng.de_run(ds, code, len(names), nat.SCC_DE_FAST, fetch="all")
    np.testing.assert_array_equal(a.p, b.p)
    np.testing.assert_array_equal(a.logfc, b.logfc)
    np.testing.assert_array_equal(a.union, b.union)


def test_invalid_inputs_fail_loudly(eng, cfg_a):
    from scconsensus_amd import _native as nat
    d, X, names, code = cfg_a
    ds = eng.dataset_csc(d.indptr, d.indices, d.data, d.G, d.N)
    bad = code.copy()
    bad[0] = len(names)
    with pytest.raises(nat.SccError):
        eng.de_run(ds, bad, len(names), nat.SCC_DE_FAST)
    vals = d.data.copy()
    vals[5] = np.nan
    ds2 = eng.dataset_csc(d.indptr, d.indices, vals, d.G, d.N)
    with pytest.raises(nat.SccError) as e:
        eng.de_run(ds2, code, len(names), nat.SCC_DE_FAST)
    assert e.value.code == nat.SCC_ERR_NONFINITE


def test_config_b_sampled_parity(eng):
    """PBMC-26k shape: exact U/ties/p on a seeded sample of (pair, gene) cells
    against the oracle's R-style rank sums, plus full-size properties."""
    from scconsensus_amd import _native as nat
    d = synth.generate("B")
    names, code = api.select_clusters(d.labels, 10)
    K = len(names)
    ds = eng.dataset_csc(d.indptr, d.indices, d.data, d.G, d.N)
    g = eng.de_run(ds, code, K, nat.SCC_DE_FAST, fetch="all")
    n = np.bincount(code[code >= 0], minlength=K).astype(np.int64)
    pairs = [(i, j) for i in range(K - 1) for j in range(i + 1, K)]
    nn = np.array([n[i] * n[j] for i, j in pairs])
    assert np.all(g.u2 >= 0) and np.all(g.u2 <= 2 * nn[:, None])
    csr = d.scipy_csc().tocsr()
    rng = np.random.default_rng(0)
    for _ in range(60):
        p = int(rng.integers(len(pairs)))
        gene = int(rng.integers(d.G))
        i, j = pairs[p]
        row = np.asarray(csr[gene].todense()).ravel()
        po, W, T, _ = O.wilcox_test(row[code == i], row[code == j])
        assert g.u2[p, gene] == int(round(2 * W))
        if np.isnan(po):  # gene zero in both clusters: R's p.value is NaN too
            assert np.isnan(g.p[p, gene])
        else:
            assert g.p[p, gene] == pytest.approx(po, rel=P_RTOL)
    assert 100 < len(g.union) <= 30 * len(pairs) * 2


def _near_tie_dataset(seed=5):
    """Genes whose values differ only in the last bits next to far larger
    values: the rank kernel's 32-bit key window merges them (mixed runs of
    <= 64 and > 64 elements) and must restore the exact order."""
    rng = np.random.default_rng(seed)
    K, per = 4, 60
    labels = np.repeat(np.array(["red", "blue", "green", "cyan"], dtype=object), per)
    rng.shuffle(labels)
    N = len(labels)
    G = 6
    X = np.zeros((G, N))
    one = np.nextafter(1.0, 2.0) - 1.0
    # gene 0: 20 near-equal values + a far value (short mixed runs)
    idx = rng.choice(N, 40, replace=False)
    X[0, idx[:20]] = 1.0 + one * rng.permutation(20)
    X[0, idx[20:]] = rng.uniform(0.1, 20.0, 20)
    # gene 1: 150 near-equal values + far values (a run > 64: full re-sort)
    idx = rng.choice(N, 200, replace=False)
    X[1, idx[:150]] = 2.0 + 2 * one * rng.permutation(150)
    X[1, idx[150:]] = rng.uniform(1e-3, 20.0, 50)
    # gene 2: exact ties mixed with near ties
    idx = rng.choice(N, 120, replace=False)
    X[2, idx] = np.where(rng.random(120) < 0.5, 3.0, 3.0 + one * 2 * rng.integers(1, 4, 120))
    X[2, idx[:5]] = 15.0
    # gene 3: negative and positive with tiny separations
    idx = rng.choice(N, 100, replace=False)
    X[3, idx] = rng.choice([-1.0, -1.0 - one, 1.0, 1.0 + one, 1e-300, -1e-300, 15.0], 100)
    # genes 4, 5: ordinary
    X[4] = np.where(rng.random(N) < 0.4, rng.gamma(2.0, 1.0, N), 0.0)
    X[5] = np.where(rng.random(N) < 0.9, np.round(rng.gamma(2.0, 1.0, N), 1), 0.0)
    return synth.from_dense(X, labels), X


def test_near_ties_exact_order(eng):
    from scconsensus_amd import _native as nat
    d, X = _near_tie_dataset()
    names, code = api.select_clusters(d.labels, 10)
    K = len(names)
    ds = eng.dataset_csc(d.indptr, d.indices, d.data, d.G, d.N)
    g = eng.de_run(ds, code, K, nat.SCC_DE_FAST, fetch="all")
    for p, (i, j) in enumerate([(i, j) for i in range(K - 1) for j in range(i + 1, K)]):
        for gene in range(d.G):
            po, W, T, _ = O.wilcox_test(X[gene, code == i], X[gene, code == j])
            assert g.u2[p, gene] == int(round(2 * W)), (p, gene)
            if np.isnan(po):
                assert np.isnan(g.p[p, gene])
            else:
                assert g.p[p, gene] == pytest.approx(po, rel=1e-12), (p, gene)
    _fast_compare(eng, ds, X, code, K, log_fc_thrs=0.01, min_per_cent=1.0)


@pytest.mark.parametrize("caps", [("64", "256"), ("128", "128")])
def test_rank_size_classes(eng, cfg_a, caps, monkeypatch):
    """Small caps push most genes to the 1024-thread LDS class and the
    HBM-resident class: same results bit for bit."""
    monkeypatch.setenv("SCC_CAP_SMALL", caps[0])
    monkeypatch.setenv("SCC_CAP_MEDIUM", caps[1])
    d, X, names, code = cfg_a
    ds = eng.dataset_csc(d.indptr, d.indices, d.data, d.G, d.N)
    _fast_compare(eng, ds, X, code, len(names))


def _dense_stretch_matrix(seed=21, G=40, N=3000, K=6, frac=0.9, nested=0):
    """Genes whose nonzeros crowd a narrow stretch of the value axis (relative
    width 1e-7) next to a few large outliers: the split's 2048-bin window puts
    the whole stretch in one bin of > 64 distinct values, which k_rank_resplit
    splits again.  Some genes are rounded to a grid (ties inside the stretch)."""
    rng = np.random.default_rng(seed)
    lab = rng.integers(0, K, N)
    names = np.array(synth.label_names(K), dtype=object)
    X = np.zeros((G, N))
    for g in range(G):
        m = rng.random(N) < frac
        v = 1.0 + rng.random(N) * 1e-7 * (1 + g % 5) + lab * 2e-8 * (g % 3)
        if g % 4 == 3:
            v = np.round(v, 9)
        X[g, m] = v[m]
        if nested:  # a tighter stretch inside the stretch: one re-split bin of > 64 distinct values
            idx = rng.choice(N, nested, replace=False)
            X[g, idx] = 1.0 + 5e-8 + rng.permutation(nested) * 1e-15 * (1 + g % 3)
        out = rng.random(N) < 0.01
        X[g, out] = 50.0 + rng.random(out.sum())
    return synth.from_dense(X, names[lab]), X


@pytest.mark.parametrize("frac", [0.9, 0.07])
@pytest.mark.parametrize("resplit,cross_wave", [("1", "0"), ("0", "0"), ("1", "1")])
def test_resplit_dense_value_stretch(eng, resplit, cross_wave, frac, monkeypatch):
    """Exact U / ties with and without the re-split route (SCC_RESPLIT=0: the
    fat buckets go to the LDS items as before); stretches of ~2700 elements
    (workgroup re-split) and ~210 (one wave per parent)."""
    monkeypatch.setenv("SCC_RESPLIT", resplit)
    monkeypatch.setenv("SCC_CROSS_WAVE", cross_wave)
    d, X = _dense_stretch_matrix(frac=frac)
    names, code = api.select_clusters(d.labels, 10)
    ds = eng.dataset_csc(d.indptr, d.indices, d.data, d.G, d.N)
    _slow_compare(eng, ds, X, code, len(names))
    _fast_compare(eng, ds, X, code, len(names), min_per_cent=5.0, log_fc_thrs=0.0)


@pytest.mark.parametrize("frac", [0.02, 0.07])
def test_resplit_second_level(eng, frac):
    """A sub-bucket of the first re-split that still holds > 64 distinct values
    goes to the second re-split level (from the wave re-split at ~210 elements
    per stretch, from the workgroup re-split at ~360)."""
    d, X = _dense_stretch_matrix(frac=frac, nested=150)
    names, code = api.select_clusters(d.labels, 10)
    ds = eng.dataset_csc(d.indptr, d.indices, d.data, d.G, d.N)
    _slow_compare(eng, ds, X, code, len(names))
    _fast_compare(eng, ds, X, code, len(names), min_per_cent=1.0, log_fc_thrs=0.0)

