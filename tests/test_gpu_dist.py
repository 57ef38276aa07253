"""GPU parity of stage 3 (cell x cell distance) against the numpy oracle.

Bar: distance entries within 1e-5 absolute (BASELINE.json north_star).  The
PCA oracle is the exact truncated SVD (irlba's target)."""
import numpy as np
import pytest

import oracle as O
from scconsensus_amd import api, synth

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def eng():
    from scconsensus_amd import _native
    return _native.Engine(0)


@pytest.fixture(scope="module")
def cfg_a():
    d = synth.generate("A")
    names, code = api.select_clusters(d.labels, 10)
    X = d.dense()
    o = O.de_fast(X, code, len(names))
    return d, X, o.union


def test_pca_euclid_matches_exact_svd(eng, cfg_a):
    from scconsensus_amd import _native as nat
    d, X, uni = cfg_a
    ds = eng.dataset_csc(d.indptr, d.indices, d.data, d.G, d.N)
    dist = eng.distance(ds, uni, nat.SCC_DIST_PCA_EUCLID)
    ref = O.dist_euclidean(O.pca_scores(X, uni))
    assert dist.shape == ref.shape
    err = np.max(np.abs(dist - ref))
    assert err < 1e-5, err
    # scores span the same subspace (signs arbitrary)
    S = eng.last_pca_scores(d.N)
    R = O.pca_scores(X, uni)
    for q in range(S.shape[1]):
        assert min(np.max(np.abs(S[:, q] - R[:, q])), np.max(np.abs(S[:, q] + R[:, q]))) < 1e-5 * max(
            1.0, np.max(np.abs(R[:, q]))) or q >= 7  # noise-level components may rotate inside near-degenerate pairs


def test_pca_euclid_fp32_output(eng, cfg_a):
    from scconsensus_amd import _native as nat
    d, X, uni = cfg_a
    ds = eng.dataset_csc(d.indptr, d.indices, d.data, d.G, d.N)
    d64 = eng.distance(ds, uni, nat.SCC_DIST_PCA_EUCLID)
    d32 = eng.distance(ds, uni, nat.SCC_DIST_PCA_EUCLID, f32=True)
    np.testing.assert_allclose(d32, d64, rtol=1e-6, atol=1e-6)


def test_pca_small_union_and_dense_input(eng, cfg_a):
    from scconsensus_amd import _native as nat
    d, X, uni = cfg_a
    small = uni[:9]  # |U| < 15 -> n = |U| components
    ds = eng.dataset_dense(X)
    dist = eng.distance(ds, small, nat.SCC_DIST_PCA_EUCLID)
    ref = O.dist_euclidean(O.pca_scores(X, small))
    assert np.max(np.abs(dist - ref)) < 1e-5


def test_pearson_matches_numpy(eng, cfg_a):
    from scconsensus_amd import _native as nat
    d, X, uni = cfg_a
    ds = eng.dataset_csc(d.indptr, d.indices, d.data, d.G, d.N)
    dist = eng.distance(ds, uni, nat.SCC_DIST_PEARSON)
    ref = O.dist_pearson(X, uni)
    assert np.max(np.abs(dist - ref)) < 1e-5


def test_pearson_nontemporal_bitwise(eng, cfg_a, monkeypatch):
    """Nontemporal epilogue stores (SCC_PEARSON_NT=1, off by default) store
    the same values: identical bits."""
    from scconsensus_amd import _native as nat
    d, X, uni = cfg_a
    ds = eng.dataset_csc(d.indptr, d.indices, d.data, d.G, d.N)
    a = eng.distance(ds, uni, nat.SCC_DIST_PEARSON)
    monkeypatch.setenv("SCC_PEARSON_NT", "1")
    b = eng.distance(ds, uni, nat.SCC_DIST_PEARSON)
    assert np.array_equal(a, b)


def test_dist_packed_order_small(eng):
    """R dist order on a tiny hand case: (1,0),(2,0),(3,0),(2,1),(3,1),(3,2)."""
    from scconsensus_amd import _native as nat
    X = np.array([[0.0, 1.0, 3.0, 6.0], [0.0, 0.0, 0.0, 0.0], [1.0, 1.0, 1.0, 1.0]])
    ds = eng.dataset_dense(X)
    dist = eng.distance(ds, np.array([0, 2]), nat.SCC_DIST_PCA_EUCLID)
    np.testing.assert_allclose(dist, [1, 3, 6, 2, 5, 3], atol=1e-12)


@pytest.mark.parametrize("n", [2, 3, 5, 8, 17, 40, 130, 255, 256, 257, 323, 700])
def test_eigensolver_sizes(eng, n, monkeypatch):
    """Multi-workgroup tridiagonalisation + per-eigenpair vectors at many |U|
    (workgroup counts 2..70, rows in registers or LDS) against numpy's exact
    SVD."""
    from scconsensus_amd import _native as nat
    monkeypatch.setenv("SCC_EIG_SI", "0")  # the direct solvers (subspace iteration: its own tests)
    monkeypatch.setenv("SCC_EIG_FSI", "0")
    rng = np.random.default_rng(100 + n)
    X = rng.standard_normal((n, 300)) * np.linspace(2.0, 0.5, n)[:, None]
    ds = eng.dataset_dense(X)
    g = np.arange(n)
    dist = eng.distance(ds, g, nat.SCC_DIST_PCA_EUCLID)
    ref = O.dist_euclidean(O.pca_scores(X, g))
    assert np.max(np.abs(dist - ref)) < 1e-5


def test_eigensolver_repeated_eigenvalues(eng):
    """Exactly repeated eigenvalues inside the top 15 (cluster re-orthogonalisation);
    the 15/16 boundary itself is well separated so the distance is defined."""
    from scconsensus_amd import _native as nat
    rng = np.random.default_rng(7)
    n, N = 40, 500
    sv = np.array([9.0] * 3 + [7.0] * 4 + [5.0] * 2 + [4.0] * 6 + [1.0] * (n - 15))
    Q, _ = np.linalg.qr(rng.standard_normal((N, n)))
    Q -= Q.mean(axis=0)  # centred cells -> the Gram is exactly V diag(sv^2) V'
    V, _ = np.linalg.qr(rng.standard_normal((n, n)))
    M = Q @ np.diag(sv) @ V.T  # cells x genes
    X = M.T
    ds = eng.dataset_dense(X)
    g = np.arange(n)
    dist = eng.distance(ds, g, nat.SCC_DIST_PCA_EUCLID)
    ref = O.dist_euclidean(O.pca_scores(X, g))
    assert np.max(np.abs(dist - ref)) < 1e-5


def test_eigensolver_rows_beyond_lds(eng, monkeypatch):
    """|U| = 2100: each workgroup's rows no longer fit its LDS (global row store)."""
    from scconsensus_amd import _native as nat
    monkeypatch.setenv("SCC_EIG_SI", "0")
    monkeypatch.setenv("SCC_EIG_FSI", "0")
    rng = np.random.default_rng(11)
    n, N = 2100, 1200
    X = rng.standard_normal((n, N)) * np.linspace(3.0, 0.5, n)[:, None]
    X[:20] += rng.standard_normal((20, 1)) * rng.standard_normal((1, N)) * 4.0  # a few spikes
    ds = eng.dataset_dense(X)
    g = np.arange(n)
    dist = eng.distance(ds, g, nat.SCC_DIST_PCA_EUCLID)
    ref = O.dist_euclidean(O.pca_scores(X, g))
    assert np.max(np.abs(dist - ref)) < 1e-5


def test_rank_deficient_and_repeated(eng, monkeypatch):
    """Identical genes (zero-norm columns: tau = 0 reflectors) and exactly
    repeated eigenvalues inside the top 15, n = 90 and 300."""
    from scconsensus_amd import _native as nat
    monkeypatch.setenv("SCC_EIG_SI", "0")
    monkeypatch.setenv("SCC_EIG_FSI", "0")
    for n in (90, 300):
        rng = np.random.default_rng(8 + n)
        N = 700
        sv = np.array([9.0] * 3 + [7.0] * 4 + [5.0] * 2 + [4.0] * 6 + [1.0] * (n - 15))
        Q, _ = np.linalg.qr(rng.standard_normal((N, n)))
        Q -= Q.mean(axis=0)
        V, _ = np.linalg.qr(rng.standard_normal((n, n)))
        X = (Q @ np.diag(sv) @ V.T).T
        ds = eng.dataset_dense(X)
        g = np.arange(n)
        assert np.max(np.abs(eng.distance(ds, g, nat.SCC_DIST_PCA_EUCLID) - O.dist_euclidean(O.pca_scores(X, g)))) < 1e-5
        X2 = np.concatenate([X[: n // 3]] * 3)  # rank <= n / 3
        ds2 = eng.dataset_dense(X2)
        dist = eng.distance(ds2, g, nat.SCC_DIST_PCA_EUCLID)
        assert np.max(np.abs(dist - O.dist_euclidean(O.pca_scores(X2, g)))) < 1e-5


@pytest.mark.parametrize("xcd", ["0", "1"])
@pytest.mark.parametrize("n,nwg", [(323, 8), (323, 32), (323, 64), (500, 48), (700, 70), (700, 256), (1500, 40),
                                   (1500, 150), (2100, 210)])
def test_eigensolver_workgroup_counts(eng, n, nwg, xcd, monkeypatch):
    """Same eigenpairs for any number of tridiagonalisation workgroups, either
    hand-off (cross-XCD write-through or one-XCD L2), rows in LDS or in HBM."""
    from scconsensus_amd import _native as nat
    monkeypatch.setenv("SCC_EIG_SI", "0")
    monkeypatch.setenv("SCC_EIG_FSI", "0")
    monkeypatch.setenv("SCC_EIG_NWG", str(nwg))
    monkeypatch.setenv("SCC_EIG_XCD", xcd)
    rng = np.random.default_rng(11)
    X = rng.standard_normal((n, 900)) * np.linspace(3.0, 0.5, n)[:, None]
    X[:20] += rng.standard_normal((20, 1)) * rng.standard_normal((1, 900)) * 4.0
    ds = eng.dataset_dense(X)
    g = np.arange(n)
    dist = eng.distance(ds, g, nat.SCC_DIST_PCA_EUCLID)
    ref = O.dist_euclidean(O.pca_scores(X, g))
    assert np.max(np.abs(dist - ref)) < 1e-5


@pytest.mark.parametrize("n", [3, 17, 64, 150, 323, 354, 400])
def test_back_transformations_agree(eng, n, monkeypatch):
    """The three back-transformations of the tridiagonal's eigenvectors give
    the same PCA: the explicit Q formed beside the eigenvector kernel, then
    Z = Q Y (SCC_EIG_BT=2, default where it fits), the one-workgroup blocked
    k_tri_back (1) and the per-eigenpair one (0); all against the exact SVD."""
    from scconsensus_amd import _native as nat
    monkeypatch.setenv("SCC_EIG_SI", "0")
    monkeypatch.setenv("SCC_EIG_FSI", "0")
    rng = np.random.default_rng(600 + n)
    X = rng.standard_normal((n, 800)) * np.linspace(3.0, 0.5, n)[:, None]
    X[: min(n, 12)] += rng.standard_normal((min(n, 12), 1)) * rng.standard_normal((1, 800)) * 3.0
    ds = eng.dataset_dense(X)
    g = np.arange(n)
    ref = O.dist_euclidean(O.pca_scores(X, g))
    outs = []
    for bt in ("2", "1", "0"):
        monkeypatch.setenv("SCC_EIG_BT", bt)
        d = eng.distance(ds, g, nat.SCC_DIST_PCA_EUCLID)
        assert np.max(np.abs(d - ref)) < 1e-7, bt
        outs.append(d)
    assert np.max(np.abs(outs[0] - outs[1])) < 1e-9
    assert np.max(np.abs(outs[0] - outs[2])) < 1e-9


@pytest.mark.parametrize("n", [2, 3, 17, 64, 150, 323, 400])
def test_twisted_vectors_agree(eng, n, monkeypatch):
    """Eigenvectors from the twisted factorization (isolated eigenvalues, the
    default) and from inverse iteration (SCC_EIG_TWIST=0) give the same PCA,
    both equal to the exact SVD; config B's bulk-edge spacing (relative gaps
    ~3e-3 among eigenvalues 11..16) included."""
    from scconsensus_amd import _native as nat
    monkeypatch.setenv("SCC_EIG_SI", "0")
    monkeypatch.setenv("SCC_EIG_FSI", "0")
    rng = np.random.default_rng(700 + n)
    X = rng.standard_normal((n, 900)) * np.linspace(1.0, 0.97, n)[:, None]  # a near-flat bulk
    X[: min(n, 10)] += rng.standard_normal((min(n, 10), 1)) * rng.standard_normal((1, 900)) * 3.0
    ds = eng.dataset_dense(X)
    g = np.arange(n)
    ref = O.dist_euclidean(O.pca_scores(X, g))
    d1 = eng.distance(ds, g, nat.SCC_DIST_PCA_EUCLID)
    monkeypatch.setenv("SCC_EIG_TWIST", "0")
    d0 = eng.distance(ds, g, nat.SCC_DIST_PCA_EUCLID)
    assert np.max(np.abs(d1 - ref)) < 1e-5
    assert np.max(np.abs(d0 - ref)) < 1e-5
    assert np.max(np.abs(d1 - d0)) < 1e-7


def test_workgroup_count_bitwise(eng, monkeypatch):
    """The tridiagonalisation's reductions have a fixed shape: 8, 20 or 32
    workgroups in the hand-off give the same distance bits."""
    from scconsensus_amd import _native as nat
    monkeypatch.setenv("SCC_EIG_SI", "0")
    monkeypatch.setenv("SCC_EIG_FSI", "0")
    rng = np.random.default_rng(21)
    n = 323
    X = rng.standard_normal((n, 900)) * np.linspace(3.0, 0.5, n)[:, None]
    ds = eng.dataset_dense(X)
    g = np.arange(n)
    outs = []
    for nwg in (8, 20, 32):
        monkeypatch.setenv("SCC_EIG_NWG", str(nwg))
        outs.append(eng.distance(ds, g, nat.SCC_DIST_PCA_EUCLID))
    assert all(np.array_equal(outs[0], o) for o in outs[1:])


@pytest.mark.parametrize("f32", [False, True])
def test_distance_kernels_agree(eng, f32, monkeypatch):
    """The distance store kernel's tile widths (64 / 128 columns), store
    kinds (plain / nontemporal), store widths (two entries per thread or
    one) and tile orders (folded grid / panel list) give bit-identical packed output (same
    arithmetic, only the store pattern differs), over the full vector and over
    column slices whose starts are not line-aligned."""
    from scconsensus_amd import _native as nat
    rng = np.random.default_rng(41)
    G, N = 60, 1337
    X = np.abs(rng.standard_normal((G, N))) * (rng.random((G, N)) < 0.4)
    X[:, 7] = X[:, 8]  # two identical cells: a zero distance (difference form)
    ds = eng.dataset_dense(X)
    g = np.arange(0, G, 2)
    outs = []
    for cols, nt, v2, order in [("64", "1", "1", "0"), ("64", "0", "1", "0"), ("128", "1", "1", "0"),
                                ("128", "0", "1", "0"), ("64", "1", "0", "0"), ("128", "0", "0", "0"),
                                ("64", "1", "1", "1"), ("128", "1", "1", "1")]:
        monkeypatch.setenv("SCC_DIST_COLS", cols)
        monkeypatch.setenv("SCC_DIST_NT", nt)
        monkeypatch.setenv("SCC_DIST_V2", v2)  # paired stores (default) or one entry per thread
        monkeypatch.setenv("SCC_DIST_ORDER", order)  # panel-ordered tile list (default from 64k cells)
        outs.append(eng.distance(ds, g, nat.SCC_DIST_PCA_EUCLID, f32=f32))
    monkeypatch.setenv("SCC_DIST_NT", "1")
    monkeypatch.setenv("SCC_DIST_V2", "1")
    monkeypatch.setenv("SCC_DIST_ORDER", "1")
    assert all(np.array_equal(outs[0], o) for o in outs[1:])
    ref = O.dist_euclidean(O.pca_scores(X, g))
    assert np.max(np.abs(outs[0] - ref)) < (1e-4 if f32 else 1e-5)
    assert outs[0][7 * (2 * N - 7 - 1) // 2] == 0.0  # pair (8, 7)
    for c_lo, c_hi in [(5, 77), (700, 1336)]:
        lo = c_lo * (2 * N - c_lo - 1) // 2
        hi = c_hi * (2 * N - c_hi - 1) // 2
        for cols in ["64", "128"]:
            monkeypatch.setenv("SCC_DIST_COLS", cols)
            part = eng.distance_cols(ds, g, c_lo, c_hi, nat.SCC_DIST_PCA_EUCLID, f32=f32)
            assert np.array_equal(part, outs[0][lo:hi])


def _spiky(n, N, nspike, seed):
    """Genes x cells with `nspike` cluster-like directions well above a noise
    bulk (the many-cluster spectrum of configs C/D)."""
    rng = np.random.default_rng(seed)
    X = rng.standard_normal((n, N)) * 0.5
    lab = rng.integers(0, nspike, N)
    M = rng.standard_normal((n, nspike)) * np.linspace(4.0, 1.5, nspike)[None, :]
    return X + M[:, lab]


@pytest.mark.parametrize("n", [450, 845, 1200])
def test_subspace_iteration(eng, n, monkeypatch, capfd):
    """Block subspace iteration (scc_subspace.hip, tried first for |U| >= 400)
    on a many-cluster spectrum: accepted (its residual test passes), equal to
    the exact SVD and to the direct solver, bit-identical from run to run."""
    monkeypatch.setenv("SCC_EIG_FSI", "0")  # the block subspace iteration itself
    from scconsensus_amd import _native as nat
    monkeypatch.setenv("SCC_EIG_SI_LOG", "1")
    X = _spiky(n, 3000, 40, 900 + n)
    ds = eng.dataset_dense(X)
    g = np.arange(n)
    d1 = eng.distance(ds, g, nat.SCC_DIST_PCA_EUCLID)
    S1 = eng.last_pca_scores(X.shape[1])
    d1b = eng.distance(ds, g, nat.SCC_DIST_PCA_EUCLID)
    err = capfd.readouterr().err
    assert f"[scc si] n={n}" in err and "flag=0 inner=0" in err, err
    assert np.array_equal(d1, d1b)
    ref = O.dist_euclidean(O.pca_scores(X, g))
    assert np.max(np.abs(d1 - ref)) < 1e-5
    monkeypatch.setenv("SCC_EIG_SI", "0")
    monkeypatch.setenv("SCC_EIG_FSI", "0")
    d0 = eng.distance(ds, g, nat.SCC_DIST_PCA_EUCLID)
    S0 = eng.last_pca_scores(X.shape[1])
    assert np.max(np.abs(d1 - d0)) < 1e-6
    np.testing.assert_allclose(S1, S0, rtol=0, atol=1e-7 * np.abs(S0).max())  # same sign rule


@pytest.mark.parametrize("case", ["bulk", "few_cells"])
def test_subspace_iteration_falls_back(eng, case, monkeypatch, capfd):
    """Slow convergence (15th eigenvalue inside a smooth bulk): the subspace
    result fails its residual test and the direct solver's answer is returned.
    A Gram of rank < 64 (40 cells): whichever path answers, the distance is the
    exact SVD's."""
    monkeypatch.setenv("SCC_EIG_FSI", "0")  # the block subspace iteration itself
    from scconsensus_amd import _native as nat
    monkeypatch.setenv("SCC_EIG_SI_LOG", "1")
    rng = np.random.default_rng(77)
    n = 500
    N = 2000 if case == "bulk" else 40
    X = rng.standard_normal((n, N)) * np.linspace(1.0, 0.9, n)[:, None]
    ds = eng.dataset_dense(X)
    g = np.arange(n)
    dist = eng.distance(ds, g, nat.SCC_DIST_PCA_EUCLID)
    err = capfd.readouterr().err
    assert f"[scc si] n={n}" in err, err
    if case == "bulk":
        assert "flag=0 inner=0" not in err, err
    ref = O.dist_euclidean(O.pca_scores(X, g))
    assert np.max(np.abs(dist - ref)) < 1e-5


def test_subspace_guard_catches_missed_eigenpair(eng, monkeypatch, capfd):
    """the residual test alone accepts Ritz pairs that are exact
    eigenpairs but not the TOP ones.  A block-diagonal Gram (genes 0..399 and
    400..499 on disjoint cells, zero-mean rows: centring keeps the blocks
    apart) whose second block holds the largest eigenvalue, with the start
    block's rows >= 400 zeroed (test hook): the iteration never sees that
    block, every residual passes, and the deflated power check (flag bit 8)
    must reject the result so the direct solver answers."""
    monkeypatch.setenv("SCC_EIG_FSI", "0")  # the block subspace iteration itself
    from scconsensus_amd import _native as nat
    rng = np.random.default_rng(12)
    n, N = 500, 3000
    X = np.zeros((n, N))
    X[:400, :1500] = _spiky(400, 1500, 30, 5)
    X[400:, 1500:] = rng.standard_normal((100, 1500)) * 0.3
    X[400:, 1500:] += rng.standard_normal((100, 1)) * rng.standard_normal((1, 1500)) * 40.0  # the top eigenvalue
    X[:400, :1500] -= X[:400, :1500].mean(axis=1, keepdims=True)
    X[400:, 1500:] -= X[400:, 1500:].mean(axis=1, keepdims=True)
    ds = eng.dataset_dense(X)
    g = np.arange(n)
    monkeypatch.setenv("SCC_EIG_SI_LOG", "1")
    monkeypatch.setenv("SCC_EIG_SI_INIT_ROWS", "400")
    dist = eng.distance(ds, g, nat.SCC_DIST_PCA_EUCLID)
    err = capfd.readouterr().err
    assert f"[scc si] n={n}" in err, err
    flag = int(err.split("flag=")[1].split()[0])
    assert flag & 8 and not flag & 2, err  # residuals passed, the guard rejected
    ref = O.dist_euclidean(O.pca_scores(X, g))
    assert np.max(np.abs(dist - ref)) < 1e-5
    monkeypatch.delenv("SCC_EIG_SI_INIT_ROWS")
    d2 = eng.distance(ds, g, nat.SCC_DIST_PCA_EUCLID)  # the normal start (whichever path answers)
    assert np.max(np.abs(d2 - ref)) < 1e-5


def test_repeat_bitwise_config_b(eng):
    """the same config-B job twice gives the same `dist` bits
    (every reduction has a fixed order; the tridiagonalisation's sums do not
    depend on how many workgroups joined its hand-off)."""
    from scconsensus_amd import _native as nat
    from scconsensus_amd import api, synth
    d = synth.generate("B")
    names, code = api.select_clusters(d.labels, 10)
    ds = eng.dataset_csc(d.indptr, d.indices, d.data, d.G, d.N)
    uni = eng.de_run(ds, code, len(names), nat.SCC_DE_FAST, fetch="union").union
    first = eng.distance(ds, uni)
    for _ in range(2):
        again = eng.distance(ds, uni)
        assert np.array_equal(first, again)


def test_gather_wide_union_fallback(eng):
    """A union wider than four LDS rows (|U| > 2048: the CSC gather's direct
    store path, whole matrix zeroed first) and a narrow one (rows assembled in
    LDS, only padding rows zeroed) both give the exact-SVD distance."""
    import scipy.sparse as sp
    from scconsensus_amd import _native as nat
    rng = np.random.default_rng(5)
    G, N = 2100, 300
    X = sp.random(G, N, density=0.05, random_state=6, format="csc") * 4.0
    X.data = np.log1p(X.data)
    Xd = X.toarray()
    ds = eng.dataset_csc(X.indptr.astype(np.int64), X.indices.astype(np.int32), X.data, G, N)
    for g in (np.arange(G), np.sort(rng.choice(G, 150, replace=False))):
        d = eng.distance(ds, g.astype(np.int32), nat.SCC_DIST_PCA_EUCLID)
        ref = O.dist_euclidean(O.pca_scores(Xd, g))
        assert np.max(np.abs(d - ref)) < 1e-5


@pytest.mark.parametrize("ld_genes", [150, 700])
def test_gather_workgroup_sizes_bitwise(eng, monkeypatch, ld_genes):
    """The LDS-map gather with 4, 8 and 16 waves per workgroup (its default
    picks the most resident waves per CU) and the per-cell gather without the
    map: the same distance bits (the gather only copies values)."""
    import scipy.sparse as sp
    from scconsensus_amd import _native as nat
    rng = np.random.default_rng(9)
    G, N = 3000, 1700
    X = sp.random(G, N, density=0.08, random_state=10, format="csc") * 4.0
    X.data = np.log1p(X.data)
    ds = eng.dataset_csc(X.indptr.astype(np.int64), X.indices.astype(np.int32), X.data, G, N)
    g = np.sort(rng.choice(G, ld_genes, replace=False)).astype(np.int32)
    monkeypatch.setenv("SCC_GATHER_LM", "0")
    base = eng.distance(ds, g, nat.SCC_DIST_PCA_EUCLID)
    monkeypatch.delenv("SCC_GATHER_LM")
    for w in ("4", "8", "16", None):
        if w is None:
            monkeypatch.delenv("SCC_GATHER_W", raising=False)
        else:
            monkeypatch.setenv("SCC_GATHER_W", w)
        assert np.array_equal(eng.distance(ds, g, nat.SCC_DIST_PCA_EUCLID), base), w


def test_de_distance_matches_two_calls(eng, cfg_a):
    """scc_de_distance (DE, then the distance over its union, one C call)
    returns the same union and the same distance bits as scc_de_run followed
    by scc_distance."""
    from scconsensus_amd import _native as nat
    from scconsensus_amd import api
    d, X, uni = cfg_a
    names, code = api.select_clusters(d.labels, 10)
    ds = eng.dataset_csc(d.indptr, d.indices, d.data, d.G, d.N)
    r1 = eng.de_run(ds, code, len(names), nat.SCC_DE_FAST, fetch="union")
    d1 = eng.distance(ds, r1.union, nat.SCC_DIST_PCA_EUCLID)
    r2, d2 = eng.de_distance(ds, code, len(names), nat.SCC_DE_FAST, nat.SCC_DIST_PCA_EUCLID)
    assert np.array_equal(r1.union, r2.union)
    assert np.array_equal(np.asarray(r2.union), np.asarray(uni))
    assert np.array_equal(d1, d2)


@pytest.mark.parametrize("engine", ["1", "0"])
def test_filtered_guard_catches_missed_eigenpair(eng, monkeypatch, capfd, engine):
    """The same hidden top eigenvalue for the filtered subspace iteration, with
    the filter loop, Rayleigh-Ritz and the guard inside the persistent engine
    (engine=1) and as a launch per step (engine=0): the guard (flag bit 8)
    rejects, the direct solver answers."""
    from scconsensus_amd import _native as nat
    rng = np.random.default_rng(12)
    n, N = 500, 3000
    X = np.zeros((n, N))
    X[:400, :1500] = _spiky(400, 1500, 30, 5)
    X[400:, 1500:] = rng.standard_normal((100, 1500)) * 0.3
    X[400:, 1500:] += rng.standard_normal((100, 1)) * rng.standard_normal((1, 1500)) * 40.0
    X[:400, :1500] -= X[:400, :1500].mean(axis=1, keepdims=True)
    X[400:, 1500:] -= X[400:, 1500:].mean(axis=1, keepdims=True)
    ds = eng.dataset_dense(X)
    g = np.arange(n)
    monkeypatch.setenv("SCC_EIG_FSI", "1")
    monkeypatch.setenv("SCC_EIG_FSI_ENGINE", engine)
    monkeypatch.setenv("SCC_EIG_SI_LOG", "1")
    monkeypatch.setenv("SCC_EIG_SI_INIT_ROWS", "400")
    dist = eng.distance(ds, g, nat.SCC_DIST_PCA_EUCLID)
    err = capfd.readouterr().err
    assert f"[scc fsi] n={n}" in err, err
    line = [x for x in err.splitlines() if x.startswith("[scc fsi]")][-1]
    assert f"engine={engine}" in line, line
    flag = int(line.split("flag=")[1].split()[0])
    # the filter's interval bound (32) and residuals (2) may reject too; the
    # guard (8) must fire on its own evidence
    assert flag & 8, line
    ref = O.dist_euclidean(O.pca_scores(X, g))
    assert np.max(np.abs(dist - ref)) < 1e-5
    monkeypatch.delenv("SCC_EIG_SI_INIT_ROWS")
    d2 = eng.distance(ds, g, nat.SCC_DIST_PCA_EUCLID)
    assert np.max(np.abs(d2 - ref)) < 1e-5


@pytest.mark.parametrize("n", [130, 257, 323, 500, 672, 700, 1000])
def test_eigensolver_sizes_default_path(eng, n):
    """The default route (the filtered subspace iteration in the persistent
    engine for 128 <= |U| <= 672, the direct solver when it rejects) against
    numpy's exact SVD, the same matrices as test_eigensolver_sizes."""
    from scconsensus_amd import _native as nat
    rng = np.random.default_rng(100 + n)
    X = rng.standard_normal((n, 300)) * np.linspace(2.0, 0.5, n)[:, None]
    ds = eng.dataset_dense(X)
    g = np.arange(n)
    dist = eng.distance(ds, g, nat.SCC_DIST_PCA_EUCLID)
    ref = O.dist_euclidean(O.pca_scores(X, g))
    assert np.max(np.abs(dist - ref)) < 1e-5


@pytest.mark.parametrize("nu", [37, 200, 450])
def test_scores_kernels_agree(eng, nu, monkeypatch):
    """Scores on fp64 MFMA (default) against the one-thread-per-cell loop: the
    same products in another summation order (1e-12 relative on the
    distance), and both against the exact SVD at the 1e-5 bar."""
    from scconsensus_amd import _native as nat
    rng = np.random.default_rng(nu + 1)
    G, N = 600, 2011
    X = np.abs(rng.standard_normal((G, N))) * (rng.random((G, N)) < 0.3)
    ds = eng.dataset_dense(X)
    g = np.sort(rng.choice(G, nu, replace=False))
    outs = []
    for mf in ("1", "0"):
        monkeypatch.setenv("SCC_SCORES_MFMA", mf)
        outs.append(eng.distance(ds, g, nat.SCC_DIST_PCA_EUCLID))
    np.testing.assert_allclose(outs[0], outs[1], rtol=1e-12, atol=1e-12)
    ref = O.dist_euclidean(O.pca_scores(X, g))
    assert np.max(np.abs(outs[0] - ref)) < 1e-5
