"""Gene-major CSR input (scc_dataset_create_csr, BASELINE config E's input
format): the device transpose gives the same resident dgCMatrix, so every DE
and distance result is bit-identical to the CSC path, which is checked
against the oracle in test_gpu_de.py / test_gpu_dist.py.  Parity against the
oracle is also checked directly on config A."""
import numpy as np
import pytest
import scipy.sparse as sp
import torch  # before the engine loads: torch's HIP runtime initialises first (as in test_gpu_shard)

import oracle as O
from scconsensus_amd import api, synth

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def eng():
    from scconsensus_amd import _native
    return _native.Engine(0)


def _csr_of(d):
    m = d.scipy_csc().tocsr()
    m.sort_indices()
    return m


def _same_de(a, b):
    np.testing.assert_array_equal(a.rows.gene, b.rows.gene)
    np.testing.assert_array_equal(a.rows.u2, b.rows.u2)
    np.testing.assert_array_equal(a.rows.ties, b.rows.ties)
    np.testing.assert_array_equal(a.rows.p, b.rows.p)
    np.testing.assert_array_equal(a.rows.avg_logfc, b.rows.avg_logfc)
    np.testing.assert_array_equal(a.union, b.union)


def test_csr_matches_csc_and_oracle(eng):
    from scconsensus_amd import _native as nat
    d = synth.generate("A")
    names, code = api.select_clusters(d.labels, 10)
    K = len(names)
    m = _csr_of(d)
    ds_r = eng.dataset_csr(m.indptr, m.indices, m.data, d.G, d.N)
    ds_c = eng.dataset_csc(d.indptr, d.indices, d.data, d.G, d.N)
    gr = eng.de_run(ds_r, code, K, nat.SCC_DE_FAST, fetch="rows")
    gc = eng.de_run(ds_c, code, K, nat.SCC_DE_FAST, fetch="rows")
    _same_de(gr, gc)
    o = O.de_fast(d.dense(), code, K)
    np.testing.assert_array_equal(gr.rows.u2, np.round(2 * o.row_W).astype(np.int64))
    np.testing.assert_allclose(gr.rows.p, o.row_p, rtol=1e-6, atol=0)
    np.testing.assert_array_equal(gr.union, o.union)
    dr = eng.distance(ds_r, gr.union, nat.SCC_DIST_PCA_EUCLID)
    dc = eng.distance(ds_c, gc.union, nat.SCC_DIST_PCA_EUCLID)
    np.testing.assert_array_equal(dr, dc)


def test_csr_slow_mode_and_empty_rows(eng):
    """Empty genes (all-zero rows) and cells without any value survive the transpose."""
    from scconsensus_amd import _native as nat
    d = synth.generate("A", G=300, N=700, K=4, seed=5)
    X = d.dense()
    X[[0, 7, 299], :] = 0.0          # empty rows
    X[:, [3, 500]] = 0.0             # empty cells
    sub = synth.from_dense(X, d.labels)
    names, code = api.select_clusters(sub.labels, 10)
    m = sp.csr_matrix(X)
    ds_r = eng.dataset_csr(m.indptr, m.indices, m.data, sub.G, sub.N)
    ds_c = eng.dataset_csc(sub.indptr, sub.indices, sub.data, sub.G, sub.N)
    a = eng.de_run(ds_r, code, len(names), nat.SCC_DE_SLOW, q_val_thrs=0.05, fc_thrs=1.5, fetch="all")
    b = eng.de_run(ds_c, code, len(names), nat.SCC_DE_SLOW, q_val_thrs=0.05, fc_thrs=1.5, fetch="all")
    np.testing.assert_array_equal(a.u2, b.u2)
    np.testing.assert_array_equal(a.p, b.p)
    np.testing.assert_array_equal(a.union, b.union)


def test_csr_device_pointers_match_host(eng):
    """The device-resident CSR path (what config E's GPU-generated input uses)."""
    from scconsensus_amd import _native as nat
    dd = synth.generate_device("A", "cuda:0", layout="csr")
    dc = synth.generate_device("A", "cuda:0", layout="csc")
    torch.cuda.synchronize()
    ds_r = eng.dataset_csr_device(dd.indptr.data_ptr(), dd.indices.data_ptr(), dd.data.data_ptr(), dd.G, dd.N, dd.nnz)
    ds_c = eng.dataset_csc_device(dc.indptr.data_ptr(), dc.indices.data_ptr(), dc.data.data_ptr(), dc.G, dc.N, dc.nnz)
    names, code = api.select_clusters(dd.labels, 10)
    a = eng.de_run(ds_r, code, len(names), nat.SCC_DE_FAST, fetch="rows")
    b = eng.de_run(ds_c, code, len(names), nat.SCC_DE_FAST, fetch="rows")
    _same_de(a, b)


def test_csr_bad_column_fails_loudly(eng):
    from scconsensus_amd import _native as nat
    indptr = np.array([0, 2, 3], np.int64)
    cols = np.array([0, 5, 1], np.int32)  # 5 >= N
    vals = np.ones(3)
    with pytest.raises(nat.SccError) as e:
        eng.dataset_csr(indptr, cols, vals, 2, 4)
    assert e.value.code == nat.SCC_ERR_INVALID
    with pytest.raises(nat.SccError):
        eng.dataset_csr(np.array([0, 2, 1], np.int64), np.array([0, 1, 2], np.int32), vals, 2, 4)


def test_api_accepts_scipy_csr(eng):
    d = synth.generate("A", G=400, N=900, K=5, seed=3)
    a = api.reclusterDEConsensusFast(d.scipy_csc().tocsr(), d.labels, deepSplitValues=(1,))
    b = api.reclusterDEConsensusFast(d.scipy_csc(), d.labels, deepSplitValues=(1,))
    assert a["deGeneUnion"] == b["deGeneUnion"]
    assert list(a["dynamicColors"]["deepsplit: 1"]) == list(b["dynamicColors"]["deepsplit: 1"])


# ---------------------------------------------------------------- the transpose itself
def _expect_csc(m):
    """scipy's own transpose of the CSR: the dgCMatrix R would hold."""
    c = m.tocsc()
    c.sort_indices()
    return c.indptr.astype(np.int64), c.indices.astype(np.int32), c.data


def _check_transpose(eng, m, G, N):
    ds = eng.dataset_csr(m.indptr, m.indices, m.data, G, N)
    ip, rows, vals = eng.read_csc(ds)
    eip, erows, evals = _expect_csc(m)
    np.testing.assert_array_equal(ip, eip)
    np.testing.assert_array_equal(rows, erows)
    np.testing.assert_array_equal(vals, evals)  # bit-identical (values are moved, never computed)
    ds.close()


@pytest.mark.parametrize("G,N,density,seed", [
    (1, 1, 1.0, 0), (1, 5000, 0.3, 1), (3000, 1, 0.5, 2), (257, 1025, 0.05, 3),
    (2000, 3000, 0.0325, 4), (600, 700, 1.0, 5), (5000, 20000, 0.002, 6), (300, 4000, 0.0, 7),
])
def test_transpose_bit_identical_to_scipy(eng, G, N, density, seed):
    """Shapes around the tile (256 genes), superblock and group edges, fully
    dense (pieces split in LDS), very sparse, empty."""
    rng = np.random.default_rng(seed)
    m = sp.random(G, N, density=density, format="csr", random_state=rng, dtype=np.float64)
    m.data = rng.standard_normal(m.nnz)
    m.sort_indices()
    _check_transpose(eng, m, G, N)


def test_transpose_dense_blocks_and_heavy_cells(eng):
    """A tile whose genes are dense over a superblock (the pass-1 piece is cut
    down to fit the LDS staging), a cell holding every gene and empty cells
    and genes (a pass-2 group past its staging, written in place)."""
    rng = np.random.default_rng(11)
    G, N = 30000, 2000
    m = sp.random(G, N, density=0.01, format="lil", random_state=rng, dtype=np.float64)
    m[256:512, 0:600] = rng.random((256, 600)) + 1.0  # dense region
    m[:, 1500] = (rng.random((G, 1)) + 2.0)           # a heavy cell: every gene
    m[:, 1700] = 0.0
    m[100, :] = 0.0
    m = sp.csr_matrix(m)
    m.eliminate_zeros()
    m.sort_indices()
    _check_transpose(eng, m, G, N)


def test_transpose_rejects_unsorted_and_repeated_columns(eng):
    from scconsensus_amd import _native as nat
    vals = np.ones(4)
    for cols in ([0, 2, 1, 3], [0, 1, 1, 3]):  # unsorted / repeated (gene, cell) in gene 0
        with pytest.raises(nat.SccError) as e:
            eng.dataset_csr(np.array([0, 3, 4], np.int64), np.array(cols, np.int32), vals, 2, 4)
        assert e.value.code == nat.SCC_ERR_INVALID
    with pytest.raises(nat.SccError) as e:  # negative column
        eng.dataset_csr(np.array([0, 1, 2], np.int64), np.array([-1, 0], np.int32), vals[:2], 2, 4)
    assert e.value.code == nat.SCC_ERR_INVALID


def test_transpose_at_the_gene_limit_and_past_it(eng):
    """The transpose's largest gene count (262,144 = 1024 tiles of 256 genes:
    include/scc.h) is exact; one gene more is refused with SCC_ERR_UNSUPPORTED."""
    from scconsensus_amd import _native as nat
    rng = np.random.default_rng(13)
    G, N = 262_144, 3000
    m = sp.random(G, N, density=2e-5, format="csr", random_state=rng, dtype=np.float64)
    m.data = rng.standard_normal(m.nnz)
    m = m.tolil()
    m[G - 1, N - 1] = 7.0  # the last gene and cell are present
    m[0, 0] = 3.0
    m = sp.csr_matrix(m)
    m.sort_indices()
    _check_transpose(eng, m, G, N)
    with pytest.raises(nat.SccError) as e:
        eng.dataset_csr(np.zeros(G + 2, np.int64), np.zeros(0, np.int32), np.zeros(0), G + 1, N)
    assert e.value.code == nat.SCC_ERR_UNSUPPORTED
