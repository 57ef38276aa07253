"""CPU: deterministic synthetic inputs of the BASELINE shapes."""
import numpy as np

from scconsensus_amd import synth


def test_config_a_deterministic():
    a = synth.generate("A")
    b = synth.generate("A")
    assert a.G == 2000 and a.N == 3000
    np.testing.assert_array_equal(a.indptr, b.indptr)
    np.testing.assert_array_equal(a.data, b.data)
    assert 0.05 < a.nnz / (a.G * a.N) < 0.2
    labs, cnt = np.unique(a.labels, return_counts=True)
    assert len(labs) == 8 and cnt.min() >= 30


def test_csc_rows_sorted_and_dense_roundtrip():
    d = synth.generate("A", G=300, N=400)
    for c in range(0, d.N, 37):
        r = d.indices[d.indptr[c]:d.indptr[c + 1]]
        assert np.all(np.diff(r) > 0)
    X = d.dense()
    e = synth.from_dense(X, d.labels)
    np.testing.assert_array_equal(e.indptr, d.indptr)
    np.testing.assert_array_equal(e.data, d.data)


def test_pbmc_sizes():
    s = synth.cluster_sizes("pbmc", 26000, 12, np.random.default_rng(0))
    assert s.sum() == 26000 and len(s) == 12 and s.min() >= 59


def test_edge_fixture_has_edges():
    d = synth.edge_fixture()
    labs, cnt = np.unique(d.labels, return_counts=True)
    cnt = dict(zip(labs, cnt))
    assert cnt["grey"] > 10 and cnt["tiny"] <= 10 and cnt["yellow"] == 15
