"""CPU: the large-configuration checkers (parity_helpers.py) accept the
oracle's own full result and reject tampered rows, so a green GPU run at
C/D/E means what it says."""
from types import SimpleNamespace

import numpy as np
import pytest

import oracle as O
from parity_helpers import (check_p_from_counts, check_rows_against_oracle_subset, check_selection, packed_index,
                            rows_of_gene_major, sample_cell_pairs)
from scconsensus_amd import api, synth


@pytest.fixture(scope="module")
def small():
    d = synth.generate("A", G=300, N=1200, K=6, seed=12)
    names, code = api.select_clusters(d.labels, 10)
    X = d.dense()
    o = O.de_fast(X, code, len(names))
    rows = SimpleNamespace(pair_tested=o.pair_tested, row_pair=o.row_pair, gene=o.row_gene, p=o.row_p, q=o.row_q,
                           avg_logfc=o.row_lfc, pct1=o.row_pct1, pct2=o.row_pct2,
                           u2=np.round(2 * o.row_W).astype(np.int64), ties=np.round(o.row_ties).astype(np.int64),
                           de=o.row_de, top=o.row_top)
    return d, X, code, len(names), o, rows


def test_selection_accepts_oracle(small):
    d, X, code, K, o, rows = small
    check_selection(rows, o.union, K)


def test_selection_rejects_swapped_rows(small):
    d, X, code, K, o, rows = small
    bad = SimpleNamespace(**vars(rows))
    bad.gene = rows.gene.copy()
    bad.gene[[0, 1]] = bad.gene[[1, 0]]
    bad.p = rows.p.copy()
    bad.p[[0, 1]] = bad.p[[1, 0]]
    with pytest.raises(AssertionError):
        check_selection(bad, o.union, K)


def test_subset_oracle_accepts_and_rejects(small):
    d, X, code, K, o, rows = small
    genes = np.arange(5, 300, 7)
    n = check_rows_against_oracle_subset(rows, X[genes], genes, code, K)
    assert n > 0
    bad = SimpleNamespace(**vars(rows))
    bad.u2 = rows.u2.copy()
    k = int(np.nonzero(np.isin(rows.gene, genes))[0][0])
    bad.u2[k] += 1
    with pytest.raises(AssertionError):
        check_rows_against_oracle_subset(bad, X[genes], genes, code, K)


def test_p_from_counts_accepts_oracle_and_rejects(small):
    d, X, code, K, o, rows = small
    assert check_p_from_counts(rows, code, K) == len(rows.p)
    bad = SimpleNamespace(**vars(rows))
    bad.p = rows.p.copy()
    k = int(np.flatnonzero(rows.p > 1e-10)[0])
    bad.p[k] *= 1.0 + 1e-6
    with pytest.raises(AssertionError):
        check_p_from_counts(bad, code, K)


def test_p_from_counts_exact_branch():
    """Small clusters without ties (wilcox.test's exact branch) and tied
    data (the normal branch), each row's p against the oracle's wilcox.test."""
    rng = np.random.default_rng(1)
    K, sizes = 4, [30, 45, 60, 200]
    code = np.repeat(np.arange(K), sizes).astype(np.int32)
    rng.shuffle(code)
    u2, ties, p, tested = [], [], [], []
    for i in range(K - 1):
        for j in range(i + 1, K):
            for g in range(20):
                x = np.where(rng.random(len(code)) < 0.6, np.round(rng.gamma(1, 2, len(code)), 1), 0.0)
                if g % 4 == 0:
                    x = rng.random(len(code))  # no ties: exact below 50 cells
                pv, W, T, _ = O.wilcox_test(x[code == i], x[code == j])
                u2.append(int(round(2 * W)))
                ties.append(T)
                p.append(pv)
            tested.append(20)
    rows = SimpleNamespace(pair_tested=np.array(tested), u2=np.array(u2), ties=np.array(ties), p=np.array(p))
    assert check_p_from_counts(rows, code, K) == len(p)


def test_packed_index_and_rows():
    N = 7
    i, j = sample_cell_pairs(N, 50, seed=1)
    assert np.all(i > j)
    from scipy.spatial.distance import squareform
    v = np.arange(N * (N - 1) // 2, dtype=float)
    M = squareform(v)
    np.testing.assert_array_equal(v[packed_index(i, j, N)], M[i, j])
    d = synth.generate("A", G=30, N=200, K=3, seed=2)
    csr = d.scipy_csc().tocsr()
    genes = np.array([0, 5, 29])
    np.testing.assert_array_equal(rows_of_gene_major(csr.indptr, csr.indices, csr.data, genes, d.N),
                                  d.dense()[genes])
