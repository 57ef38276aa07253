"""The wave buckets' pair counts on the int8 matrix cores (k_rank_mfma16, K <= 64)
against the per-pair slot kernel (k_rank_waves, SCC_RANK_MFMA=0), every gene on
the matrix cores (SCC_RANK_MFMA=2; by default only genes past 512 tested pairs): the same
integers (U for every pair and gene, and the p-values, which carry the tie
terms E, X, F), FAST over every (pair, gene) cell and SLOW; then the oracle on
a tie-heavy dataset at K = 64 (the largest K on the matrix cores, 2016 pairs)."""
import numpy as np
import pytest

import oracle as O
from scconsensus_amd import api, synth

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def eng():
    from scconsensus_amd import _native
    return _native.Engine(0)


def _dataset(K, G, N, seed, decimals):
    """NB-like values; rounding to `decimals` puts many equal values in a
    bucket (tie groups across and within clusters)."""
    d = synth.generate("A", G=G, N=N, K=K, seed=seed)
    X = d.dense()
    if decimals is not None:
        X = np.round(X, decimals)
    names = np.asarray(d.labels, dtype=object)
    return synth.from_dense(X, names), X


@pytest.mark.parametrize("K,decimals", [(12, None), (12, 1), (30, 2), (40, 1), (64, 1)])
def test_mfma_matches_slot_kernel(eng, K, decimals, monkeypatch):
    from scconsensus_amd import _native as nat
    d, X = _dataset(K, 160, 12000, 3 + K, decimals)
    names, code = api.select_clusters(d.labels, 10)
    Kc = len(names)
    ds = eng.dataset_csc(d.indptr, d.indices, d.data, d.G, d.N)
    res = {}
    # every gene on the matrix-core kernel / the genes past 512 pairs /
    # none; "16": the matrix cores (K <= 32) also for the genes the slot kernels take
    for flag in ("2", "1", "0", "16"):
        monkeypatch.setenv("SCC_RANK_MFMA", "1" if flag == "16" else flag)
        monkeypatch.setenv("SCC_RANK_MFMA16", "1" if flag == "16" else "0")  # (default: on at K <= 16)
        f = eng.de_run(ds, code, Kc, nat.SCC_DE_FAST, fetch="all", test_all=True, min_per_cent=1.0,
                       log_fc_thrs=0.0)
        s = eng.de_run(ds, code, Kc, nat.SCC_DE_SLOW, fetch="all")
        res[flag] = (f, s)
    monkeypatch.delenv("SCC_RANK_MFMA16")
    f16, s16 = res["16"]
    f0, s0 = res["0"]
    np.testing.assert_array_equal(f16.u2, f0.u2)
    np.testing.assert_array_equal(f16.p, f0.p)
    np.testing.assert_array_equal(s16.u2, s0.u2)
    np.testing.assert_array_equal(s16.p, s0.p)
    f1, s1 = res["2"]
    f0, s0 = res["0"]
    np.testing.assert_array_equal(f1.u2, f0.u2)
    np.testing.assert_array_equal(f1.p, f0.p)
    np.testing.assert_array_equal(f1.rows.ties, f0.rows.ties)
    np.testing.assert_array_equal(s1.u2, s0.u2)
    np.testing.assert_array_equal(s1.p, s0.p)
    np.testing.assert_array_equal(s1.union, s0.union)
    fh, sh = res["1"]
    np.testing.assert_array_equal(fh.u2, f0.u2)
    np.testing.assert_array_equal(sh.u2, s0.u2)
    np.testing.assert_array_equal(sh.p, s0.p)
    assert (f1.u2 > 0).sum() > 0.5 * f1.u2.size


def test_mfma_k64_ties_oracle(eng, monkeypatch):
    from scconsensus_amd import _native as nat
    monkeypatch.setenv("SCC_RANK_MFMA", "2")
    d, X = _dataset(64, 40, 6000, 17, 1)
    names, code = api.select_clusters(d.labels, 10)
    K = len(names)
    assert K == 64
    ds = eng.dataset_csc(d.indptr, d.indices, d.data, d.G, d.N)
    g = eng.de_run(ds, code, K, nat.SCC_DE_FAST, fetch="rows", min_per_cent=1.0, log_fc_thrs=0.0)
    o = O.de_fast(X, code, K, min_per_cent=1.0, log_fc_thrs=0.0)
    r = g.rows
    np.testing.assert_array_equal(r.gene, o.row_gene)
    np.testing.assert_array_equal(r.u2, np.round(2 * o.row_W).astype(np.int64))
    np.testing.assert_array_equal(r.ties, np.round(o.row_ties).astype(np.int64))
    np.testing.assert_allclose(r.p, o.row_p, rtol=1e-6, atol=0)
    assert (r.ties > 0).mean() > 0.5  # the tie products ran
