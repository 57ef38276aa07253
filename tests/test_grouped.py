"""The group-pair decomposition libscc uses past 128 clusters
(tests/group_model.py mirrors scc_runtime.cpp de_run_grouped), with the
oracle standing in for the device: the runs reassembled in (i, j) order equal
one oracle run over all K, FAST (rows, order, union) and SLOW (per-pair
vectors, de flags, union).  tests/test_gpu_grouped.py runs the engine's
implementation at K = 150."""
import numpy as np
import pytest

import oracle as O
from group_model import de_fast_grouped, de_slow_grouped, groups, runs
from scconsensus_amd import api, synth


@pytest.mark.parametrize("K,gmax", [(9, 4), (10, 3), (7, 3), (150, 64)])
def test_runs_cover_every_pair_once(K, gmax):
    taken = [gp for _, take in runs(K, gmax) for gp in take.values()]
    assert sorted(taken) == list(range(K * (K - 1) // 2))
    assert all(len(cl) <= 2 * gmax for cl, _ in runs(K, gmax))
    assert sum(len(g) for g in groups(K, gmax)) == K


@pytest.mark.parametrize("K,gmax", [(9, 4), (10, 3), (7, 3)])
def test_fast_grouped_equals_single_run(K, gmax):
    d = synth.generate("A", G=150, N=900, K=K, seed=13)
    names, code = api.select_clusters(d.labels, 10)
    X = d.dense()
    kw = dict(min_per_cent=5.0, log_fc_thrs=0.1)
    tested, rows, union = de_fast_grouped(X, code, len(names), gmax, **kw)
    o = O.de_fast(X, code, len(names), **kw)
    np.testing.assert_array_equal(tested, o.pair_tested)
    np.testing.assert_array_equal(rows["gene"], o.row_gene)
    np.testing.assert_array_equal(rows["p"], o.row_p)
    np.testing.assert_array_equal(rows["q"], o.row_q)
    np.testing.assert_array_equal(rows["top"], o.row_top)
    np.testing.assert_array_equal(union, o.union)


@pytest.mark.parametrize("K,gmax", [(9, 4), (8, 3)])
def test_slow_grouped_equals_single_run(K, gmax):
    d = synth.generate("A", G=80, N=800, K=K, seed=15)
    names, code = api.select_clusters(d.labels, 10)
    X = d.dense()
    v, union = de_slow_grouped(X, code, len(names), gmax, 0.05, 1.5, 5.0)
    o = O.de_slow(X, code, len(names), 0.05, 1.5, 5.0)
    np.testing.assert_array_equal(v["p"], o.p)
    np.testing.assert_array_equal(v["q"], o.q)
    np.testing.assert_array_equal(v["W"], o.W)
    np.testing.assert_array_equal(v["de"], o.de)
    np.testing.assert_array_equal(union, o.union)
