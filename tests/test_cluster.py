"""Host clustering: libscc's scc_hclust_ward_d2 and
scc_cutree_hybrid, the restatements of fastcluster::hclust(d, "ward.D2")
(Fast:406-411) and dynamicTreeCut::cutreeDynamic(hybrid, pamStage = FALSE)
(Fast:421-427).  Host code: no GPU needed.

hclust is pinned to scipy's Ward linkage (the same method; fastcluster's own
documentation equates R "ward.D2" with Python "ward").  cutreeHybrid has no
implementation in this image and R is absent, so it is "parity unpinned": the
C++ is checked against the oracle's independent line-by-line Python
restatement (oracle.cutree_hybrid) over a parameter grid and against
hand-worked dendrograms whose outcome follows from the published rules."""
import numpy as np
import pytest
from scipy.spatial.distance import pdist, squareform

import oracle as O
from scconsensus_amd import _native as nat
from scconsensus_amd.api import labels2colors


def _blobs(rng, sizes, sep, dim=5):
    return np.concatenate([rng.standard_normal((s, dim)) + sep * i for i, s in enumerate(sizes)])


@pytest.mark.parametrize("n", [2, 3, 4, 7, 64, 500])
def test_ward_d2_matches_scipy(n):
    rng = np.random.default_rng(n)
    X = rng.standard_normal((n, 6)) * rng.uniform(0.2, 3.0, (n, 1))
    d = pdist(X)
    merge, height, order = nat.hclust_ward_d2(d, n)
    mr, hr = O.ward_d2_r(d, n)
    assert np.array_equal(merge, mr)
    np.testing.assert_allclose(height, hr, rtol=1e-12, atol=1e-12)
    assert sorted(order.tolist()) == list(range(1, n + 1))
    assert np.all(np.diff(height) >= 0)


def test_ward_d2_order_is_left_to_right():
    # two far groups: the order lists one group's leaves, then the other's
    rng = np.random.default_rng(1)
    X = _blobs(rng, [10, 10], 100.0)
    merge, height, order = nat.hclust_ward_d2(pdist(X), 20)
    first = set(order[:10].tolist())
    assert first in ({*range(1, 11)}, {*range(11, 21)})
    # the last merge joins the two groups; its children come out in merge order
    last = merge[-1]
    assert (last < 0).sum() == 0


def test_ward_d2_rejects_nonfinite():
    d = np.array([1.0, np.nan, 2.0])
    with pytest.raises(nat.SccError):
        nat.hclust_ward_d2(d, 3)


@pytest.mark.parametrize("seed", range(6))
def test_cutree_matches_restatement(seed):
    rng = np.random.default_rng(100 + seed)
    k = int(rng.integers(2, 9))
    sizes = rng.integers(5, 80, k)
    X = _blobs(rng, sizes, float(rng.uniform(1.5, 6.0)), dim=int(rng.integers(2, 12)))
    X *= rng.uniform(0.5, 2.0, (len(X), 1))
    n = len(X)
    d = pdist(X)
    D = squareform(d)
    merge, height, _ = nat.hclust_ward_d2(d, n)
    for ds in range(5):
        for mcs in (3, 5, 10, 20, 40):
            lab, cut = nat.cutree_hybrid(merge, height, d, ds, mcs)
            ref = O.cutree_hybrid(merge, height, D, ds, mcs)
            assert np.array_equal(lab, ref), (ds, mcs)
            assert cut <= height.max() + 1e-12
            # labels are 0 or 1..m, ranked by decreasing size
            cnt = np.bincount(lab)[1:]
            assert np.all(cnt > 0) and np.all(np.diff(cnt) <= 0)


def test_cutree_two_separated_groups():
    # two compact groups far apart: each is a top basic branch passing size,
    # scatter and gap; the larger is label 1
    rng = np.random.default_rng(7)
    X = _blobs(rng, [30, 20], 50.0)
    d = pdist(X)
    merge, height, _ = nat.hclust_ward_d2(d, 50)
    for ds in (0, 1):
        lab, _ = nat.cutree_hybrid(merge, height, d, ds, 10)
        assert np.array_equal(lab, np.r_[np.ones(30, int), np.full(20, 2)])


def test_cutree_too_few_merges_below_cut_is_unlabeled():
    # nMergeBelowCut < minClusterSize -> every object unassigned (label 0)
    rng = np.random.default_rng(3)
    X = rng.standard_normal((8, 3))
    d = pdist(X)
    merge, height, _ = nat.hclust_ward_d2(d, 8)
    lab, _ = nat.cutree_hybrid(merge, height, d, 1, 20)
    assert not lab.any()


def test_cutree_default_cut_height():
    rng = np.random.default_rng(5)
    X = _blobs(rng, [40, 40, 40], 8.0)
    d = pdist(X)
    merge, height, _ = nat.hclust_ward_d2(d, 120)
    _, cut = nat.cutree_hybrid(merge, height, d, 1, 10)
    ref_h = height[max(round(119 * 0.05), 1) - 1]
    assert cut == pytest.approx(0.99 * (height.max() - ref_h) + ref_h, rel=1e-15)


def test_cutree_deepsplit_range():
    d = pdist(np.random.default_rng(0).standard_normal((30, 2)))
    merge, height, _ = nat.hclust_ward_d2(d, 30)
    with pytest.raises(nat.SccError):
        nat.cutree_hybrid(merge, height, d, 5, 5)
    with pytest.raises(nat.SccError):
        nat.cutree_hybrid(merge, height, d, -1, 5)


def test_deeper_split_never_fewer_clusters_on_blobs():
    rng = np.random.default_rng(11)
    X = _blobs(rng, [60, 50, 40, 30, 20], 3.0)
    d = pdist(X)
    merge, height, _ = nat.hclust_ward_d2(d, len(X))
    ncl = [nat.cutree_hybrid(merge, height, d, ds, 10)[0].max() for ds in range(5)]
    assert ncl == sorted(ncl)


def test_labels2colors():
    assert labels2colors([0, 1, 2, 3, 7, 17, 34]) == ["grey", "turquoise", "blue", "brown", "black", "grey60",
                                                        "darkmagenta"]


def test_select_clusters_table_filters_and_missing_labels():
    """Cluster selection as Fast:39-47: table() counts, `> minClusterSize`, no
    "grey", names in code-point (C locale) order; NA / None / NaN labels are no
    cluster (R's table() drops NA) and their cells get code -1."""
    import pandas as pd
    from scconsensus_amd.api import select_clusters
    labels = ["b"] * 5 + ["a"] * 4 + ["grey"] * 9 + ["c"] * 2 + [None] * 6 + [float("nan")] * 6 + [pd.NA] * 6
    names, code = select_clusters(labels, 3)
    assert names == ["a", "b"]
    want = [1] * 5 + [0] * 4 + [-1] * 9 + [-1] * 2 + [-1] * 18
    assert code.tolist() == want
    # the string "nan" is a real label (R would count it)
    names2, code2 = select_clusters(["nan"] * 5 + ["x"] * 5, 3)
    assert names2 == ["nan", "x"] and code2.tolist() == [0] * 5 + [1] * 5
