"""GPU: north_star's final parity criterion — "deepSplit labels identical when
the host clustering is fed the GPU distance matrix" (Fast:398-428).  The GPU
distance (PCA15 + dist, libscc) and the oracle's distance (numpy exact PCA +
dist) each go through the same host hclust(ward.D2) + cutreeDynamic(hybrid,
pamStage = FALSE); the trees and the labels for deepSplit 1..4 must agree.
Also the Python API mirror end to end (dynamicColors present, R's naming)."""
import numpy as np
import pytest
from scipy.spatial.distance import squareform

import oracle as O
from scconsensus_amd import _native as nat
from scconsensus_amd import api, synth

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def cfg_a():
    eng = nat.Engine(0)
    d = synth.generate("A")
    names, code = api.select_clusters(d.labels, 10)
    ds = eng.dataset_csc(d.indptr, d.indices, d.data, d.G, d.N)
    union = eng.de_run(ds, code, len(names), nat.SCC_DE_FAST, fetch="union").union
    gpu = eng.distance(ds, union, nat.SCC_DIST_PCA_EUCLID)
    ref = O.dist_euclidean(O.pca_scores(d.dense(), union))
    return d, gpu, ref


def test_tree_from_gpu_distance_matches_oracle(cfg_a):
    d, gpu, ref = cfg_a
    assert np.max(np.abs(gpu - ref)) < 1e-5
    mg, hg, og = nat.hclust_ward_d2(gpu, d.N)
    mr, hr, orr = nat.hclust_ward_d2(ref, d.N)
    assert np.array_equal(mg, mr)
    assert np.array_equal(og, orr)
    np.testing.assert_allclose(hg, hr, rtol=0, atol=1e-5)


@pytest.mark.parametrize("min_cluster_size", [10, 30])
def test_deepsplit_labels_identical(cfg_a, min_cluster_size):
    d, gpu, ref = cfg_a
    mg, hg, _ = nat.hclust_ward_d2(gpu, d.N)
    mr, hr, _ = nat.hclust_ward_d2(ref, d.N)
    D = squareform(ref)
    for dsv in (1, 2, 3, 4):
        lg, _ = nat.cutree_hybrid(mg, hg, gpu, dsv, min_cluster_size)
        lr, _ = nat.cutree_hybrid(mr, hr, ref, dsv, min_cluster_size)
        assert np.array_equal(lg, lr), dsv
        # and the oracle's own Python restatement on the oracle's distance
        assert np.array_equal(lr, O.cutree_hybrid(mr, hr, D, dsv, min_cluster_size)), dsv


def test_api_mirror_returns_dynamic_colors(cfg_a):
    d, gpu, _ = cfg_a
    out = api.reclusterDEConsensusFast(d, d.labels, deepSplitValues=(1, 2, 3, 4), minClusterSize=10)
    assert list(out["dynamicColors"]) == [f"deepsplit: {k}" for k in (1, 2, 3, 4)]
    for cols in out["dynamicColors"].values():
        assert len(cols) == d.N
    tree = out["cellTree"]
    assert tree["merge"].shape == (d.N - 1, 2) and tree["method"] == "ward.D2"
    mg, hg, _ = nat.hclust_ward_d2(gpu, d.N)
    assert np.array_equal(tree["merge"], mg)
    lab, _ = nat.cutree_hybrid(mg, hg, gpu, 2, 10)
    assert out["dynamicColors"]["deepsplit: 2"] == api.labels2colors(lab)


def test_api_deepsplit_info_silhouette(cfg_a):
    """The reference's deepSplitInfo (Fast:433): per deepSplit the number of
    clusters and SI = mean of summary(cluster::silhouette(groups,
    as.matrix(d)))$clus.avg.widths, here from the engine's silhouette on the
    HBM-resident distance; checked against sklearn's silhouette_samples on the
    same distance (per-cluster means, singletons 0 as in cluster::silhouette)."""
    from sklearn.metrics import silhouette_samples
    d, gpu, _ = cfg_a
    out = api.reclusterDEConsensusFast(d, d.labels, deepSplitValues=(1, 2), minClusterSize=10, return_details=True)
    info = out["_details"]["deepSplitInfo"]
    dist = out["_details"]["dist"]
    M = squareform(dist)
    tree = out["cellTree"]
    assert [r["DeepSplit"] for r in info] == [1, 2]
    for r in info:
        lab, _ = nat.cutree_hybrid(tree["merge"], tree["height"], dist, int(r["DeepSplit"]), 10)
        lab = np.asarray(lab)
        ks = np.unique(lab)
        assert r["NumbersOfClusters"] == len(ks)
        s = silhouette_samples(M, lab, metric="precomputed")
        ref = np.mean([s[lab == k].mean() for k in ks])
        assert abs(r["SI"] - ref) < 1e-9, (r, ref)
