"""GPU: silhouette widths on the HBM-resident distance vector (SURVEY §8f-2,
Fast:433 cluster::silhouette(grp, dmatrix = as.matrix(d))) against an
independent implementation: sklearn.metrics.silhouette_samples on the square
matrix (parity with R's cluster package itself is unpinned: R is absent)."""
import numpy as np
import pytest
from scipy.spatial.distance import squareform
from sklearn.metrics import silhouette_samples

from scconsensus_amd import _native as nat
from scconsensus_amd import api, synth

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def setup():
    eng = nat.Engine(0)
    d = synth.generate("A")
    names, code = api.select_clusters(d.labels, 10)
    ds = eng.dataset_csc(d.indptr, d.indices, d.data, d.G, d.N)
    union = eng.de_run(ds, code, len(names), nat.SCC_DE_FAST, fetch="union").union
    return eng, ds, d, code, union


def _ref(dist, groups):
    w = silhouette_samples(squareform(dist), groups, metric="precomputed")
    ids = np.unique(groups)
    return w, np.array([w[groups == k].mean() for k in ids])


@pytest.mark.parametrize("kind", ["codes", "random5", "random100", "singletons"])
def test_silhouette_matches_sklearn(setup, kind):
    eng, ds, d, code, union = setup
    rng = np.random.default_rng(0)
    groups = {"codes": code,
              "random5": rng.integers(0, 5, d.N),
              "random100": rng.integers(-3, 97, d.N),   # > 64 clusters: two cluster passes
              "singletons": np.r_[np.arange(3) + 50, rng.integers(0, 4, d.N - 3)]}[kind].astype(np.int32)
    dist = eng.distance(ds, union)           # host copy; the engine keeps its device copy
    w, ca = eng.silhouette(d.N, groups)
    rw, rca = _ref(dist, groups)
    np.testing.assert_allclose(w, rw, rtol=1e-9, atol=1e-12)
    np.testing.assert_allclose(ca, rca, rtol=1e-9, atol=1e-12)
    if kind == "singletons":
        assert (w[:3] == 0).all()


def test_silhouette_f32_distance(setup):
    eng, ds, d, code, union = setup
    dist32 = eng.distance(ds, union, f32=True)
    w, ca = eng.silhouette(d.N, code)
    rw, _ = _ref(dist32.astype(np.float64), code)
    np.testing.assert_allclose(w, rw, rtol=1e-9, atol=1e-9)


def test_silhouette_rejects_one_cluster(setup):
    eng, ds, d, code, union = setup
    eng.distance(ds, union, device_out_ptr=0)
    with pytest.raises(nat.SccError):
        eng.silhouette(d.N, np.zeros(d.N, np.int32))
