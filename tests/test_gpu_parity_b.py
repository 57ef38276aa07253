"""GPU parity at config B (26k cells x 10k genes, K = 12: the metric's
configuration) for the paths test_gpu_configs.py leaves out there:

* SLOW (reclusterDEConsensus, slow:32-227): the oracle on 80 genes over all
  cells and all 66 pairs (exact U, p / logFC within the bar), the global
  threshold (slow:36) restated from the stored values, and the FULL-size
  selection restated from the engine's per-pair vectors: BH with n = G, the DE
  flags with the expression gate of every gene (R's long-double means), the
  first-30 union.
* The `t` test (DiffTTest, Fast:185-196): the oracle on a gene subset over all
  cells and pairs, and the full-size FAST selection from the engine's rows.
* north_star's label bar: hclust(ward.D2) + cutreeDynamic (deepSplit 1..4,
  pamStage = FALSE) on the GPU distance and on the exact-SVD distance give the
  same merges and the same labels (Fast:398-428; B's lambda16 / lambda15 = 0.996
  makes the PCA subspace the delicate part).
"""
import numpy as np
import pytest
import torch  # noqa: F401  (torch's HIP runtime first)

import oracle as O
from parity_helpers import (check_rows_against_oracle_subset, check_selection, check_slow_against_oracle_subset,
                            check_slow_selection, slow_gate, slow_log_threshold)
from scconsensus_amd import _native as nat
from scconsensus_amd import api, synth

pytestmark = pytest.mark.gpu


def _say(*a):  # progress in the GPU log (long tests)
    print("[progress]", *a, flush=True)


@pytest.fixture(scope="module")
def cfg_b():
    d = synth.generate("B")
    names, code = api.select_clusters(d.labels, 10)
    assert len(names) == 12
    eng = nat.Engine(0)
    ds = eng.dataset_csc(d.indptr, d.indices, d.data, d.G, d.N)
    csr = d.scipy_csc().tocsr()
    yield d, code, eng, ds, csr
    ds.close()
    eng.close()


def test_slow_config_b(cfg_b):
    d, code, eng, ds, csr = cfg_b
    K, qthr, fc, msf = 12, 0.05, 1.5, 5.0
    g = eng.de_run(ds, code, K, nat.SCC_DE_SLOW, q_val_thrs=qthr, fc_thrs=fc, mean_scaling_factor=msf, fetch="all")
    assert g.p.shape == (66, d.G)
    _say("SLOW B engine done")
    assert g.log_thr == pytest.approx(slow_log_threshold(d.data, d.G, d.N, msf), rel=1e-13)
    rng = np.random.default_rng(8)
    genes = np.sort(rng.choice(d.G, 80, replace=False))
    Xs = csr[genes].toarray()
    assert check_slow_against_oracle_subset(g, Xs, genes, code, K, qthr, fc, msf) == 66 * 80
    # the gate of EVERY gene (R means over the dense rows, a block of genes at a time)
    gate = np.zeros((66, d.G), bool)
    for a in range(0, d.G, 500):
        gate[:, a:a + 500] = slow_gate(csr[a:a + 500].toarray(), code, K, g.log_thr)
    _say("SLOW B gates done")
    check_slow_selection(g, qthr, fc, gate=gate)
    assert len(g.union) > 30


def test_t_test_config_b(cfg_b):
    d, code, eng, ds, csr = cfg_b
    K = 12
    g = eng.de_run(ds, code, K, nat.SCC_DE_FAST, fetch="rows", test="t")
    r = g.rows
    assert (r.u2 == 0).all() and len(g.union) > 30
    check_selection(r, g.union, K)
    rng = np.random.default_rng(9)
    genes = np.unique(np.concatenate([rng.choice(np.unique(r.gene), 40, replace=False),
                                      rng.choice(d.G, 40, replace=False)]))
    assert check_rows_against_oracle_subset(r, csr[genes].toarray(), genes, code, K, test="t") >= 500


def test_deepsplit_labels_config_b(cfg_b):
    d, code, eng, ds, csr = cfg_b
    union = eng.de_run(ds, code, 12, nat.SCC_DE_FAST, fetch="union").union
    gpu = eng.distance(ds, union, nat.SCC_DIST_PCA_EUCLID)
    ref = O.dist_euclidean(O.pca_scores(csr[union].toarray(), np.arange(len(union))))
    err = float(np.max(np.abs(gpu - ref)))
    assert err < 1e-5, err
    _say("B distances done, max |gpu - exact| =", err)
    mg, hg, og = nat.hclust_ward_d2(gpu, d.N)
    _say("B Ward (GPU dist) done")
    mr, hr, orr = nat.hclust_ward_d2(ref, d.N)
    _say("B Ward (exact dist) done")
    rows_differ = np.flatnonzero((mg != mr).any(axis=1))
    _say("merge rows that differ:", len(rows_differ), "first at height",
         float(hg[rows_differ[0]]) if len(rows_differ) else None,
         "max height there", float(hg[rows_differ].max()) if len(rows_differ) else None)
    # identical union-gene expression (e.g. no union gene expressed) makes
    # cells coincide in PCA space: their distances are 0 up to rounding, so
    # their merge order among themselves is a tie either tree may break
    Xu = csr[union]
    key = [hash(Xu[:, c].toarray().tobytes()) for c in range(0, d.N)]
    _, cnt = np.unique(key, return_counts=True)
    _say("cells sharing their union-gene profile with another cell:", int(cnt[cnt > 1].sum()))
    np.testing.assert_allclose(np.sort(hg), np.sort(hr), rtol=0, atol=1e-6)
    assert np.all(hg[rows_differ] < 1e-6), "merges differ above the tie level"
    for dsv in (1, 2, 3, 4):
        lg, cg = nat.cutree_hybrid(mg, hg, gpu, dsv, 10)
        lr, cr = nat.cutree_hybrid(mr, hr, ref, dsv, 10)
        assert np.array_equal(lg, lr), dsv
        assert cg == pytest.approx(cr, abs=1e-5)
        assert len(np.unique(lg)) >= 2
