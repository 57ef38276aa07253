"""Regression tests for context-lifetime and argument-forwarding bugs.

* An engine-kept distance (device_out_ptr=0, the eigensolver's hand-off flag
  left pending in the context's mapped pinned word) followed by a DE run whose
  host tables outgrow the pinned table buffer: the regrow must not free the
  flag word (round-3 ADVICE, scc_runtime.cpp), and the flag must still be
  reported and the context destroyed cleanly.
* ``Engine.de_distance(test="t")`` runs the t test, as ``de_run`` does.
"""
import numpy as np
import pytest

from scconsensus_amd import _native as nat
from scconsensus_amd import api, synth

pytestmark = pytest.mark.gpu


def test_kept_distance_then_larger_de_run():
    small = synth.generate("A", G=400, N=600, K=4, seed=11)
    big = synth.generate("A", G=1500, N=2500, K=12, seed=12)
    eng = nat.Engine(0)
    try:
        ds_s = eng.dataset_csc(small.indptr, small.indices, small.data, small.G, small.N)
        names, code = api.select_clusters(small.labels, 10)
        de = eng.de_run(ds_s, code, len(names), fetch="union")
        assert len(de.union) > 15
        eng.distance(ds_s, de.union, nat.SCC_DIST_PCA_EUCLID, device_out_ptr=0)  # kept, flag pending
        ds_b = eng.dataset_csc(big.indptr, big.indices, big.data, big.G, big.N)
        names_b, code_b = api.select_clusters(big.labels, 10)
        de_b = eng.de_run(ds_b, code_b, len(names_b), fetch="union")  # reads the pending flag
        assert len(de_b.union) > 0
        d2 = eng.distance(ds_b, de_b.union[:40], nat.SCC_DIST_PCA_EUCLID)
        assert np.isfinite(d2).all()
        eng.synchronize()
    finally:
        eng.close()


def test_de_distance_forwards_test():
    d = synth.generate("A", G=600, N=900, K=5, seed=13)
    eng = nat.Engine(0)
    try:
        ds = eng.dataset_csc(d.indptr, d.indices, d.data, d.G, d.N)
        names, code = api.select_clusters(d.labels, 10)
        K = len(names)
        ref_t = eng.de_run(ds, code, K, fetch="union", test="t")
        ref_w = eng.de_run(ds, code, K, fetch="union", test="wilcox")
        de_t, _ = eng.de_distance(ds, code, K, device_out_ptr=0, test="t")
        np.testing.assert_array_equal(de_t.union, ref_t.union)
        assert not np.array_equal(ref_t.union, ref_w.union)  # the two tests pick different unions here
        with pytest.raises(TypeError):
            eng.de_distance(ds, code, K, device_out_ptr=0, tset="t")
    finally:
        eng.close()
