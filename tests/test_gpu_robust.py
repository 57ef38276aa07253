"""The PCA eigensolve (Fast:398) under concurrency and faults, and the ingest's
rows-only counting pass on data with stored zeros.

* Two engine contexts on device 0 driven from two host threads at once: every
  distance is bit-identical to the same call made alone, and the persistent
  engine answers (path 3): each thread has its own verdict word, each context
  its own graphs.
* Workspace freed and reallocated between two distances (a larger union in
  between grows the eigensolver's scratch): the third call is bit-identical to
  the first (graphs are keyed on the context and its workspace generation).
* The persistent engine's hand-off time-out, forced on the host
  (SCC_EIG_FSI_FORCE_HERR) and on the device (SCC_EIG_FX_SPIN=0: every poll
  that does not succeed at once aborts): the launch path answers with the
  engine's bits; after a time-out the engine cools down for
  SCC_EIG_FX_COOL calls.
* The direct solver's time-out (SCC_EIG_FORCE_TIMEOUT): the one-workgroup
  rerun answers (path 4), within 1e-9 of the cooperative solve.
* A dgCMatrix with explicit stored zeros: two full FAST runs give identical
  rows and nodg (the second, validated run must keep reading values), equal to
  the same matrix with the zeros dropped.
"""
import threading

import numpy as np
import pytest

from scconsensus_amd import _native as nat
from scconsensus_amd import api, synth

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def job():
    d = synth.generate("A", seed=1)
    names, code = api.select_clusters(d.labels, 10)
    eng = nat.Engine(0)
    try:
        ds = eng.dataset_csc(d.indptr, d.indices, d.data, d.G, d.N)
        union = eng.de_run(ds, code, len(names), fetch="union").union
        ds.close()
    finally:
        eng.close()
    assert 128 <= len(union) <= 1024, len(union)  # the filtered eigensolver's range
    return d, union


def _dist_with_path(eng, ds, genes):
    out = eng.distance(ds, genes, nat.SCC_DIST_PCA_EUCLID)
    return out, int(eng.lib.scc_diag_eig_last_path())


def _engine(d):
    eng = nat.Engine(0)
    return eng, eng.dataset_csc(d.indptr, d.indices, d.data, d.G, d.N)


def test_two_contexts_two_threads(job):
    d, union = job
    engs = [_engine(d) for _ in range(2)]
    try:
        ref, path = _dist_with_path(*engs[0], union)
        assert path == 3, "the persistent engine did not answer"
        res = [[] for _ in engs]
        errs = []

        def run(i):
            try:
                for _ in range(4):
                    res[i].append(_dist_with_path(*engs[i], union))
            except Exception as ex:  # reported below
                errs.append(ex)

        th = [threading.Thread(target=run, args=(i,)) for i in range(2)]
        for t in th:
            t.start()
        for t in th:
            t.join(timeout=120)
        assert not errs, errs
        for r in res:
            assert len(r) == 4
            for out, p in r:
                assert p == 3
                assert np.array_equal(out, ref)
    finally:
        for eng, ds in engs:
            ds.close()
            eng.close()


def test_scratch_reallocated_between_distances(job):
    d, union = job
    eng, ds = _engine(d)
    try:
        first, p1 = _dist_with_path(eng, ds, union)
        big = np.arange(min(d.G, 900), dtype=np.int32)  # grows the eigensolver's scratch and the Gram
        eng.distance(ds, big, nat.SCC_DIST_PCA_EUCLID, device_out_ptr=0)
        eng.synchronize()
        again, p2 = _dist_with_path(eng, ds, union)
        assert p1 == 3 and p2 == 3
        assert np.array_equal(first, again)
    finally:
        ds.close()
        eng.close()


def test_engine_timeout_takes_launch_path(job, monkeypatch):
    d, union = job
    eng, ds = _engine(d)
    try:
        monkeypatch.setenv("SCC_EIG_FSI", "1")  # the filtered iteration without the engine: a launch per step
        monkeypatch.setenv("SCC_EIG_FSI_ENGINE", "0")
        launch, p = _dist_with_path(eng, ds, union)
        assert p == 2
        monkeypatch.delenv("SCC_EIG_FSI_ENGINE")
        monkeypatch.delenv("SCC_EIG_FSI")
        monkeypatch.setenv("SCC_EIG_FX_COOL", "2")
        monkeypatch.setenv("SCC_EIG_FSI_FORCE_HERR", "1")
        forced, p = _dist_with_path(eng, ds, union)
        assert p == 2 and np.array_equal(forced, launch)
        monkeypatch.delenv("SCC_EIG_FSI_FORCE_HERR")
        paths = [_dist_with_path(eng, ds, union)[1] for _ in range(3)]
        assert paths == [2, 2, 3], paths  # two calls cool down, then the engine again
        # the device-side abort: a poll that does not succeed at once times out
        monkeypatch.setenv("SCC_EIG_FX_COOL", "0")
        monkeypatch.setenv("SCC_EIG_FX_SPIN", "0")
        spun, p = _dist_with_path(eng, ds, union)
        assert p in (2, 3) and np.array_equal(spun, launch)
        monkeypatch.delenv("SCC_EIG_FX_SPIN")
        back, p = _dist_with_path(eng, ds, union)
        assert p == 3 and np.array_equal(back, launch)
    finally:
        ds.close()
        eng.close()


def test_direct_solver_timeout_rerun(job, monkeypatch):
    d, union = job
    monkeypatch.setenv("SCC_EIG_FSI", "0")  # the direct solver answers at this size
    eng, ds = _engine(d)
    try:
        coop, p = _dist_with_path(eng, ds, union)
        assert p == 0
        monkeypatch.setenv("SCC_EIG_FORCE_TIMEOUT", "1")
        rerun, p = _dist_with_path(eng, ds, union)
        assert p == 4, "the one-workgroup rerun did not answer"
        np.testing.assert_allclose(rerun, coop, rtol=1e-9, atol=1e-9)
    finally:
        ds.close()
        eng.close()


def _explicit_zeros(d, frac=0.05, seed=3):
    """The same matrix with a fraction of its stored values set to 0.0 (stored
    zeros, as a dgCMatrix may hold), and the equivalent without them."""
    import scipy.sparse as sp
    rng = np.random.default_rng(seed)
    vals = d.data.copy()
    vals[rng.random(len(vals)) < frac] = 0.0
    with_z = (d.indptr.copy(), d.indices.copy(), vals)
    m = sp.csc_matrix((vals.copy(), d.indices.copy(), d.indptr.copy()), shape=(d.G, d.N))  # (compacted in place)
    m.eliminate_zeros()
    m.sort_indices()
    no_z = (m.indptr.astype(d.indptr.dtype), m.indices.astype(d.indices.dtype), m.data)
    return with_z, no_z


def test_stored_zeros_rows_only_count():
    d = synth.generate("A", G=600, N=900, K=5, seed=21)
    names, code = api.select_clusters(d.labels, 10)
    K = len(names)
    with_z, no_z = _explicit_zeros(d)
    assert len(with_z[2]) > len(no_z[2])
    eng = nat.Engine(0)
    try:
        ds = eng.dataset_csc(*with_z, d.G, d.N)
        a = eng.de_run(ds, code, K, fetch="rows")  # validating full read (sees the stored zeros)
        b = eng.de_run(ds, code, K, fetch="rows")  # validated: must not take the rows-only count
        ds0 = eng.dataset_csc(*no_z, d.G, d.N)
        c = eng.de_run(ds0, code, K, fetch="rows")
        c2 = eng.de_run(ds0, code, K, fetch="rows")  # the rows-only count on zero-free data
        for r in (b, c, c2):
            assert np.array_equal(r.nodg, a.nodg)
            assert np.array_equal(r.union, a.union)
            for f in ("row_pair", "gene", "u2", "ties", "p", "q", "avg_logfc", "pct1", "pct2", "de", "top"):
                assert np.array_equal(getattr(r.rows, f), getattr(a.rows, f)), f
    finally:
        eng.close()
