"""Round-5 scheduling and ingest paths against their references, bit for bit:
the wave kernels' slot-class launches and the re-splits on side streams
(SCC_RW_STREAMS=2: the re-splits' too, which the default takes only past 64 M
stored values) against one stream, and the validated dataset's lean counting pass
(`k_ing_count_ro`, tile starts from the dataset cache) against the full
counting pass (SCC_COUNT_RO=0 / SCC_INGEST_FULL=1), whole-range and in forced
small gene windows (reference: R/reclusterDEConsensusFast.R:78-91, the rank
sums every tested (pair, gene) cell needs)."""
import numpy as np
import pytest
import torch  # before the engine loads (torch's HIP runtime first)

from scconsensus_amd import _native as nat
from scconsensus_amd import api, synth

pytestmark = pytest.mark.gpu

FAST_FIELDS = ("pair_tested", "gene", "p", "q", "avg_logfc", "pct1", "pct2", "u2", "ties", "de", "top")


@pytest.fixture(scope="module")
def eng():
    e = nat.Engine(0)
    yield e
    e.close()


def _same(a, b):
    np.testing.assert_array_equal(a.union, b.union)
    np.testing.assert_array_equal(a.nodg, b.nodg)
    for f in FAST_FIELDS:
        np.testing.assert_array_equal(getattr(a.rows, f), getattr(b.rows, f), err_msg=f)


def test_side_streams_bitwise(eng, monkeypatch):
    """K = 40 (780 pairs): genes spread over the 2-, 4- and 8-slot classes and
    the matrix-core class, so several class launches share the side streams."""
    d = synth.generate("A", G=1500, N=6000, K=40, seed=7)
    names, code = api.select_clusters(d.labels, 10)
    K = len(names)
    assert K >= 30
    ds = eng.dataset_csc(d.indptr, d.indices, d.data, d.G, d.N)
    monkeypatch.setenv("SCC_RW_STREAMS", "0")
    one = eng.de_run(ds, code, K, nat.SCC_DE_FAST, fetch="rows")
    monkeypatch.setenv("SCC_RW_STREAMS", "2")  # (2: the re-splits' side streams too, at any size)
    for _ in range(2):
        _same(eng.de_run(ds, code, K, nat.SCC_DE_FAST, fetch="rows"), one)
    # SLOW: every gene tested by every pair (the wide slot classes and windows)
    sub = synth.from_dense(d.dense()[:300], d.labels)
    dss = eng.dataset_csc(sub.indptr, sub.indices, sub.data, sub.G, sub.N)
    kw = dict(q_val_thrs=0.05, fc_thrs=1.5, mean_scaling_factor=5.0)
    monkeypatch.setenv("SCC_RW_STREAMS", "0")
    slow1 = eng.de_run(dss, code, K, nat.SCC_DE_SLOW, fetch="all", **kw)
    monkeypatch.setenv("SCC_RW_STREAMS", "2")
    slow2 = eng.de_run(dss, code, K, nat.SCC_DE_SLOW, fetch="all", **kw)
    for f in ("union", "p", "q", "logfc", "u2", "de"):
        np.testing.assert_array_equal(getattr(slow2, f), getattr(slow1, f), err_msg=f)


@pytest.mark.parametrize("window", ["", "100", "777"])
def test_lean_count_matches_full_count(eng, window, monkeypatch):
    if window:
        monkeypatch.setenv("SCC_HIST_WINDOW", window)
    d = synth.generate("A", G=1000, N=1500, K=6, seed=43)
    names, code = api.select_clusters(d.labels, 10)
    K = len(names)
    ds = eng.dataset_csc(d.indptr, d.indices, d.data, d.G, d.N)
    first = eng.de_run(ds, code, K, nat.SCC_DE_FAST, fetch="rows")  # validating read (k_ing_hist)
    lean = eng.de_run(ds, code, K, nat.SCC_DE_FAST, fetch="rows")   # validated: k_ing_count_ro
    monkeypatch.setenv("SCC_COUNT_RO", "0")
    hist = eng.de_run(ds, code, K, nat.SCC_DE_FAST, fetch="rows")   # validated: k_ing_hist rows-only
    monkeypatch.setenv("SCC_INGEST_FULL", "1")
    full = eng.de_run(ds, code, K, nat.SCC_DE_FAST, fetch="rows")
    for r in (lean, hist, full):
        _same(r, first)
