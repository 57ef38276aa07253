"""The segment rank engine (scc_rank_seg.hip) against the bucket engine it
replaces (SCC_RANK_SEG=0), bit for bit, on every (pair, gene) cell (test_all:
the rank sums of all pairs, R's wilcox.test statistic W = 2U / 2 and its tie
term, Fast:78-91 / slow:99-103):

* whole genes of <= 2048 nonzeros (one segment, read in place) and split genes
  (sampled splitters, interval and equality segments, the cross-segment term);
* heavy ties (a handful of distinct values), one value repeated over a whole
  gene (an equality segment larger than a workgroup's sort), negative values
  and a key range too wide for the composite key (the (key, cluster) sort);
* K = 3 .. 128 clusters (1 .. 8 cluster tiles), FAST and SLOW.
The accumulators are integer atomics, so the engines agree exactly, and the
bucket engine is itself checked against the oracle (test_gpu_de.py)."""
import numpy as np
import pytest

from scconsensus_amd import _native as nat

pytestmark = pytest.mark.gpu


def _csc(X):
    """dgCMatrix slots of a dense genes x cells matrix (CSC over cells)."""
    G, N = X.shape
    nz = X != 0
    counts = nz.sum(axis=0)
    indptr = np.zeros(N + 1, np.int64)
    indptr[1:] = np.cumsum(counts)
    rows = np.nonzero(nz.T)  # (cell, gene) in cell-major order
    indices = rows[1].astype(np.int32)
    data = X.T[nz.T].astype(np.float64)
    return indptr, indices, data


def _matrix(N, G, seed):
    rng = np.random.default_rng(seed)
    X = np.zeros((G, N))
    dens = rng.uniform(0.02, 0.3, G)
    for g in range(G):
        m = rng.random(N) < dens[g]
        X[g, m] = np.log1p(rng.gamma(0.6, 3.0, m.sum()) + 0.01)
    # dense genes (> 2048 stored values: the splitter)
    X[0] = np.log1p(rng.gamma(0.6, 3.0, N) + 0.01)
    X[1] = rng.integers(1, 6, N) * 0.5                       # five distinct values: heavy ties
    X[2] = 1.0                                                # one value over the whole gene
    X[2, rng.choice(N, 7, replace=False)] = 2.0               # ... and a few others
    X[3] = rng.choice([-1.0, 1.0], N) * 10.0 ** rng.uniform(-30, 1, N)  # negatives, a huge key range
    X[4, : N // 2] = np.round(rng.uniform(0.1, 3.0, N // 2), 2)  # rounded: ties inside and across segments
    X[5] = np.where(rng.random(N) < 0.5, 0.0, 3.25)           # one value, half the cells
    return X


def _run(eng, ds, code, K, mode, monkeypatch, seg):
    monkeypatch.setenv("SCC_RANK_SEG", "1" if seg else "0")
    r = eng.de_run(ds, code, K, mode, fetch="all")
    return r


@pytest.mark.parametrize("K,N,mode", [(3, 6000, nat.SCC_DE_FAST), (12, 9000, nat.SCC_DE_FAST),
                                      (12, 5000, nat.SCC_DE_SLOW), (40, 8000, nat.SCC_DE_FAST),
                                      (100, 12000, nat.SCC_DE_FAST), (128, 14000, nat.SCC_DE_SLOW)])
def test_segment_engine_bitwise(K, N, mode, monkeypatch):
    G = 60
    X = _matrix(N, G, seed=K + N)
    rng = np.random.default_rng(K)
    sizes = rng.dirichlet(np.full(K, 1.5)) * (N - 15 * K) + 15
    code = np.repeat(np.arange(K), np.floor(sizes).astype(int))[:N]
    code = np.r_[code, np.full(N - len(code), K - 1)].astype(np.int32)
    rng.shuffle(code)
    indptr, indices, data = _csc(X)
    eng = nat.Engine(0)
    try:
        ds = eng.dataset_csc(indptr, indices, data, G, N)
        new = _run(eng, ds, code, K, mode, monkeypatch, True)
        old = _run(eng, ds, code, K, mode, monkeypatch, False)
        assert np.array_equal(new.u2, old.u2)
        assert np.array_equal(new.p, old.p, equal_nan=True)
        assert np.array_equal(new.union, old.union)
        if mode == nat.SCC_DE_FAST:
            for f in ("row_pair", "gene", "u2", "ties", "p", "q"):
                assert np.array_equal(getattr(new.rows, f), getattr(old.rows, f), equal_nan=True), f
        else:
            assert np.array_equal(new.q, old.q, equal_nan=True)
            assert np.array_equal(new.de, old.de)
    finally:
        eng.close()


def test_segment_engine_repeat_bitwise(monkeypatch):
    """Segment order and atomics order vary run to run; the sums do not."""
    N, G, K = 9000, 30, 9
    X = _matrix(N, G, seed=5)
    code = (np.arange(N) % K).astype(np.int32)
    eng = nat.Engine(0)
    try:
        ds = eng.dataset_csc(*_csc(X), G, N)
        a = _run(eng, ds, code, K, nat.SCC_DE_FAST, monkeypatch, True)
        b = _run(eng, ds, code, K, nat.SCC_DE_FAST, monkeypatch, True)
        assert np.array_equal(a.u2, b.u2) and np.array_equal(a.p, b.p, equal_nan=True)
    finally:
        eng.close()


@pytest.mark.parametrize("mode", [nat.SCC_DE_FAST, nat.SCC_DE_SLOW])
def test_oversized_segments_refined(mode, monkeypatch):
    """One sample key per segment (SCC_SEG_OVERSAMPLE=1): many interval
    segments outgrow SG_CAP and are re-cut by k_seg_refine (sorted in LDS, cut
    at value changes, the cross-sub-segment part added there)."""
    N, G, K = 16000, 24, 11
    X = _matrix(N, G, seed=9)
    code = (np.arange(N) * 7 % K).astype(np.int32)
    eng = nat.Engine(0)
    try:
        ds = eng.dataset_csc(*_csc(X), G, N)
        old = _run(eng, ds, code, K, mode, monkeypatch, False)
        monkeypatch.setenv("SCC_SEG_OVERSAMPLE", "1")
        new = _run(eng, ds, code, K, mode, monkeypatch, True)
        assert np.array_equal(new.u2, old.u2)
        assert np.array_equal(new.p, old.p, equal_nan=True)
    finally:
        eng.close()
