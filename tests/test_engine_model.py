"""CPU: the engine's count-based rank-sum algorithm (modelled in numpy by
tests/engine_model.py, mirroring scc_rank.hip) equals R's rank definition
(the oracle) exactly, including zeros, negatives and cross-cluster ties."""
import numpy as np
import pytest
from hypothesis import given, settings
from hypothesis import strategies as st

import engine_model as M
import oracle as O


def _check(vals, codes, sizes):
    u2, tt = M.gene_u2_ties(vals, codes, sizes)
    K = len(sizes)
    for a in range(K - 1):
        for b in range(a + 1, K):
            _, W, T, _ = O.wilcox_test(vals[codes == a], vals[codes == b])
            assert u2[(a, b)] == int(round(2 * W))
            assert tt[(a, b)] == int(round(T))


@settings(max_examples=150, deadline=None)
@given(st.lists(st.tuples(st.integers(0, 3), st.sampled_from([0.0, 0.0, 0.0, 1.0, 2.0, -1.0, 0.5, 3.25])),
                min_size=2, max_size=40))
def test_count_formula_hypothesis(cells):
    codes = np.array([c for c, _ in cells])
    vals = np.array([v for _, v in cells])
    present = np.unique(codes)
    if len(present) < 2:
        return
    remap = {c: i for i, c in enumerate(present)}
    codes = np.array([remap[c] for c in codes])
    sizes = np.bincount(codes)
    _check(vals, codes, sizes)


def test_count_formula_continuous():
    rng = np.random.default_rng(3)
    for _ in range(50):
        K = int(rng.integers(2, 6))
        sizes = rng.integers(1, 30, K)
        codes = np.repeat(np.arange(K), sizes)
        rng.shuffle(codes)
        vals = np.where(rng.random(len(codes)) < 0.5, 0.0, np.log1p(rng.gamma(2, 2, len(codes))))
        _check(vals, codes, sizes)


@pytest.mark.parametrize("seed", range(8))
@pytest.mark.parametrize("target,bits", [(4, 11), (8, 3), (1000, 11), (3, 1)])
def test_bucketed_engine_matches(seed, target, bits):
    """Value buckets with cross-bucket histogram terms, per-bucket sorted
    positions + binary searches, and run-based tie statistics (the kernel
    pipeline) == the direct count formula, for many bucket shapes (fat bins,
    single-bin genes, buckets of one distinct value)."""
    from engine_model import gene_u2_ties, gene_u2_ties_buckets
    rng = np.random.default_rng(seed)
    K = int(rng.integers(2, 7))
    N = int(rng.integers(5, 150))
    codes = rng.integers(0, K, N)
    codes[:K] = np.arange(K)
    vals = rng.choice([-2.0, -1.0, 0.0, 0.0, 1.0, 1.5, 2.0, 3.0], N) if seed % 2 else np.round(rng.normal(0, 1, N), 1)
    n_clu = np.bincount(codes, minlength=K)
    a = gene_u2_ties(vals, codes, n_clu)
    b = gene_u2_ties_buckets(vals, codes, n_clu, target, bits)
    assert a == b
