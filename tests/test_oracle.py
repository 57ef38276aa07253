"""CPU: pin the oracle (oracle/scc_oracle.c) before trusting it.

(1) R-documented known answers (tests/golden/r_documented_kats.json),
(2) an independent implementation (scipy) of the same statistics,
(3) brute force over the definition of the rank-sum statistic."""
import json
import math
import os

import numpy as np
import pytest
from scipy import stats

import oracle as O

GOLD = json.load(open(os.path.join(os.path.dirname(__file__), "golden", "r_documented_kats.json")))


@pytest.mark.parametrize("case", GOLD["wilcox"], ids=lambda c: c["name"])
def test_wilcox_r_documented(case):
    p, W, T, meth = O.wilcox_test(case["x"], case["y"])
    assert W == case["W"]
    assert meth == case["method"]
    if case["p"] is None:
        assert math.isnan(p)
    elif "p_digits" in case:  # R prints format.pval(digits = 4)
        assert float(f"{p:.4g}") == case["p"]
    else:
        assert p == pytest.approx(case["p"], rel=1e-14)


@pytest.mark.parametrize("case", GOLD["p_adjust_bh"])
def test_bh_r_documented(case):
    p = np.array([np.nan if v is None else v for v in case["p"]])
    q = O.p_adjust_bh(p, case["n"])
    exp = np.array([np.nan if v is None else v for v in case["q"]])
    np.testing.assert_allclose(q, exp, rtol=1e-14, equal_nan=True)


@pytest.mark.parametrize("case", GOLD["pnorm"])
def test_pnorm_r_documented(case):
    assert O.pnorm(case["x"], case["lower"]) == pytest.approx(case["p"], rel=1e-14, abs=0)


def test_pnorm_cody_matches_erfc():
    # Cody's rational approximations (R nmath/pnorm.c) vs an independent erfc
    for z in np.concatenate([np.linspace(-37.5, 8.2, 4001), [-0.6744, 0.6745, 5.656, 5.657]]):
        ref = 0.5 * math.erfc(-z / math.sqrt(2))
        if ref > 1e-300:
            assert O.pnorm(z, True) == pytest.approx(ref, rel=2e-13 * max(1.0, z * z / 10))
    assert O.pnorm(-37.52, True) == 0.0


def _r_rule_p(x, y):
    x, y = np.asarray(x, float), np.asarray(y, float)
    ties = len(np.unique(np.concatenate([x, y]))) < len(x) + len(y)
    exact = len(x) < 50 and len(y) < 50 and not ties
    r = stats.mannwhitneyu(x, y, alternative="two-sided", use_continuity=True,
                           method="exact" if exact else "asymptotic")
    return r.statistic, r.pvalue


@pytest.mark.parametrize("seed", range(40))
def test_wilcox_vs_scipy(seed):
    rng = np.random.default_rng(seed)
    nx, ny = rng.integers(2, 70, 2)
    kind = seed % 3
    if kind == 0:
        x, y = rng.normal(0, 1, nx), rng.normal(0.3, 1, ny)
    elif kind == 1:
        x, y = rng.integers(0, 5, nx).astype(float), rng.integers(0, 6, ny).astype(float)
    else:
        x = np.where(rng.random(nx) < 0.6, 0.0, rng.gamma(2, 1, nx))
        y = np.where(rng.random(ny) < 0.4, 0.0, rng.gamma(2, 1, ny))
    p, W, T, meth = O.wilcox_test(x, y)
    U, ps = _r_rule_p(x, y)
    assert W == U
    if math.isnan(ps):
        assert math.isnan(p)
    else:
        assert p == pytest.approx(ps, rel=1e-9, abs=1e-300)
    # tie term against its definition
    _, cnt = np.unique(np.concatenate([x, y]), return_counts=True)
    assert T == float(np.sum(cnt.astype(np.int64) ** 3 - cnt))


def test_rank_sum_bruteforce():
    rng = np.random.default_rng(7)
    for _ in range(200):
        x = rng.integers(-3, 4, rng.integers(1, 9)).astype(float)
        y = rng.integers(-3, 4, rng.integers(1, 9)).astype(float)
        _, W, _, _ = O.wilcox_test(x, y)
        brute = sum((a > b) + 0.5 * (a == b) for a in x for b in y)
        assert W == brute


@pytest.mark.parametrize("seed", range(10))
def test_bh_vs_scipy(seed):
    rng = np.random.default_rng(seed)
    p = rng.random(rng.integers(1, 300)) ** 3
    p[rng.random(len(p)) < 0.1] = p[0]  # ties
    q = O.p_adjust_bh(p)
    np.testing.assert_allclose(q, stats.false_discovery_control(p, method="bh"), rtol=1e-12)


def test_pwilcox_distribution_sums_to_one():
    for m, n in [(3, 4), (10, 12), (30, 31), (49, 49)]:
        assert O.pwilcox(m * n, m, n) == 1.0
        tot = O.pwilcox(m * n // 2, m, n) + O.pwilcox(m * n // 2, m, n, lower_tail=False)
        assert tot == pytest.approx(1.0, abs=1e-12)
        # symmetry of the null distribution
        assert O.pwilcox(5, m, n) == pytest.approx(O.pwilcox(m * n - 6, m, n, lower_tail=False), rel=1e-12)


def test_r_mean_long_double():
    x = np.array([1e16, 1.0, -1e16, 3.0])
    assert O.r_mean(x) == 1.0
    rng = np.random.default_rng(1)
    v = rng.gamma(0.5, 3, 5000)
    exact = math.fsum(v) / len(v)
    assert O.r_mean(v) == pytest.approx(exact, rel=2e-16)


# ------------------------------------------------------------------ t test (DiffTTest, Fast:185-196)
@pytest.mark.parametrize("seed", range(6))
def test_t_test_vs_scipy(seed):
    from scipy import stats
    rng = np.random.default_rng(seed)
    for _ in range(40):
        nx, ny = rng.integers(3, 400, 2)
        x = rng.gamma(rng.uniform(0.2, 3), 1.0, nx) * (rng.random(nx) < 0.6)
        y = rng.gamma(rng.uniform(0.2, 3), 1.0, ny) * (rng.random(ny) < 0.6) + rng.uniform(0, 2)
        p, const = O.t_test_p(x, y)
        ref = stats.ttest_ind(x, y, equal_var=False).pvalue
        assert not const
        assert abs(p - ref) <= 1e-12 * max(ref, 1e-300) + 1e-300, (p, ref)


def test_t_test_tails_and_constant():
    from scipy import stats
    x = np.r_[np.zeros(50), 10.0 + np.arange(5) * 1e-3]
    y = np.r_[np.full(60, 20.0), 20.001, 19.999]
    p, const = O.t_test_p(x, y)
    assert p == pytest.approx(stats.ttest_ind(x, y, equal_var=False).pvalue, rel=1e-10)
    _, const = O.t_test_p(np.full(5, 2.0), np.full(7, 2.0))
    assert const                                      # R: "data are essentially constant"


@pytest.mark.parametrize("df", [1.0, 2.5, 7.0, 30.0, 1e3, 1e5])
def test_pt_vs_scipy(df):
    from scipy import stats
    for t in [-40.0, -8.0, -3.0, -1.0, -0.1, 0.0, 0.5, 2.0, 6.0]:
        assert O.pt(t, df) == pytest.approx(stats.t.cdf(t, df), rel=1e-10, abs=1e-300)  # power series vs cephes


def test_de_fast_t_matches_scipy_per_row():
    from scipy import stats
    from scconsensus_amd import synth, api
    d = synth.generate("A", G=150, N=600, K=4, seed=3)
    names, code = api.select_clusters(d.labels, 10)
    X = d.dense()
    o = O.de_fast(X, code, len(names), test="t", log_fc_thrs=0.1, min_per_cent=10.0)
    assert o.status == 0 and len(o.row_gene) > 20
    pairs = [(i, j) for i in range(len(names)) for j in range(i + 1, len(names))]
    for r in range(len(o.row_gene)):
        i, j = pairs[o.row_pair[r]]
        x, y = X[o.row_gene[r], code == i], X[o.row_gene[r], code == j]
        assert o.row_p[r] == pytest.approx(stats.ttest_ind(x, y, equal_var=False).pvalue, rel=1e-10)
    assert (o.row_W == 0).all()
