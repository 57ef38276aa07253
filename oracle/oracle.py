"""TEST INFRASTRUCTURE ONLY — Python face of the CPU oracle.

Loads ``oracle/liborc.so`` (the C restatement of the reference R semantics,
``oracle/scc_oracle.c``) through ctypes and adds the PCA + ``dist`` restatement
in numpy.  Only ``tests/``, ``__graft_entry__.smoke()`` and the ``bench.py``
``cpu_baseline`` leg import this module; the product path never does.

Parity status ("parity unpinned"): the reference is an R
package with no tests and no fixtures, and R is absent from the build
container, so the oracle is pinned by (1) hand known-answer tests taken from
R's documented outputs, (2) an independent scipy implementation of the same
statistics, and (3) exhaustive brute-force checks — not by running R.
"""
from __future__ import annotations

import ctypes
import os
import subprocess
from dataclasses import dataclass

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
_LIB = None


def build() -> str:
    path = os.path.join(_HERE, "liborc.so")
    src = os.path.join(_HERE, "scc_oracle.c")
    if not os.path.exists(path) or os.path.getmtime(path) < os.path.getmtime(src):
        subprocess.run(["make", "-s", "-C", _HERE], check=True)
    return path


def lib():
    global _LIB
    if _LIB is None:
        _LIB = ctypes.CDLL(build())
        L = _LIB
        dp = ctypes.POINTER(ctypes.c_double)
        ip = ctypes.POINTER(ctypes.c_int)
        L.orc_r_mean.restype = ctypes.c_double
        L.orc_r_mean.argtypes = [dp, ctypes.c_long]
        L.orc_pnorm.restype = ctypes.c_double
        L.orc_pnorm.argtypes = [ctypes.c_double, ctypes.c_int]
        L.orc_pwilcox.restype = ctypes.c_double
        L.orc_pwilcox.argtypes = [ctypes.c_double, ctypes.c_int, ctypes.c_int, ctypes.c_int]
        L.orc_choose.restype = ctypes.c_double
        L.orc_choose.argtypes = [ctypes.c_double, ctypes.c_double]
        L.orc_wilcox_p.restype = ctypes.c_double
        L.orc_wilcox_p.argtypes = [dp, ctypes.c_int, dp, ctypes.c_int, dp, dp, ip]
        L.orc_p_adjust_bh.restype = None
        L.orc_p_adjust_bh.argtypes = [dp, ctypes.c_int, ctypes.c_long, dp]
        L.orc_nodg.restype = None
        L.orc_nodg.argtypes = [dp, ctypes.c_int, ctypes.c_int, ip]
    return _LIB


def _dp(a):
    return a.ctypes.data_as(ctypes.POINTER(ctypes.c_double))


def _ip(a):
    return a.ctypes.data_as(ctypes.POINTER(ctypes.c_int))


def _u8p(a):
    return a.ctypes.data_as(ctypes.POINTER(ctypes.c_uint8))


def r_mean(x) -> float:
    x = np.ascontiguousarray(x, dtype=np.float64)
    return lib().orc_r_mean(_dp(x), len(x))


def pnorm(x: float, lower_tail: bool = True) -> float:
    return lib().orc_pnorm(float(x), 1 if lower_tail else 0)


def pwilcox(q: float, m: int, n: int, lower_tail: bool = True) -> float:
    return lib().orc_pwilcox(float(q), int(m), int(n), 1 if lower_tail else 0)


def wilcox_test(x, y):
    """stats::wilcox.test(x, y) (two-sided, correct=TRUE, exact=NULL).

    Returns (p_value, W, tie_term, method) with method 'exact' or 'normal'."""
    x = np.ascontiguousarray(x, dtype=np.float64)
    y = np.ascontiguousarray(y, dtype=np.float64)
    W = ctypes.c_double()
    T = ctypes.c_double()
    m = ctypes.c_int()
    p = lib().orc_wilcox_p(_dp(x), len(x), _dp(y), len(y), ctypes.byref(W), ctypes.byref(T),
                           ctypes.byref(m))
    return p, W.value, T.value, ("exact" if m.value == 1 else "normal")


def p_adjust_bh(p, n=None):
    p = np.ascontiguousarray(p, dtype=np.float64)
    q = np.empty_like(p)
    lib().orc_p_adjust_bh(_dp(p), len(p), -1 if n is None else int(n), _dp(q))
    return q


@dataclass
class FastResult:
    pair_tested: np.ndarray   # [P] tested features per pair
    row_pair: np.ndarray      # [R]
    row_gene: np.ndarray
    row_p: np.ndarray
    row_q: np.ndarray
    row_lfc: np.ndarray       # signed avg_logFC (natural log)
    row_pct1: np.ndarray
    row_pct2: np.ndarray
    row_W: np.ndarray         # wilcox STATISTIC (U of cluster i)
    row_ties: np.ndarray      # sum(NTIES^3 - NTIES)
    row_de: np.ndarray        # q < qValThrs and pair kept (tested > 1)
    row_top: np.ndarray       # survived top_n
    union: np.ndarray         # deGeneUnion (gene indices, R order)
    status: int = 0           # 5 (RSTOP): R's t.test stops on constant data


def _check_dense(X, code, K):
    X = np.ascontiguousarray(X, dtype=np.float64)
    code = np.ascontiguousarray(code, dtype=np.int32)
    G, N = X.shape
    assert code.shape == (N,)
    assert code.max() < K
    return X, code, G, N


def t_test_p(x, y):
    """stats::t.test(x, y)$p.value (Welch); (p, constant) where constant means
    R stops with "data are essentially constant"."""
    L = lib()
    x = np.ascontiguousarray(x, np.float64)
    y = np.ascontiguousarray(y, np.float64)
    f = L.orc_t_test_p
    f.restype = ctypes.c_double
    t = ctypes.c_double()
    c = ctypes.c_int()
    p = f(_dp(x), len(x), _dp(y), len(y), ctypes.byref(t), ctypes.byref(c))
    return p, bool(c.value)


def pt(x, n, lower_tail=True):
    f = lib().orc_pt
    f.restype = ctypes.c_double
    f.argtypes = [ctypes.c_double, ctypes.c_double, ctypes.c_int]
    return f(x, n, 1 if lower_tail else 0)


def de_fast(X, code, K, q_val_thrs=0.1, log_fc_thrs=0.5, min_per_cent=20.0, top_n=30, test="wilcox") -> FastResult:
    """reclusterDEConsensusFast DE stage. X is gene-major dense (G x N).
    test: "wilcox" (WilcoxDETest) or "t" (DiffTTest)."""
    L = lib()
    X, code, G, N = _check_dense(X, code, K)
    P = K * (K - 1) // 2

    class Prm(ctypes.Structure):
        _fields_ = [("q", ctypes.c_double), ("lfc", ctypes.c_double), ("mpc", ctypes.c_double),
                    ("top", ctypes.c_int), ("test", ctypes.c_int), ("status", ctypes.c_int)]

    prm = Prm(q_val_thrs, log_fc_thrs, min_per_cent, top_n, 1 if test == "t" else 0, 0)
    cap = max(1, P * G)
    tested = np.zeros(P, np.int32)
    gene = np.zeros(cap, np.int32)
    arr = {k: np.zeros(cap, np.float64) for k in ("p", "q", "lfc", "pct1", "pct2", "W", "T")}
    flags = np.zeros(cap, np.uint8)
    uni = np.zeros(G, np.int32)
    nu = ctypes.c_int()
    f = L.orc_de_fast
    f.restype = ctypes.c_long
    nrows = f(_dp(X), G, N, _ip(code), K, ctypes.byref(prm), _ip(tested), _ip(gene), _dp(arr["p"]),
              _dp(arr["q"]), _dp(arr["lfc"]), _dp(arr["pct1"]), _dp(arr["pct2"]), _dp(arr["W"]),
              _dp(arr["T"]), _u8p(flags), _ip(uni), ctypes.byref(nu))
    pair = np.repeat(np.arange(P, dtype=np.int32), tested)
    return FastResult(tested, pair, gene[:nrows].copy(), arr["p"][:nrows].copy(), arr["q"][:nrows].copy(),
                      arr["lfc"][:nrows].copy(), arr["pct1"][:nrows].copy(), arr["pct2"][:nrows].copy(),
                      arr["W"][:nrows].copy(), arr["T"][:nrows].copy(), (flags[:nrows] & 1) > 0,
                      (flags[:nrows] & 2) > 0, uni[: nu.value].copy(), prm.status)


@dataclass
class SlowResult:
    p: np.ndarray      # [P, G]
    q: np.ndarray
    lfc: np.ndarray
    W: np.ndarray
    ties: np.ndarray
    de: np.ndarray     # uint8 0/1 (2 = NA, R would stop)
    union: np.ndarray
    log_thr: float
    status: int


def de_slow(X, code, K, q_val_thrs, fc_thrs, mean_scaling_factor=5.0) -> SlowResult:
    """reclusterDEConsensus (method = "Wilcoxon") DE stage."""
    L = lib()
    X, code, G, N = _check_dense(X, code, K)
    P = K * (K - 1) // 2

    class Prm(ctypes.Structure):
        _fields_ = [("q", ctypes.c_double), ("fc", ctypes.c_double), ("msf", ctypes.c_double)]

    prm = Prm(q_val_thrs, fc_thrs, mean_scaling_factor)
    out = {k: np.zeros((P, G), np.float64) for k in ("p", "q", "lfc", "W", "T")}
    de = np.zeros((P, G), np.uint8)
    uni = np.zeros(G, np.int32)
    nu = ctypes.c_int()
    lthr = ctypes.c_double()
    f = L.orc_de_slow
    f.restype = ctypes.c_int
    st = f(_dp(X), G, N, _ip(code), K, ctypes.byref(prm), _dp(out["p"]), _dp(out["q"]), _dp(out["lfc"]),
           _dp(out["W"]), _dp(out["T"]), _u8p(de), _ip(uni), ctypes.byref(nu), ctypes.byref(lthr))
    return SlowResult(out["p"], out["q"], out["lfc"], out["W"], out["T"], de, uni[: nu.value].copy(),
                      lthr.value, st)


def nodg(X):
    X = np.ascontiguousarray(X, dtype=np.float64)
    G, N = X.shape
    out = np.zeros(N, np.int32)
    lib().orc_nodg(_dp(X), G, N, _ip(out))
    return out


# ------------------------------------------------------------------ distance
def pca_scores(X, genes, ncomp=None):
    """irlba::prcomp_irlba(t(X[genes, ]), n = min(|U|, 15), center = TRUE,
    scale. = FALSE)$x restated as an EXACT truncated SVD (reference
    R/reclusterDEConsensusFast.R:398).  irlba uses a random start and a 1e-5
    tolerance; the exact SVD is the deterministic quantity both
    approximate.  Component signs are arbitrary and do not affect ``dist``."""
    Xu = np.asarray(X, dtype=np.float64)[np.asarray(genes)].T  # N x |U|
    k = min(len(genes), 15) if ncomp is None else ncomp
    Xc = Xu - Xu.mean(axis=0, keepdims=True)
    U, S, _ = np.linalg.svd(Xc, full_matrices=False)
    return U[:, :k] * S[:k]


def dist_euclidean(scores):
    """stats::dist(x, "euclidean") packed lower triangle (R column-major order,
    identical to scipy's condensed order).  Reference Fast:400."""
    from scipy.spatial.distance import pdist
    return pdist(np.asarray(scores, dtype=np.float64), "euclidean")


def dist_pearson(X, genes):
    """as.dist(1 - cor(X[genes, ], method = "pearson")) (reference Fast:403,
    the commented-out alternative) — cells are the variables."""
    from scipy.spatial.distance import squareform
    Xu = np.asarray(X, dtype=np.float64)[np.asarray(genes)]
    C = np.corrcoef(Xu.T)
    D = 1.0 - C
    np.fill_diagonal(D, 0.0)
    return squareform(D, checks=False)


# ---------------------------------------------------------------------------
# Host clustering restatements, checkers for libscc's
# scc_hclust_ward_d2 / scc_cutree_hybrid.  Pure Python, small N only.
#
# hclust(ward.D2) (fastcluster, Fast:406-411) is pinned to scipy's Ward
# linkage, which fastcluster's documentation names as the same method
# ("ward.D2" in R == "ward" in Python): ward_d2_r converts scipy's linkage to
# R's hclust merge / height convention.  cutreeDynamic(hybrid, pamStage =
# FALSE) (dynamicTreeCut, Fast:421-427) has no independent implementation in
# this image: cutree_hybrid below restates the package's published
# cutreeHybrid line by line on a full distM (R vectors, 1-based branch ids),
# and is itself "parity unpinned" — it cross-checks the C++ restatement and
# is checked against hand-worked dendrograms in tests/test_cluster.py.

def ward_d2_r(dist_packed, n):
    """R hclust(d, "ward.D2") merge (n-1 x 2, R convention), height via scipy."""
    from scipy.cluster.hierarchy import linkage
    Z = linkage(np.asarray(dist_packed, np.float64), method="ward")
    merge = np.zeros((n - 1, 2), np.int64)
    for k in range(n - 1):
        a, b = sorted((int(Z[k, 0]), int(Z[k, 1])))
        merge[k] = [-(a + 1) if a < n else a - n + 1, -(b + 1) if b < n else b - n + 1]
    return merge, Z[:, 2].copy()


def _interpolate(data, index):
    i = round(index)  # Python round == R round (half to even)
    n = len(data)
    if i < 1:
        return data[0]
    if i >= n:
        return data[n - 1]
    r = index - i
    return data[i - 1] * (1 - r) + data[i] * r


def _core_size(branch_size, min_cluster_size):
    base = min_cluster_size / 2 + 1
    return int(base + np.sqrt(branch_size - base)) if base < branch_size else branch_size


def cutree_hybrid(merge, height, distM, deepSplit=1, minClusterSize=20):
    """dynamicTreeCut::cutreeHybrid(..., pamStage = FALSE)$labels."""
    merge = np.asarray(merge)
    height = np.asarray(height, np.float64)
    nMerge = len(height)
    nPoints = nMerge + 1
    refMerge = max(int(round(nMerge * 0.05)), 1)
    refHeight = height[refMerge - 1]
    cutHeight = 0.99 * (height.max() - refHeight) + refHeight
    nMergeBelowCut = int((height <= cutHeight).sum())
    if nMergeBelowCut < minClusterSize:
        return np.zeros(nPoints, np.int64)
    defMCS = [0.64, 0.73, 0.82, 0.91, 0.95]
    defMG = [(1 - x) * 3 / 4 for x in defMCS]
    ds = deepSplit + 1
    maxCoreScatter = _interpolate(defMCS, ds)
    minGap = _interpolate(defMG, ds)
    maxAbsCoreScatter = refHeight + maxCoreScatter * (cutHeight - refHeight)
    minAbsGap = minGap * (cutHeight - refHeight)
    minAbsSplitHeight = refHeight + 0 * (cutHeight - refHeight)

    isBasic, isTopBasic, failSize, attachHeight = {}, {}, {}, {}
    size, singletons, basicClusters, mergedInto = {}, {}, {}, {}
    IndMergeToBranch = [0] * nMerge
    nBranches = 0

    def scatter(b):
        cs = _core_size(len(singletons[b]), minClusterSize)
        core = np.array(singletons[b][:cs]) - 1
        sub = distM[np.ix_(core, core)]
        return float(np.mean(sub.sum(axis=0) / (cs - 1)))

    for m in range(nMerge):
        if not height[m] <= cutHeight:
            continue
        a, b = int(merge[m, 0]), int(merge[m, 1])
        h = height[m]
        if a < 0 and b < 0:
            nBranches += 1
            isBasic[nBranches] = isTopBasic[nBranches] = True
            failSize[nBranches] = False
            attachHeight[nBranches] = None
            size[nBranches] = 2
            singletons[nBranches] = [-a, -b]
            basicClusters[nBranches] = []
            IndMergeToBranch[m] = nBranches
        elif (a < 0) != (b < 0):
            clust = IndMergeToBranch[max(a, b) - 1]
            gene = -min(a, b)
            if isBasic[clust]:
                singletons[clust].append(gene)
            size[clust] += 1
            IndMergeToBranch[m] = clust
        else:
            clusts = [IndMergeToBranch[a - 1], IndMergeToBranch[b - 1]]
            sizes = [size[c] for c in clusts]
            small, large = (clusts[1], clusts[0]) if sizes[0] > sizes[1] else (clusts[0], clusts[1])
            SmAveDist = scatter(small) if isBasic[small] else 0.0
            LgAveDist = scatter(large) if isBasic[large] else 0.0
            Sm = [isBasic[small], size[small] < minClusterSize, SmAveDist > maxAbsCoreScatter,
                  h - SmAveDist < minAbsGap, h < minAbsSplitHeight]
            if Sm[0] and sum(Sm[1:]) > 0:
                DoMerge, SmallerFailSize = True, not (Sm[2] or Sm[3])
            else:
                Lg = [isBasic[large], size[large] < minClusterSize, LgAveDist > maxAbsCoreScatter,
                      h - LgAveDist < minAbsGap, h < minAbsSplitHeight]
                if Lg[0] and sum(Lg[1:]) > 0:
                    DoMerge, SmallerFailSize = True, not (Lg[2] or Lg[3])
                    small, large = large, small
                else:
                    DoMerge = False
            if DoMerge:
                failSize[small] = SmallerFailSize
                mergedInto[small] = large
                attachHeight[small] = h
                isTopBasic[small] = False
                if isBasic[large]:
                    singletons[large] = singletons[large] + singletons[small]
                size[large] += size[small]
                IndMergeToBranch[m] = large
            else:
                if isBasic[large] and not isBasic[small]:
                    small, large = large, small
                if isBasic[large]:
                    nBranches += 1
                    attachHeight[large] = attachHeight[small] = h
                    mergedInto[large] = mergedInto[small] = nBranches
                    add = [small] if isBasic[small] else list(basicClusters[small])
                    add += [large] if isBasic[large] else list(basicClusters[large])
                    isBasic[nBranches] = isTopBasic[nBranches] = False
                    failSize[nBranches] = False
                    attachHeight[nBranches] = None
                    basicClusters[nBranches] = add
                    singletons[nBranches] = []
                    size[nBranches] = size[small] + size[large]
                    IndMergeToBranch[m] = nBranches
                else:
                    add = [small] if isBasic[small] else list(basicClusters[small])
                    basicClusters[large] = basicClusters[large] + add
                    size[large] += size[small]
                    attachHeight[small] = h
                    mergedInto[small] = large
                    IndMergeToBranch[m] = large

    Colors = np.zeros(nPoints, np.int64)
    color = 0
    for clust in range(1, nBranches + 1):
        if attachHeight[clust] is None:
            attachHeight[clust] = cutHeight
        if isTopBasic[clust]:
            cs = scatter(clust)
            if size[clust] >= minClusterSize and cs < maxAbsCoreScatter and attachHeight[clust] - cs > minAbsGap:
                color += 1
                Colors[np.array(singletons[clust]) - 1] = color
    # relabel by decreasing size, 0 (unlabeled) kept
    counts = np.bincount(Colors, minlength=color + 1)
    order = sorted(range(1, color + 1), key=lambda c: (-counts[c], c))
    rel = np.zeros(color + 1, np.int64)
    for r, c in enumerate(order):
        rel[c] = r + 1
    return rel[Colors]
