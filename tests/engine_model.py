"""Pure-numpy model of the GPU rank kernel's ALGORITHM (scconsensus_amd/csrc/
scc_rank.hip), used only by tests to validate the count formula on the CPU
against the oracle's R-style rank sums.  Not product code.

Per gene: kept nonzeros sorted by (value, cluster code); S[a][b] = number of
b-elements at earlier positions than each a-element (summed); with ties
ordered by code, for a < b this is #{(x in a, y in b): x > y}.  Zeros are the
implicit tie group placed between negatives and positives:
    2U_ab = 2*(S_ab + z_a*neg_b + pos_a*z_b) + E_ab + z_a*z_b
    T_ab  = F_a + F_b + f(z_a) + f(z_b) + 3*(X_ab + z_a*z_b*(z_a+z_b))
"""
import numpy as np


def f(c):
    c = np.asarray(c, dtype=np.int64)
    return c * c * c - c


def gene_u2_ties(values, codes, n_clu):
    """values/codes: all kept cells of one gene (zeros included); returns
    dicts (a,b)->2U and (a,b)->T for a < b."""
    values = np.asarray(values, np.float64)
    codes = np.asarray(codes, np.int64)
    K = len(n_clu)
    nz = values != 0
    v, c = values[nz], codes[nz]
    order = np.lexsort((c, v))  # by value, then code
    v, c = v[order], c[order]
    n = len(v)
    S = np.zeros((K, K), np.int64)
    C = np.zeros(K, np.int64)
    for i in range(n):
        S[c[i]] += C
        C[c[i]] += 1
    pos = np.array([np.sum((values > 0) & (codes == a)) for a in range(K)], np.int64)
    neg = np.array([np.sum((values < 0) & (codes == a)) for a in range(K)], np.int64)
    z = np.asarray(n_clu, np.int64) - pos - neg
    F = np.zeros(K, np.int64)
    E = np.zeros((K, K), np.int64)
    X = np.zeros((K, K), np.int64)
    i = 0
    while i < n:
        e = i + 1
        while e < n and v[e] == v[i]:
            e += 1
        if e - i >= 2:
            runs = []
            r = i
            while r < e:
                r2 = r + 1
                while r2 < e and c[r2] == c[r]:
                    r2 += 1
                runs.append((c[r], r2 - r))
                r = r2
            for ai, (a, ca) in enumerate(runs):
                if ca >= 2:
                    F[a] += f(ca)
                for b, cb in runs[ai + 1:]:
                    E[a, b] += ca * cb
                    X[a, b] += ca * cb * (ca + cb)
        i = e
    u2, tt = {}, {}
    for a in range(K - 1):
        for b in range(a + 1, K):
            s = S[a, b] + z[a] * neg[b] + pos[a] * z[b]
            u2[(a, b)] = int(2 * s + E[a, b] + z[a] * z[b])
            tt[(a, b)] = int(F[a] + F[b] + f(z[a]) + f(z[b]) + 3 * (X[a, b] + z[a] * z[b] * (z[a] + z[b])))
    return u2, tt


def _okey(v):
    """orderable u64 key of a double (scc_common.hpp scc_key_of)."""
    b = np.asarray(v, np.float64).view(np.uint64)
    neg = (b >> np.uint64(63)) == 1
    return np.where(neg, ~b, b | np.uint64(1 << 63))


def gene_u2_ties_buckets(values, codes, n_clu, target=8, bins_bits=11):
    """The kernel pipeline (scc_rank.hip): the nonzeros are cut into value
    buckets (k_rank_split: 2^bins_bits-bin histogram of the key window, runs
    of bins with equal floor(excl / target), fat bins alone); the
    cross-bucket part of S comes from per-bucket cluster histograms; inside a
    bucket (k_rank_item) the elements are sorted by (value, cluster), the
    sorted positions are partitioned by cluster, S_ab is the sum of binary
    searches of the smaller cluster's positions in the larger one's, and the
    tie statistics come from runs of equal (value, cluster)."""
    values = np.asarray(values, np.float64)
    codes = np.asarray(codes, np.int64)
    K = len(n_clu)
    nz = values != 0
    v, c = values[nz], codes[nz]
    n = len(v)
    S = np.zeros((K, K), np.int64)
    E = np.zeros((K, K), np.int64)
    X = np.zeros((K, K), np.int64)
    F = np.zeros(K, np.int64)
    if n:
        k = _okey(v)
        kmn, kmx = k.min(), k.max()
        rng = int(kmx - kmn)
        bits = rng.bit_length()
        sh = max(0, bits - bins_bits)
        d = ((k - kmn) >> np.uint64(sh)).astype(np.int64)
        nb = 1 << bins_bits
        hist = np.bincount(d, minlength=nb)
        excl = np.concatenate([[0], np.cumsum(hist)[:-1]])
        fat = hist > target
        start = np.zeros(nb, bool)
        start[0] = True
        start[1:] = fat[1:] | fat[:-1] | ((excl[1:] // target) != (excl[:-1] // target))
        bid = np.cumsum(start) - 1
        bk = bid[d]
        nbk = bid[-1] + 1
        hb = np.zeros((nbk, K), np.int64)
        np.add.at(hb, (bk, c), 1)
        for a in range(K):  # cross-bucket: x in a above every y of a lower bucket
            for b in range(K):
                below = np.concatenate([[0], np.cumsum(hb[:, b])[:-1]])
                S[a, b] += int(np.sum(hb[:, a] * below))
        for q in range(nbk):
            sel = bk == q
            vv, cc = v[sel], c[sel]
            o = np.lexsort((cc, vv))
            vv, cc = vv[o], cc[o]
            pl = [np.nonzero(cc == a)[0] for a in range(K)]  # sorted positions by cluster
            for a in range(K):
                for b in range(K):
                    if a == b:
                        continue
                    sm, lg = (pl[a], pl[b]) if len(pl[a]) <= len(pl[b]) else (pl[b], pl[a])
                    lb = np.searchsorted(lg, sm, side="left")
                    S[a, b] += int(lb.sum()) if sm is pl[a] else int((len(pl[a]) - lb).sum())
            # runs of equal (value, cluster); groups of equal value
            m = len(vv)
            starts = [i for i in range(m) if i == 0 or vv[i] != vv[i - 1] or cc[i] != cc[i - 1]] + [m]
            for r in range(len(starts) - 1):
                s0, ln = starts[r], starts[r + 1] - starts[r]
                a = cc[s0]
                if ln >= 2:
                    F[a] += f(ln)
                q2 = r
                while q2 > 0 and vv[starts[q2] - 1] == vv[starts[q2]]:
                    q2 -= 1
                    ps, lb2 = starts[q2], starts[q2 + 1] - starts[q2]
                    b = cc[ps]
                    E[b, a] += ln * lb2
                    X[b, a] += ln * lb2 * (ln + lb2)
    pos = np.array([np.sum((values > 0) & (codes == a)) for a in range(K)], np.int64)
    neg = np.array([np.sum((values < 0) & (codes == a)) for a in range(K)], np.int64)
    z = np.asarray(n_clu, np.int64) - pos - neg
    u2, tt = {}, {}
    for a in range(K - 1):
        for b in range(a + 1, K):
            s = S[a, b] + z[a] * neg[b] + pos[a] * z[b]
            u2[(a, b)] = int(2 * s + z[a] * z[b] + E[a, b])
            tt[(a, b)] = int(F[a] + F[b] + f(z[a]) + f(z[b]) + 3 * z[a] * z[b] * (z[a] + z[b]) + 3 * X[a, b])
    return u2, tt
