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


def gene_u2_ties_sweep(values, codes, n_clu, W=4):
    """The kernel's actual sweep (scc_rank.hip step 3+4): the sorted array is
    cut into W wave chunks; each chunk keeps C_b (count of b before) and G_b
    (count of b before inside the current tie group, recovered by walking back
    when a group runs into the chunk) and accumulates
        S[a][b] += C_b, E[b][a] += G_b, X[b][a] += G_b (2 G_a + 1 + G_b)  (b < a),
        F_a += 3 G_a (G_a + 1)
    at every element of code a."""
    values = np.asarray(values, np.float64)
    codes = np.asarray(codes, np.int64)
    K = len(n_clu)
    nz = values != 0
    v, c = values[nz], codes[nz]
    order = np.lexsort((c, v))
    v, c = v[order], c[order]
    n = len(v)
    eqn = np.zeros(n, bool)
    eqn[:-1] = v[1:] == v[:-1]
    S = np.zeros((K, K), np.int64)
    E = np.zeros((K, K), np.int64)
    X = np.zeros((K, K), np.int64)
    F = np.zeros(K, np.int64)
    ch = (n + W - 1) // W if n else 0
    for w in range(W):
        c0, c1 = min(n, w * ch), min(n, w * ch + ch)
        C = np.bincount(c[:c0], minlength=K).astype(np.int64)
        G = np.zeros(K, np.int64)
        peq = False
        if c0 < c1 and c0 > 0 and eqn[c0 - 1]:
            peq = True
            j = c0 - 1
            while j >= 0 and (j == c0 - 1 or eqn[j]):
                G[c[j]] += 1
                j -= 1
        for i in range(c0, c1):
            a = c[i]
            if not peq:
                G[:] = 0
            else:
                for b in range(a):
                    if G[b]:
                        E[b, a] += G[b]
                        X[b, a] += G[b] * (2 * G[a] + 1 + G[b])
            F[a] += 3 * G[a] * (G[a] + 1)
            S[a] += C
            C[a] += 1
            G[a] += 1
            peq = bool(eqn[i])
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
