"""numpy model of libscc's group-pair runs (scc_runtime.cpp de_run_grouped):
more consensus clusters than one engine run ranks (128) are cut into
ceil(K / gmax) balanced groups, the engine runs once per group pair (u < v) on
the cells of those clusters (others coded -1), and each global pair (i, j) is
taken from exactly one run -- the run of its two groups, or for a pair inside
one group the first run holding that group.  The device is replaced by the
oracle here, so the CPU suite checks the decomposition itself against one
oracle run over all K (Fast:57-392, slow:69-227); tests/test_gpu_grouped.py
checks the engine's implementation."""
import numpy as np

import oracle as O


def groups(K, gmax):
    ng = -(-K // gmax)
    return [list(range(u * K // ng, (u + 1) * K // ng)) for u in range(ng)]


def runs(K, gmax):
    """[(clusters of the run, {local pair: global pair taken from it})]"""
    grp = groups(K, gmax)
    gid = {a: u for u, g in enumerate(grp) for a in g}
    covered, out = set(), []
    for u in range(len(grp)):
        for v in range(u + 1, len(grp)):
            cl = grp[u] + grp[v]
            take, lp = {}, 0
            for li in range(len(cl)):
                for lj in range(li + 1, len(cl)):
                    gi, gj = cl[li], cl[lj]
                    if gid[gi] != gid[gj] or gid[gi] not in covered:
                        take[lp] = gi * K - gi * (gi + 1) // 2 + (gj - gi - 1)
                    lp += 1
            covered.update((u, v))
            out.append((cl, take))
    return out


def _sub_code(code, cl, K):
    lut = np.full(K + 1, -1, np.int32)
    lut[cl] = np.arange(len(cl), dtype=np.int32)
    return lut[np.where(code >= 0, code, K)]


def de_fast_grouped(X, code, K, gmax, **kw):
    """(pair_tested [P], rows dict in global (i, j) order, union)"""
    P = K * (K - 1) // 2
    parts = [None] * P
    for cl, take in runs(K, gmax):
        o = O.de_fast(X, _sub_code(code, cl, K), len(cl), **kw)
        st = np.concatenate([[0], np.cumsum(o.pair_tested)])
        for lp, gp in take.items():
            sl = slice(st[lp], st[lp + 1])
            parts[gp] = dict(gene=o.row_gene[sl], p=o.row_p[sl], q=o.row_q[sl], W=o.row_W[sl], top=o.row_top[sl],
                             de=o.row_de[sl])
    assert all(p is not None for p in parts)
    tested = np.array([len(p["gene"]) for p in parts])
    rows = {f: np.concatenate([p[f] for p in parts]) for f in parts[0]}
    top = rows["gene"][rows["top"]]
    _, first = np.unique(top, return_index=True)
    return tested, rows, top[np.sort(first)]


def de_slow_grouped(X, code, K, gmax, q, fc, msf):
    """(per-pair [P][G] p, q, lfc, W, de; union)"""
    P, G = K * (K - 1) // 2, X.shape[0]
    out = {f: np.full((P, G), np.nan) for f in ("p", "q", "lfc", "W")}
    out["de"] = np.zeros((P, G), np.uint8)
    for cl, take in runs(K, gmax):
        o = O.de_slow(X, _sub_code(code, cl, K), len(cl), q, fc, msf)
        for lp, gp in take.items():
            out["p"][gp], out["q"][gp], out["lfc"][gp], out["W"][gp] = o.p[lp], o.q[lp], o.lfc[lp], o.W[lp]
            out["de"][gp] = o.de[lp]
    union = []
    for gp in range(P):  # slow:209-227: first 30 of sort(|logfc|, decreasing) per pair, union in (i, j) order
        de = np.flatnonzero(out["de"][gp] == 1)
        o = np.argsort(-np.abs(out["lfc"][gp][de]), kind="stable")
        for g in de[o][:30]:
            if g not in union:
                union.append(g)
    return out, np.array(union, np.int32)
