"""More consensus clusters than one engine run holds (> 128).

The rank kernels hold a cluster in 7 bits, so one scc_de_run covers up to 128
clusters (BASELINE config E's K = 100 is one run).  Every per-pair quantity of the
FAST path is a function of the pair's two clusters alone (pct, log-mean
logFC, the filters, the Wilcoxon test, BH with the pair's own tested-row
count, the pair's top-N; Fast:57-392), so the K clusters are cut into groups
of <= 64 and the engine runs once per group pair (u < v) on the cells of
those <= 128 clusters (the rest get code -1).  Each global pair (i, j) is taken
from exactly one run -- the run of its two groups, or for a pair inside one
group the first run containing that group -- and the rows are concatenated
in the reference's (i, j) order; the union is `unique(Gene)` over the top
rows in that order (Fast:386-392).  Local cluster order follows global order
inside every run, so Cluster1 / Cluster2 orientation is preserved.

Host orchestration only: all statistics come from the device runs.
"""
from __future__ import annotations

import numpy as np

from . import _native as nat

GROUP = 64
MIN_K = 129  # K <= 128: one engine run


def _groups(K, group):
    return [np.arange(s, min(K, s + group)) for s in range(0, K, group)]


def de_fast_grouped(eng, ds, code, K, group=GROUP, min_k=MIN_K, **kw) -> nat.DeResult:
    """scc_de_run(SCC_DE_FAST, fetch="rows") for any K (group <= 64); K < min_k
    runs the engine once."""
    code = np.ascontiguousarray(code, np.int32)
    if K < min_k:
        return eng.de_run(ds, code, K, nat.SCC_DE_FAST, fetch="rows", **kw)
    if not 2 <= group <= 64:
        raise ValueError("group must be in [2, 64]")
    grp = _groups(K, group)
    gid = np.concatenate([np.full(len(g), u) for u, g in enumerate(grp)])
    P = K * (K - 1) // 2
    pair_of = {}
    for i in range(K):
        for j in range(i + 1, K):
            pair_of[(i, j)] = len(pair_of)
    taken_within = set()
    parts = [None] * P   # per global pair: (local run rows slice)
    tested = np.zeros(P, np.int64)
    nodg = None
    runs = [(u, v) for u in range(len(grp)) for v in range(u + 1, len(grp))] if len(grp) > 1 else [(0, 0)]
    for (u, v) in runs:
        clusters = np.concatenate([grp[u], grp[v]]) if u != v else grp[u]
        lut = np.full(K + 1, -1, np.int32)
        lut[clusters] = np.arange(len(clusters), dtype=np.int32)
        sub = lut[np.where(code >= 0, code, K)]
        r = eng.de_run(ds, sub, len(clusters), nat.SCC_DE_FAST, fetch="rows", **kw)
        if r.status:
            return r
        if nodg is None:
            nodg = r.nodg
        rows = r.rows
        Kl = len(clusters)
        lp = 0
        starts = np.concatenate([[0], np.cumsum(rows.pair_tested)])
        for li in range(Kl):
            for lj in range(li + 1, Kl):
                gi, gj = int(clusters[li]), int(clusters[lj])
                gu, gv = gid[gi], gid[gj]
                if gu != gv:
                    want = True
                else:
                    want = gu not in taken_within
                if want:
                    p = pair_of[(gi, gj)]
                    parts[p] = (rows, starts[lp], starts[lp + 1])
                    tested[p] = rows.pair_tested[lp]
                lp += 1
        taken_within.update({u, v})
    fields = ("gene", "p", "q", "avg_logfc", "pct1", "pct2", "u2", "ties", "de", "top")
    cat = {f: [] for f in fields}
    row_pair = []
    for p in range(P):
        rows, a, b = parts[p]
        for f in fields:
            cat[f].append(getattr(rows, f)[a:b])
        row_pair.append(np.full(b - a, p, np.int32))
    out = {f: np.concatenate(cat[f]) for f in fields}
    fr = nat.FastRows(pair_tested=tested, row_pair=np.concatenate(row_pair), **out)
    top_genes = fr.gene[fr.top.astype(bool)]
    _, first = np.unique(top_genes, return_index=True)
    union = top_genes[np.sort(first)].astype(np.int32)
    return nat.DeResult(mode=nat.SCC_DE_FAST, K=K, n_pairs=P, union=union, nodg=nodg, rows=fr)


def runs_for(K, group=GROUP, min_k=MIN_K) -> int:
    """Engine runs de_fast_grouped makes for K clusters."""
    if K < min_k:
        return 1
    ng = -(-K // group)
    return max(1, ng * (ng - 1) // 2)
