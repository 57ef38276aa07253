"""Parity checks shared by the large-configuration GPU tests (configs B-E).

Two halves, so that configurations too large for a full oracle run are still
checked end to end:

* ``check_rows_against_oracle_subset`` — the oracle (C restatement of
  ``ComputePairWiseDE``, R/reclusterDEConsensusFast.R:229-351) run on a seeded
  SUBSET of genes over ALL cells and ALL pairs.  Every per-(pair, gene)
  quantity — the FAST filters (which genes a pair tests), W, the tie term, p,
  avg_logFC, pct.1/pct.2 — depends on that gene alone, so for the sampled
  genes the engine's rows must equal the oracle's exactly (and in the same
  relative order inside each pair).
* ``check_p_from_counts`` — every tested row's p at FULL size, restated in numpy
  from the row's exact 2U and tie term and the two cluster sizes
  (``wilcox.test.default``'s exact / normal rule), so that a wrong p on a gene
  the subset oracle does not sample cannot pass.
* ``check_selection`` — the per-pair selection at FULL size, restated in numpy
  from the engine's own per-row statistics: R's row order ``order(p,
  -avg_logFC)`` (Fast:346), BH with the lazy n (Fast:347-350), the
  ``dim(tmp)[1] > 1`` / ``q < qValThrs`` rule (Fast:376-377), ``top_n`` with
  ties (Fast:391) and ``unique(Gene)`` (Fast:392).

Test infrastructure only (imports the oracle).
"""
from __future__ import annotations

import numpy as np

import oracle as O

P_RTOL = 1e-6


def pair_list(K):
    return [(i, j) for i in range(K - 1) for j in range(i + 1, K)]


def check_selection(rows, union, K, q_val_thrs=0.1, top_n=30):
    """Full-size selection parity from the engine's own rows (FAST)."""
    P = K * (K - 1) // 2
    tested = np.asarray(rows.pair_tested, np.int64)
    assert tested.shape == (P,)
    starts = np.concatenate([[0], np.cumsum(tested)])
    assert starts[-1] == len(rows.gene)
    top_rows = []
    for p in range(P):
        a, b = int(starts[p]), int(starts[p + 1])
        if a == b:
            continue
        g, pv, lfc = rows.gene[a:b], rows.p[a:b], rows.avg_logfc[a:b]
        # order(p, -avg_logFC): p ascending with NaN last, then logFC descending, then gene row
        nan = np.isnan(pv)
        order = np.lexsort((g, -lfc, np.where(nan, 0.0, pv), nan))
        assert np.array_equal(order, np.arange(b - a)), f"pair {p}: rows not in R's order(p, -avg_logFC)"
        assert len(np.unique(g)) == b - a, f"pair {p}: repeated gene"
        q = O.p_adjust_bh(pv)
        np.testing.assert_allclose(rows.q[a:b], q, rtol=1e-12, atol=0, equal_nan=True,
                                   err_msg=f"pair {p}: BH q")
        de = (b - a > 1) & (rows.q[a:b] < q_val_thrs)
        assert np.array_equal(rows.de[a:b], de), f"pair {p}: kept-row flags"
        w = np.abs(lfc)
        wd = w[de]
        above = (wd[None, :] > w[:, None]).sum(axis=1)
        top = de & (above + 1 <= top_n)
        assert np.array_equal(rows.top[a:b], top), f"pair {p}: top_n flags"
        top_rows.append(g[top])
    top_genes = np.concatenate(top_rows) if top_rows else np.zeros(0, np.int32)
    _, first = np.unique(top_genes, return_index=True)
    np.testing.assert_array_equal(union, top_genes[np.sort(first)])


def check_p_from_counts(rows, code, K, rtol=1e-9):
    """R's wilcox.test.default p-value (two-sided, correct = TRUE, exact
    for n.x < 50 and n.y < 50 without ties) restated in numpy for EVERY
    tested row from the engine's exact W = u2 / 2, its tie term
    sum(NTIES^3 - NTIES) and the cluster sizes; the normal tail by
    scipy's ndtr with R's pnorm underflow (|z| > 37.5193 gives 0).  Returns the
    number of rows checked (the exact ones through the oracle's pwilcox)."""
    from scipy.special import ndtr
    P = K * (K - 1) // 2
    n = np.bincount(np.asarray(code)[np.asarray(code) >= 0], minlength=K).astype(np.float64)
    pa = np.array([i for i in range(K - 1) for j in range(i + 1, K)])
    pb = np.array([j for i in range(K - 1) for j in range(i + 1, K)])
    row_pair = np.repeat(np.arange(P), np.asarray(rows.pair_tested, np.int64))
    nx, ny = n[pa[row_pair]], n[pb[row_pair]]
    W = np.asarray(rows.u2, np.float64) / 2.0
    ties = np.asarray(rows.ties, np.float64)
    exact = (nx < 50) & (ny < 50) & (ties == 0)
    z = W - nx * ny / 2.0
    sigma = np.sqrt((nx * ny / 12.0) * ((nx + ny + 1.0) - ties / ((nx + ny) * (nx + ny - 1.0))))
    z = (z - np.sign(z) * 0.5) / sigma
    tail = np.where(-np.abs(z) < -37.5193, 0.0, ndtr(-np.abs(z)))
    want = np.minimum(1.0, 2.0 * tail)
    for k in np.flatnonzero(exact):  # (rare at B-E: clusters of < 50 cells)
        m, nn, q = int(nx[k]), int(ny[k]), W[k]
        p = O.pwilcox(q, m, nn) if q <= m * nn / 2 else O.pwilcox(q - 1, m, nn, lower_tail=False)
        want[k] = min(1.0, 2.0 * p)
    got = np.asarray(rows.p, np.float64)
    np.testing.assert_allclose(got, want, rtol=rtol, atol=1e-300, err_msg="p from (2U, ties, n.x, n.y)")
    return len(got)


def check_rows_against_oracle_subset(rows, Xsub, genes, code, K, **params):
    """The oracle on genes ``genes`` (dense rows ``Xsub`` over all cells) vs the
    engine's rows restricted to those genes: the same tested (pair, gene) set
    in the same relative order, exact W / ties, pct, and p, logFC within the
    bar.  Returns the number of (pair, gene) rows compared."""
    genes = np.asarray(genes)
    o = O.de_fast(Xsub, code, K, **params)
    P = K * (K - 1) // 2
    gstarts = np.concatenate([[0], np.cumsum(rows.pair_tested)])
    ostarts = np.concatenate([[0], np.cumsum(o.pair_tested)])
    n = 0
    for p in range(P):
        a, b = int(gstarts[p]), int(gstarts[p + 1])
        g = rows.gene[a:b]
        sel = np.nonzero(np.isin(g, genes))[0]
        oa, ob = int(ostarts[p]), int(ostarts[p + 1])
        og = genes[o.row_gene[oa:ob]]
        assert np.array_equal(g[sel], og), f"pair {p}: tested genes / order differ from the oracle"
        r = a + sel
        np.testing.assert_array_equal(rows.u2[r], np.round(2 * o.row_W[oa:ob]).astype(np.int64), err_msg=f"pair {p} 2U")
        np.testing.assert_array_equal(rows.ties[r], np.round(o.row_ties[oa:ob]).astype(np.int64),
                                      err_msg=f"pair {p} ties")
        np.testing.assert_allclose(rows.p[r], o.row_p[oa:ob], rtol=P_RTOL, atol=0, equal_nan=True,
                                   err_msg=f"pair {p} p")
        np.testing.assert_allclose(rows.avg_logfc[r], o.row_lfc[oa:ob], rtol=1e-12, atol=5e-14,
                                   err_msg=f"pair {p} logFC")
        np.testing.assert_array_equal(rows.pct1[r], o.row_pct1[oa:ob], err_msg=f"pair {p} pct.1")
        np.testing.assert_array_equal(rows.pct2[r], o.row_pct2[oa:ob], err_msg=f"pair {p} pct.2")
        n += ob - oa
    return n


def rows_of_gene_major(indptr, cols, vals, genes, N):
    """Dense rows (len(genes) x N) from a gene-major CSR held as numpy arrays
    or torch tensors (device or host)."""
    out = np.zeros((len(genes), N))
    for k, g in enumerate(np.asarray(genes)):
        a, b = int(indptr[g]), int(indptr[g + 1])
        c = cols[a:b]
        v = vals[a:b]
        if hasattr(c, "cpu"):
            c, v = c.cpu().numpy(), v.cpu().numpy()
        out[k, np.asarray(c, np.int64)] = v
    return out


def packed_index(i, j, N):
    """Entry of cells i > j in R's packed `dist` vector (column-major lower triangle)."""
    i = np.asarray(i, np.int64)
    j = np.asarray(j, np.int64)
    return j * (2 * N - j - 1) // 2 + (i - j - 1)


def sample_cell_pairs(N, n, seed):
    rng = np.random.default_rng(seed)
    a = rng.integers(0, N, n)
    b = rng.integers(0, N - 1, n)
    b = np.where(b >= a, b + 1, b)
    return np.maximum(a, b), np.minimum(a, b)


def slow_gate(Xs, code, K, log_thr):
    """The SLOW expression gate of genes ``Xs`` (dense rows over all cells),
    [P][len(Xs)] bool: mean(x_i) > log(thr) | mean(x_j) > log(thr) with R's
    long-double two-pass mean (slow:109-113)."""
    m = np.array([[O.r_mean(x[code == a]) for a in range(K)] for x in Xs])  # [genes][K]
    up = m > log_thr
    return np.array([up[:, i] | up[:, j] for i, j in pair_list(K)])


def slow_log_threshold(vals, G, N, mean_scaling_factor):
    """log(meanScalingFactor * mean(expm1(X))) (slow:36) from the stored values
    (zeros add expm1(0) = 0), R's LDOUBLE two-pass mean."""
    e = np.expm1(np.asarray(vals, np.float64)).astype(np.longdouble)
    tot = np.longdouble(G) * np.longdouble(N)
    s = e.sum() / tot
    t = (e - s).sum() + (tot - len(e)) * (-s)
    s = s + t / tot
    return float(np.log(np.longdouble(mean_scaling_factor) * np.longdouble(float(s))))


def check_slow_selection(g, q_val_thrs, fc_thrs, gate=None, gate_genes=None):
    """SLOW selection at FULL size from the engine's per-pair vectors [P][G]:
    BH with n = G, NaN counted (slow:116-121); every DE flag implies q <
    qValThrs & |logfc| > log(fcThrs) (slow:165-170) and, where ``gate`` is
    given (for ``gate_genes``, default all), equals it exactly; the union of
    the first 30 of sort(|logfc|, decreasing) per pair in (i, j) order
    (slow:209-227)."""
    P, G = g.p.shape
    cut = np.log(fc_thrs)
    cols = np.arange(G) if gate_genes is None else np.asarray(gate_genes)
    union, seen = [], set()
    for p in range(P):
        q = O.p_adjust_bh(g.p[p], n=G)
        np.testing.assert_allclose(g.q[p], q, rtol=1e-12, atol=0, equal_nan=True, err_msg=f"pair {p}: BH q (n = G)")
        must = ~np.isnan(q) & (q < q_val_thrs) & (np.abs(g.logfc[p]) > cut)
        de = g.de[p] == 1
        assert not np.any(de & ~must), f"pair {p}: DE flag without q / logFC"
        if gate is not None:
            np.testing.assert_array_equal(de[cols], must[cols] & gate[p], err_msg=f"pair {p}: DE flags")
        idx = np.flatnonzero(de)
        o = np.argsort(-np.abs(g.logfc[p][idx]), kind="stable")
        for gene in idx[o][:30]:
            if gene not in seen:
                seen.add(gene)
                union.append(gene)
    np.testing.assert_array_equal(g.union, np.array(union, np.int32))


def check_slow_against_oracle_subset(g, Xs, genes, code, K, q_val_thrs, fc_thrs, msf):
    """The oracle (orc_de_slow, slow:69-187) on a gene subset over ALL cells
    and pairs: exact W, p and logFC within the bar (q and the gate depend on
    all genes: check_slow_selection).  Returns the number of cells compared."""
    o = O.de_slow(Xs, code, K, q_val_thrs, fc_thrs, msf)
    genes = np.asarray(genes)
    np.testing.assert_array_equal(g.u2[:, genes], np.round(2 * o.W).astype(np.int64), err_msg="2U")
    np.testing.assert_allclose(g.p[:, genes], o.p, rtol=P_RTOL, atol=0, equal_nan=True, err_msg="p")
    np.testing.assert_allclose(g.logfc[:, genes], o.lfc, rtol=1e-12, atol=5e-14, err_msg="logFC")
    return o.p.size
