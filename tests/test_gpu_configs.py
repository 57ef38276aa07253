"""GPU parity at the BASELINE.json configurations B, C and E (A is in
test_gpu_de.py, D in test_gpu_large.py).

* B (26k x 10k, K = 12, the metric's configuration): the FULL FAST result —
  every tested row, its order, exact U / ties, p, q, logFC, pct, the kept and
  top_n flags and the union — against one full oracle run (~20 s single
  threaded); every entry of the packed PCA15-Euclidean `dist` against the
  exact-SVD oracle; every entry of the Pearson `1 - cor` distance against an
  fp64 torch product.
* C (100k x 15k, K = 30) and E (1M-cell CSR, K = 100): the oracle on a seeded
  gene subset over all cells and pairs (exact tested sets, U, ties, pct; p and
  logFC within the bar), EVERY tested row's exact 2U and tie term against an
  independent full-size torch computation (tests/torch_ranksum.py: one global
  sort and prefix counts), every row's p restated from its exact 2U / ties and
  the cluster sizes, the full-size selection restated from the engine's own
  rows, and at C every one of the 5e9 `dist` entries against the exact SVD
  (fp64 torch distances from the oracle's scores, on the GPU).
"""
import time

import numpy as np
import pytest
import torch  # before the engine loads (torch's HIP runtime first)

import oracle as O
import torch_ranksum as TR
from parity_helpers import (check_p_from_counts, check_rows_against_oracle_subset, check_selection, packed_index,
                            rows_of_gene_major, sample_cell_pairs)
from scconsensus_amd import api, synth

pytestmark = pytest.mark.gpu

DIST_ATOL = 1e-5  # north_star: distance entries within 1e-5 absolute


def _free():
    import gc
    gc.collect()
    torch.cuda.synchronize()
    torch.cuda.empty_cache()


def test_config_b_full_fast_parity():
    from scconsensus_amd import _native as nat
    d = synth.generate("B")
    names, code = api.select_clusters(d.labels, 10)
    K = len(names)
    assert K == 12
    X = d.dense()
    eng = nat.Engine(0)
    ds = eng.dataset_csc(d.indptr, d.indices, d.data, d.G, d.N)
    g = eng.de_run(ds, code, K, nat.SCC_DE_FAST, fetch="rows")
    o = O.de_fast(X, code, K)
    r = g.rows
    np.testing.assert_array_equal(r.pair_tested, o.pair_tested)
    np.testing.assert_array_equal(r.gene, o.row_gene)
    np.testing.assert_array_equal(r.u2, np.round(2 * o.row_W).astype(np.int64))
    np.testing.assert_array_equal(r.ties, np.round(o.row_ties).astype(np.int64))
    np.testing.assert_allclose(r.p, o.row_p, rtol=1e-6, atol=0)
    np.testing.assert_allclose(r.q, o.row_q, rtol=1e-6, atol=0)
    np.testing.assert_allclose(r.avg_logfc, o.row_lfc, rtol=1e-12, atol=5e-14)
    np.testing.assert_array_equal(r.pct1, o.row_pct1)
    np.testing.assert_array_equal(r.pct2, o.row_pct2)
    np.testing.assert_array_equal(r.de, o.row_de)
    np.testing.assert_array_equal(r.top, o.row_top)
    np.testing.assert_array_equal(g.union, o.union)
    np.testing.assert_array_equal(g.nodg, O.nodg(X))
    check_selection(r, g.union, K)
    # stage 3 on the same union: every packed entry against the exact SVD
    dist = eng.distance(ds, g.union, nat.SCC_DIST_PCA_EUCLID)
    ref = O.dist_euclidean(O.pca_scores(X, g.union))
    assert dist.shape == ref.shape == (d.N * (d.N - 1) // 2,)
    err = float(np.max(np.abs(dist - ref)))
    assert err < DIST_ATOL, err
    del dist, ref
    # the opt-in Pearson metric (Fast:403): every packed entry against fp64 1 - cor (torch, on the GPU)
    pe = eng.distance(ds, g.union, nat.SCC_DIST_PEARSON)
    Xu = X[g.union]
    Z = Xu - Xu.mean(axis=0, keepdims=True)
    Z /= np.sqrt((Z * Z).sum(axis=0, keepdims=True))
    Zt = torch.from_numpy(np.ascontiguousarray(Z)).to("cuda:0")
    err = TR.packed_max_err(torch.from_numpy(pe).to("cuda:0"), lambda j0, j1: 1.0 - Zt[:, j0:j1].T @ Zt, d.N)
    assert err < DIST_ATOL, err
    ds.close()
    eng.close()


def _de_large(name, n_genes_sample, seed, dist_pairs=0):
    """Config ``name`` generated in HBM as a gene-major CSR (so the device
    CSR -> CSC transpose runs at full size), FAST DE over all pairs in ONE
    engine run, then the subset-oracle and full-size selection checks."""
    from scconsensus_amd import _native as nat
    d = synth.generate_device(name, "cuda:0", layout="csr")
    torch.cuda.synchronize()
    names, code = api.select_clusters(d.labels, 10)
    K = len(names)
    eng = nat.Engine(0)
    ds = eng.dataset_csr_device(d.indptr.data_ptr(), d.indices.data_ptr(), d.data.data_ptr(), d.G, d.N, d.nnz)
    g = eng.de_run(ds, code, K, nat.SCC_DE_FAST, fetch="rows")  # K <= 128: ONE engine run (config E included)
    r = g.rows
    P = K * (K - 1) // 2
    n = np.bincount(code[code >= 0], minlength=K).astype(np.int64)
    pairs = [(i, j) for i in range(K - 1) for j in range(i + 1, K)]
    nn = np.array([n[i] * n[j] for i, j in pairs])
    assert r.pair_tested.shape == (P,)
    assert np.all(r.u2 >= 0) and np.all(r.u2 <= 2 * nn[r.row_pair])
    assert np.all((r.ties >= 0))
    assert 100 < len(g.union) <= 30 * P
    check_selection(r, g.union, K)
    assert check_p_from_counts(r, code, K) == len(r.gene)  # every row's p from its exact counts
    # EVERY tested row's exact 2U and tie term against an independent full-size torch computation
    t0 = time.perf_counter()
    u2_all, ties_all = TR.pair_stats(d.indptr, d.indices, d.data, code, K, max_chunk=min(16 << 20, (512 << 20) // K))
    gi = torch.from_numpy(r.gene.astype(np.int64)).to("cuda:0")
    pi = torch.from_numpy(r.row_pair.astype(np.int64)).to("cuda:0")
    np.testing.assert_array_equal(u2_all[gi, pi].cpu().numpy(), r.u2)
    np.testing.assert_array_equal(ties_all[gi, pi].cpu().numpy(), r.ties)
    print(f"{name}: {len(r.gene)} rows checked against the full-size torch rank sums "
          f"({time.perf_counter() - t0:.1f} s)")
    del u2_all, ties_all, gi, pi
    _free()
    # the oracle on a seeded gene sample: half drawn from the tested rows, half uniform
    rng = np.random.default_rng(seed)
    tg = np.unique(r.gene)
    genes = np.unique(np.concatenate([rng.choice(tg, n_genes_sample // 2, replace=False),
                                      rng.choice(d.G, n_genes_sample - n_genes_sample // 2, replace=False)]))
    ip = d.indptr.cpu().numpy()
    Xs = rows_of_gene_major(ip, d.indices, d.data, genes, d.N)
    ncmp = check_rows_against_oracle_subset(r, Xs, genes, code, K)
    assert ncmp >= 200, ncmp
    out = dict(d=d, eng=eng, ds=ds, g=g, code=code, K=K, ip=ip)
    return out


def test_config_c_parity():
    from scconsensus_amd import _native as nat
    t = _de_large("C", 80, seed=31)
    d, eng, ds, g = t["d"], t["eng"], t["ds"], t["g"]
    assert t["K"] == 30
    # distance at C (5e9 entries, 40 GB fp64 in HBM): sampled entries vs the exact SVD
    N = d.N
    out = torch.empty(N * (N - 1) // 2, dtype=torch.float64, device="cuda:0")
    eng.distance(ds, g.union, nat.SCC_DIST_PCA_EUCLID, device_out_ptr=out.data_ptr())
    eng.synchronize()
    Xu = rows_of_gene_major(t["ip"], d.indices, d.data, g.union, N)
    S = O.pca_scores(Xu, np.arange(len(g.union)))
    # EVERY one of the 5e9 packed entries against the exact-SVD scores (torch, fp64, on the GPU)
    St = torch.from_numpy(np.ascontiguousarray(S)).to("cuda:0")
    err = TR.packed_max_err(out, TR.euclid_block(St), N)
    print(f"C: max |dist - exact SVD| over all {out.numel()} entries {err:.3g}")
    assert err < DIST_ATOL, err
    assert bool(torch.isfinite(out).all()) and float(out.min()) >= 0.0
    del out
    ds.close()
    eng.close()
    del t, d
    _free()


def test_config_e_parity():
    """1M cells, K = 100 (4950 pairs) from a gene-major CSR."""
    t = _de_large("E", 40, seed=51)
    assert t["K"] == 100
    t["ds"].close()
    t["eng"].close()
    del t
    _free()
