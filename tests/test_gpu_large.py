"""Config D shape (200k cells x 20k genes, K = 50, 1225 pairs) end to end on
the device, with the input generated in HBM as a gene-major CSR (so the CSR
transpose runs at full size too).

DE: full-size properties (U within [0, 2 n_a n_b]; the re-split route and the
plain LDS-item route bit-identical), every tested row's exact 2U and tie term
(and under SLOW all 1225 x 20000 2U values) against an independent full-size
torch computation (tests/torch_ranksum.py), the oracle on a seeded gene subset over
all cells and pairs (exact tested sets, U, ties, pct; p / logFC within the
bar), and the full-size per-pair selection restated from the engine's rows.
Distance: the 2e10-entry packed fp64 `dist` (160 GB, HBM-resident), every
entry against the exact SVD of X[U, ] (fp64 torch distances on the GPU)."""
import numpy as np
import pytest
import torch  # before the engine loads (torch's HIP runtime first)

import oracle as O
import torch_ranksum as TR
from parity_helpers import (check_p_from_counts, check_rows_against_oracle_subset, check_selection,
                            check_slow_against_oracle_subset,
                            check_slow_selection, packed_index, rows_of_gene_major, sample_cell_pairs, slow_gate,
                            slow_log_threshold)
from scconsensus_amd import api, synth

pytestmark = pytest.mark.gpu


def _say(*a):  # progress in the GPU log (long tests)
    print("[progress]", *a, flush=True)


def test_config_d_parity(monkeypatch):
    from scconsensus_amd import _native as nat
    d = synth.generate_device("D", "cuda:0", layout="csr")
    torch.cuda.synchronize()
    eng = nat.Engine(0)
    ds = eng.dataset_csr_device(d.indptr.data_ptr(), d.indices.data_ptr(), d.data.data_ptr(), d.G, d.N, d.nnz)
    names, code = api.select_clusters(d.labels, 10)
    K = len(names)
    assert K == 50
    g = eng.de_run(ds, code, K, nat.SCC_DE_FAST, fetch="rows")
    r = g.rows
    pairs = [(i, j) for i in range(K - 1) for j in range(i + 1, K)]
    n = np.bincount(code[code >= 0], minlength=K).astype(np.int64)
    nn = np.array([n[i] * n[j] for i, j in pairs])
    assert np.all(r.u2 >= 0) and np.all(r.u2 <= 2 * nn[r.row_pair])
    assert 100 < len(g.union) <= 30 * len(pairs)
    check_selection(r, g.union, K)
    assert check_p_from_counts(r, code, K) == len(r.gene)  # every row's p from its exact counts
    # EVERY tested row's exact 2U and tie term against the independent full-size torch rank sums
    u2_all, ties_all = TR.pair_stats(d.indptr, d.indices, d.data, code, K, max_chunk=(512 << 20) // K)
    gi = torch.from_numpy(r.gene.astype(np.int64)).to("cuda:0")
    pi = torch.from_numpy(r.row_pair.astype(np.int64)).to("cuda:0")
    np.testing.assert_array_equal(u2_all[gi, pi].cpu().numpy(), r.u2)
    np.testing.assert_array_equal(ties_all[gi, pi].cpu().numpy(), r.ties)
    _say(f"D: {len(r.gene)} rows match the full-size torch rank sums")
    del u2_all, ties_all, gi, pi
    # the same DE with the re-split route off (fat buckets ranked as LDS items)
    # and the gene-level cross terms by the per-(gene, pair) wave kernel
    monkeypatch.setenv("SCC_RESPLIT", "0")
    monkeypatch.setenv("SCC_CROSS_WAVE", "1")
    g0 = eng.de_run(ds, code, K, nat.SCC_DE_FAST, fetch="rows")
    monkeypatch.delenv("SCC_RESPLIT")
    monkeypatch.delenv("SCC_CROSS_WAVE")
    np.testing.assert_array_equal(g0.rows.gene, r.gene)
    np.testing.assert_array_equal(g0.rows.u2, r.u2)
    np.testing.assert_array_equal(g0.rows.ties, r.ties)
    np.testing.assert_array_equal(g0.union, g.union)
    # the oracle on a seeded gene subset (half from the tested rows)
    ip = d.indptr.cpu().numpy()
    rng = np.random.default_rng(4)
    genes = np.unique(np.concatenate([rng.choice(np.unique(r.gene), 30, replace=False),
                                      rng.choice(d.G, 30, replace=False)]))
    Xs = rows_of_gene_major(ip, d.indices, d.data, genes, d.N)
    assert check_rows_against_oracle_subset(r, Xs, genes, code, K) >= 200
    del Xs
    # stage 3: packed fp64 dist of 2e10 entries kept in HBM, sampled vs the exact SVD
    N = d.N
    out = torch.empty(N * (N - 1) // 2, dtype=torch.float64, device="cuda:0")
    eng.distance(ds, g.union, nat.SCC_DIST_PCA_EUCLID, device_out_ptr=out.data_ptr())
    eng.synchronize()
    Xu = rows_of_gene_major(ip, d.indices, d.data, g.union, N)
    S = O.pca_scores(Xu, np.arange(len(g.union)))
    i, j = sample_cell_pairs(N, 200_000, seed=6)
    got = out[torch.from_numpy(packed_index(i, j, N)).to("cuda:0")].cpu().numpy()
    want = np.sqrt(((S[i] - S[j]) ** 2).sum(axis=1))
    err = float(np.max(np.abs(got - want)))
    assert err < 1e-5, err
    # EVERY one of the 2e10 packed entries against the exact-SVD scores (torch, fp64, on the GPU)
    St = torch.from_numpy(np.ascontiguousarray(S)).to("cuda:0")
    err = TR.packed_max_err(out, TR.euclid_block(St),
                            N, cols=512)
    _say(f"D: max |dist - exact SVD| over all {out.numel()} entries {err:.3g}")
    assert err < 1e-5, err
    # the last column block (the packed vector's tail) in full
    tail = out[-(200 * 199 // 2):].cpu().numpy()
    ii, jj = np.tril_indices(200, -1)
    ref_tail = np.sqrt(((S[N - 200 + ii] - S[N - 200 + jj]) ** 2).sum(axis=1))
    order = np.argsort(packed_index(N - 200 + ii, N - 200 + jj, N))
    assert np.max(np.abs(tail - ref_tail[order])) < 1e-5
    assert float(out.min()) >= 0.0
    del out
    ds.close()
    eng.close()


def test_config_d_slow():
    """reclusterDEConsensus (SLOW: every gene x every pair, slow:69-227) at
    config D: the oracle on 60 genes over all 200k cells and 1225 pairs (exact
    U, p / logFC within the bar), the global threshold restated from all 463 M
    stored values, and the full-size selection from the engine's [1225][20000]
    vectors: BH with n = G, DE flags (the gate restated on the subset genes),
    the first-30 union."""
    from scconsensus_amd import _native as nat
    d = synth.generate_device("D", "cuda:0", layout="csr")
    torch.cuda.synchronize()
    eng = nat.Engine(0)
    ds = eng.dataset_csr_device(d.indptr.data_ptr(), d.indices.data_ptr(), d.data.data_ptr(), d.G, d.N, d.nnz)
    names, code = api.select_clusters(d.labels, 10)
    K, qthr, fc, msf = len(names), 0.05, 1.5, 5.0
    assert K == 50
    g = eng.de_run(ds, code, K, nat.SCC_DE_SLOW, q_val_thrs=qthr, fc_thrs=fc, mean_scaling_factor=msf, fetch="all")
    assert g.p.shape == (1225, d.G)
    _say("SLOW D engine done")
    # ALL 1225 x 20000 exact 2U values against the independent full-size torch rank sums
    u2_all, _ = TR.pair_stats(d.indptr, d.indices, d.data, code, K, max_chunk=(512 << 20) // K)
    np.testing.assert_array_equal(u2_all.T.cpu().numpy(), g.u2)
    del u2_all
    _say("SLOW D: all 24.5 M (pair, gene) 2U values match the torch rank sums")
    assert g.log_thr == pytest.approx(slow_log_threshold(d.data.cpu().numpy(), d.G, d.N, msf), rel=1e-13)
    ip = d.indptr.cpu().numpy()
    rng = np.random.default_rng(12)
    genes = np.sort(rng.choice(d.G, 60, replace=False))
    Xs = rows_of_gene_major(ip, d.indices, d.data, genes, d.N)
    _say("SLOW D threshold / rows done")
    assert check_slow_against_oracle_subset(g, Xs, genes, code, K, qthr, fc, msf) == 1225 * 60
    _say("SLOW D subset oracle done")
    check_slow_selection(g, qthr, fc, gate=slow_gate(Xs, code, K, g.log_thr), gate_genes=genes)
    assert len(g.union) > 30
    ds.close()
    eng.close()
