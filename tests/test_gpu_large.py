"""Config D shape (200k cells x 20k genes, K = 50, 1225 pairs) end to end on
the device, with the input generated in HBM as a gene-major CSR (so the CSR
transpose runs at full size too).  Parity at full size through properties
(U within [0, 2 n_a n_b], the re-split route and the plain LDS-item route
giving bit-identical rows) and exactly against the oracle on a seeded sample
of tested (pair, gene) rows."""
import numpy as np
import pytest
import torch  # before the engine loads (torch's HIP runtime first)

import oracle as O
from scconsensus_amd import api, synth

pytestmark = pytest.mark.gpu


def test_config_d_rows_sampled_parity(monkeypatch):
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
    # exact U / ties / p on sampled tested rows against the oracle
    ip = d.indptr.cpu().numpy()
    rng = np.random.default_rng(4)
    for k in rng.choice(len(r.gene), 40, replace=False):
        gene, p = int(r.gene[k]), int(r.row_pair[k])
        i, j = pairs[p]
        row = np.zeros(d.N)
        row[d.indices[ip[gene]:ip[gene + 1]].cpu().numpy()] = d.data[ip[gene]:ip[gene + 1]].cpu().numpy()
        po, W, T, _ = O.wilcox_test(row[code == i], row[code == j])
        assert r.u2[k] == int(round(2 * W))
        assert r.ties[k] == int(round(T))
        assert r.p[k] == pytest.approx(po, rel=1e-6)
    ds.close()
