"""Host logic of the > 64-cluster FAST path (scconsensus_amd/grouped.py):
group-pair runs reassembled in (i, j) order must equal one run over all K.
The device is mocked by the oracle here (CPU); tests/test_gpu_grouped.py runs
the same orchestration on the GPU engine."""
import numpy as np
import pytest

import oracle as O
from scconsensus_amd import _native as nat
from scconsensus_amd import api, grouped, synth


class OracleEngine:
    """de_run with the engine's FAST rows contract, computed by the oracle."""

    def __init__(self, X):
        self.X = X

    def de_run(self, ds, code, K, mode, fetch="rows", **kw):
        assert mode == nat.SCC_DE_FAST and fetch == "rows"
        o = O.de_fast(self.X, code, K, **kw)
        n = len(o.row_gene)
        rows = nat.FastRows(pair_tested=o.pair_tested, row_pair=np.zeros(n, np.int32), gene=o.row_gene,
                            p=o.row_p, q=o.row_q, avg_logfc=o.row_lfc, pct1=o.row_pct1, pct2=o.row_pct2,
                            u2=np.round(2 * o.row_W).astype(np.int64), ties=o.row_ties, de=o.row_de, top=o.row_top)
        return nat.DeResult(mode=mode, K=K, n_pairs=K * (K - 1) // 2, union=o.union, nodg=np.zeros(3), rows=rows)


@pytest.mark.parametrize("K,group", [(9, 4), (10, 3), (7, 7)])
def test_grouped_equals_single_run(K, group):
    d = synth.generate("A", G=150, N=900, K=K, seed=13)
    names, code = api.select_clusters(d.labels, 10)
    X = d.dense()
    eng = OracleEngine(X)
    kw = dict(min_per_cent=5.0, log_fc_thrs=0.1)
    g = grouped.de_fast_grouped(eng, None, code, len(names), group=group, min_k=0, **kw)
    o = O.de_fast(X, code, len(names), **kw)
    np.testing.assert_array_equal(g.rows.pair_tested, o.pair_tested)
    np.testing.assert_array_equal(g.rows.gene, o.row_gene)
    np.testing.assert_array_equal(g.rows.p, o.row_p)
    np.testing.assert_array_equal(g.rows.q, o.row_q)
    np.testing.assert_array_equal(g.rows.top, o.row_top)
    np.testing.assert_array_equal(g.union, o.union)
