"""> 64 clusters on the GPU (BASELINE config E has K = 100): the grouped
orchestration over the engine, checked against one oracle run over all K."""
import numpy as np
import pytest

import oracle as O
from scconsensus_amd import api, grouped, synth

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def eng():
    from scconsensus_amd import _native
    return _native.Engine(0)


def test_fast_70_clusters_matches_oracle(eng):
    from scconsensus_amd import _native as nat
    d = synth.generate("A", G=160, N=5000, K=70, seed=17)
    names, code = api.select_clusters(d.labels, 10)
    K = len(names)
    assert K == 70
    ds = eng.dataset_csc(d.indptr, d.indices, d.data, d.G, d.N)
    with pytest.raises(nat.SccError) as e:  # one engine run holds <= 64 clusters
        eng.de_run(ds, code, K, nat.SCC_DE_FAST, fetch="rows")
    assert e.value.code == nat.SCC_ERR_UNSUPPORTED
    g = grouped.de_fast_grouped(eng, ds, code, K)
    o = O.de_fast(d.dense(), code, K)
    np.testing.assert_array_equal(g.rows.pair_tested, o.pair_tested)
    np.testing.assert_array_equal(g.rows.gene, o.row_gene)
    np.testing.assert_array_equal(g.rows.u2, np.round(2 * o.row_W).astype(np.int64))
    np.testing.assert_array_equal(g.rows.ties, np.round(o.row_ties).astype(np.int64))
    np.testing.assert_allclose(g.rows.p, o.row_p, rtol=1e-6, atol=0)
    np.testing.assert_allclose(g.rows.q, o.row_q, rtol=1e-6, atol=0)
    np.testing.assert_array_equal(g.rows.top, o.row_top)
    np.testing.assert_array_equal(g.union, o.union)
