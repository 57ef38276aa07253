"""The device list behind the C ABI (scc_opts.n_devices / devices, include/scc.h):
ONE job driven over several engines from one host process -- here [0, 0] and
[0, 0, 0], engines on the box's one GPU exchanging by device copies, the same
code path as peers over xGMI -- must give the one-device result bit for bit:
the gene-block DE with its record gather (FAST rows, t test, SLOW vectors,
K > 128 group-pair runs), the column-sliced distance to host and device
buffers, and the silhouette on the engine-kept distance whose slices live on
the other engines (reference Fast:61-65,384: the nCores pool
this replaces)."""
import numpy as np
import pytest
import torch  # before the engine loads (torch's HIP runtime first)

from scconsensus_amd import _native as nat
from scconsensus_amd import api, synth

pytestmark = pytest.mark.gpu

FAST_FIELDS = ("pair_tested", "gene", "p", "q", "avg_logfc", "pct1", "pct2", "u2", "ties", "de", "top")


@pytest.fixture(scope="module")
def engines():
    es = [nat.Engine(0), nat.Engine(0, devices=[0, 0]), nat.Engine(0, devices=[0, 0, 0])]
    yield es
    for e in es:
        e.close()


@pytest.fixture(scope="module")
def cfg_a():
    d = synth.generate("A")
    names, code = api.select_clusters(d.labels, 10)
    return d, names, code


def _datasets(engines, d):
    return [e.dataset_csc(d.indptr, d.indices, d.data, d.G, d.N) for e in engines]


@pytest.mark.parametrize("test", ["wilcox", "t"])
def test_fast_bitwise(engines, cfg_a, test):
    d, names, code = cfg_a
    K = len(names)
    dss = _datasets(engines, d)
    res = [e.de_run(ds, code, K, nat.SCC_DE_FAST, fetch="rows", test=test) for e, ds in zip(engines, dss)]
    for r in res[1:]:
        np.testing.assert_array_equal(r.union, res[0].union)
        np.testing.assert_array_equal(r.nodg, res[0].nodg)
        for f in FAST_FIELDS:
            np.testing.assert_array_equal(getattr(r.rows, f), getattr(res[0].rows, f), err_msg=f)
    # a second run on the same datasets (validated: gene blocks read only their tiles)
    again = engines[2].de_run(dss[2], code, K, nat.SCC_DE_FAST, fetch="rows", test=test)
    np.testing.assert_array_equal(again.rows.p, res[0].rows.p)


def test_slow_bitwise(engines, cfg_a):
    d, names, code = cfg_a
    sub = synth.from_dense(d.dense()[:500], d.labels)
    kw = dict(q_val_thrs=0.05, fc_thrs=1.5, mean_scaling_factor=5.0)
    res = [e.de_run(ds, code, len(names), nat.SCC_DE_SLOW, fetch="all", **kw)
           for e, ds in zip(engines, _datasets(engines, sub))]
    for r in res[1:]:
        assert r.log_thr == res[0].log_thr
        for f in ("union", "p", "q", "logfc", "u2", "de"):
            np.testing.assert_array_equal(getattr(r, f), getattr(res[0], f), err_msg=f)


def test_grouped_over_devices(engines):
    """K = 150: every group-pair run is itself sharded over the devices."""
    d = synth.generate("A", G=60, N=12000, K=150, seed=31)
    names, code = api.select_clusters(d.labels, 10)
    kw = dict(min_per_cent=5.0, log_fc_thrs=0.2)
    a = engines[0].de_run(_datasets(engines[:1], d)[0], code, 150, nat.SCC_DE_FAST, fetch="rows", **kw)
    b = engines[1].de_run(_datasets(engines[1:2], d)[0], code, 150, nat.SCC_DE_FAST, fetch="rows", **kw)
    np.testing.assert_array_equal(b.union, a.union)
    for f in FAST_FIELDS:
        np.testing.assert_array_equal(getattr(b.rows, f), getattr(a.rows, f), err_msg=f)


def test_distance_slices_bitwise(engines, cfg_a):
    d, names, code = cfg_a
    dss = _datasets(engines, d)
    uni = engines[0].de_run(dss[0], code, len(names), nat.SCC_DE_FAST, fetch="union").union
    N = d.N
    ref = engines[0].distance(dss[0], uni)
    lab = np.arange(N, dtype=np.int32) % 7
    w_ref, avg_ref = engines[0].silhouette(N, lab)
    for e, ds in zip(engines[1:], dss[1:]):
        host = e.distance(ds, uni)
        np.testing.assert_array_equal(host, ref)
        w, avg = e.silhouette(N, lab)  # the kept copy: peer slices gathered on first use
        np.testing.assert_array_equal(w, w_ref)
        np.testing.assert_array_equal(avg, avg_ref)
        dev = torch.empty(N * (N - 1) // 2, dtype=torch.float64, device="cuda:0")
        e.distance(ds, uni, device_out_ptr=dev.data_ptr())
        e.synchronize()
        np.testing.assert_array_equal(dev.cpu().numpy(), ref)
        lo, hi = 100, 2000  # a column slice
        part = e.distance_cols(ds, uni, lo, hi)
        a0 = lo * (2 * N - lo - 1) // 2
        np.testing.assert_array_equal(part, ref[a0: a0 + len(part)])
        f32 = e.distance(ds, uni, f32=True)
        np.testing.assert_array_equal(f32, engines[0].distance(dss[0], uni, f32=True))


def test_pearson_slices_bitwise(engines, cfg_a):
    """1 - r (Fast:403) over the device list: each device writes its column
    slice from its own copy of the z-scores with the one-device kernel, so the
    output is bit-identical to one device (host, device and f32 outputs, and a
    column slice)."""
    d, names, code = cfg_a
    dss = _datasets(engines, d)
    uni = engines[0].de_run(dss[0], code, len(names), nat.SCC_DE_FAST, fetch="union").union
    N = d.N
    ref = engines[0].distance(dss[0], uni, nat.SCC_DIST_PEARSON)
    ref32 = engines[0].distance(dss[0], uni, nat.SCC_DIST_PEARSON, f32=True)
    for e, ds in zip(engines[1:], dss[1:]):
        np.testing.assert_array_equal(e.distance(ds, uni, nat.SCC_DIST_PEARSON), ref)
        np.testing.assert_array_equal(e.distance(ds, uni, nat.SCC_DIST_PEARSON, f32=True), ref32)
        dev = torch.empty(N * (N - 1) // 2, dtype=torch.float64, device="cuda:0")
        e.distance(ds, uni, nat.SCC_DIST_PEARSON, device_out_ptr=dev.data_ptr())
        e.synchronize()
        np.testing.assert_array_equal(dev.cpu().numpy(), ref)
        lo, hi = 300, 1700
        part = e.distance_cols(ds, uni, lo, hi, metric=nat.SCC_DIST_PEARSON)
        a0 = lo * (2 * N - lo - 1) // 2
        np.testing.assert_array_equal(part, ref[a0: a0 + len(part)])
