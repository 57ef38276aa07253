"""GPU diagnostics of the eigensolver paths (dev script): the test matrices of
tests/test_gpu_fsi.py through each path with SCC_EIG_SI_LOG, and the
hidden-eigenvalue guard case of tests/test_gpu_dist.py under a time limit per
variant (each in its own process).

    python scripts/fsi_diag.py eig      # path / flag per matrix and engine setting
    python scripts/fsi_diag.py guard    # the n=500 guard case per env variant
"""
import ctypes
import os
import subprocess
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))


def b_like(n, rng):
    top = np.array([15.14, 10.09, 8.97, 7.95, 6.82, 6.22, 3.59, 2.21, 1.655, 1.469, 1.055, 1.021, 1.009, 1.0045, 1.0])
    bulk = np.sort(rng.uniform(0.184, 0.996, n - 15))[::-1]
    bulk[0] = 0.996
    bulk[49] = 0.877
    return np.concatenate([top, np.sort(bulk)[::-1]]) * 4.1e4


def eig():
    import torch
    from scconsensus_amd import _native as nat
    L = nat.load()
    L.scc_diag_eigen_topk.restype = ctypes.c_int
    os.environ["SCC_EIG_FSI"] = "1"
    os.environ["SCC_EIG_SI_LOG"] = "1"
    for n, seed in ((323, 5), (323, 323), (130, 130), (500, 500)):
        rng = np.random.default_rng(seed)
        lam = b_like(n, rng)
        V, _ = np.linalg.qr(np.random.default_rng(11 if seed == n else 9).standard_normal((n, n)))
        C = (V * lam) @ V.T
        Cd = torch.tensor(C, dtype=torch.float64, device="cuda:0")
        res = {}
        for e in ("1", "0"):
            os.environ["SCC_EIG_FSI_ENGINE"] = e
            Z = torch.zeros(n * 16, dtype=torch.float64, device="cuda:0")
            W = torch.zeros(16, dtype=torch.float64, device="cuda:0")
            path = ctypes.c_int(-1)
            t0 = time.time()
            rc = L.scc_diag_eigen_topk(ctypes.c_void_p(Cd.data_ptr()), n, n, 15, ctypes.c_void_p(Z.data_ptr()),
                                       ctypes.c_void_p(W.data_ptr()), ctypes.byref(path))
            res[e] = (Z.cpu().numpy(), W.cpu().numpy())
            print(f"n={n} seed={seed} engine={e} rc={rc} path={path.value} {1e3 * (time.time() - t0):.1f} ms", flush=True)
        dz = np.max(np.abs(res["1"][0] - res["0"][0]))
        dw = np.max(np.abs(res["1"][1] - res["0"][1]))
        print(f"   max |dZ| {dz:.3g}  max |dW| {dw:.3g}", flush=True)


def guard_case(variant):
    from scconsensus_amd import _native as nat
    from test_gpu_dist import _spiky
    for kv in variant.split(","):
        if kv:
            k, v = kv.split("=")
            os.environ[k] = v
    os.environ["SCC_EIG_SI_LOG"] = "1"
    rng = np.random.default_rng(12)
    n, N = 500, 3000
    X = np.zeros((n, N))
    X[:400, :1500] = _spiky(400, 1500, 30, 5)
    X[400:, 1500:] = rng.standard_normal((100, 1500)) * 0.3
    X[400:, 1500:] += rng.standard_normal((100, 1)) * rng.standard_normal((1, 1500)) * 40.0
    X[:400, :1500] -= X[:400, :1500].mean(axis=1, keepdims=True)
    X[400:, 1500:] -= X[400:, 1500:].mean(axis=1, keepdims=True)
    eng = nat.Engine()
    ds = eng.dataset_dense(X)
    t0 = time.time()
    d = eng.distance(ds, np.arange(n), nat.SCC_DIST_PCA_EUCLID)
    print(f"variant {variant!r}: {time.time() - t0:.2f} s, dist[0:3] {d[:3]}", flush=True)


def guard():
    variants = ["SCC_EIG_SI=0", "SCC_GRAM_T=64,SCC_EIG_SI=0", "SCC_GRAM_T=64", "",
                "SCC_EIG_SI_INIT_ROWS=400,SCC_GRAM_T=64", "SCC_EIG_SI_INIT_ROWS=400"]
    for v in variants:
        t0 = time.time()
        try:
            r = subprocess.run([sys.executable, __file__, "guard1", v], timeout=60, capture_output=True, text=True)
            print(r.stdout.strip(), "|", r.stderr.strip()[-400:], f"(rc {r.returncode}, {time.time() - t0:.1f} s)",
                  flush=True)
        except subprocess.TimeoutExpired:
            print(f"variant {v!r}: TIMEOUT after 60 s", flush=True)
            break  # a hung GPU step: stop here


def stamps():
    import torch
    from scconsensus_amd import _native as nat
    L = nat.load()
    os.environ["SCC_EIG_FSI"] = "1"
    os.environ["SCC_EIG_FSI_STAMPS"] = "1"
    n = 323
    rng = np.random.default_rng(5)
    lam = b_like(n, rng)
    V, _ = np.linalg.qr(np.random.default_rng(9).standard_normal((n, n)))
    Cd = torch.tensor((V * lam) @ V.T, dtype=torch.float64, device="cuda:0")
    Z = torch.zeros(n * 16, dtype=torch.float64, device="cuda:0")
    W = torch.zeros(16, dtype=torch.float64, device="cuda:0")
    path = ctypes.c_int(-1)
    for it in range(3):
        if it == 2:
            os.environ["SCC_EIG_SI_LOG"] = "1"
        L.scc_diag_eigen_topk(ctypes.c_void_p(Cd.data_ptr()), n, n, 15, ctypes.c_void_p(Z.data_ptr()),
                              ctypes.c_void_p(W.data_ptr()), ctypes.byref(path))
    print("path", path.value, flush=True)


def repeat():
    """the bitwise-test sequence many times: path and flag per call"""
    import torch
    from scconsensus_amd import _native as nat
    L = nat.load()
    os.environ["SCC_EIG_FSI"] = "1"
    os.environ["SCC_EIG_SI_LOG"] = "1"
    mats = []
    for n, seed, vs in ((323, 5, 9), (323, 323, 11)):
        lam = b_like(n, np.random.default_rng(seed))
        V, _ = np.linalg.qr(np.random.default_rng(vs).standard_normal((n, n)))
        mats.append((V * lam) @ V.T)
    for it in range(12):
        for mi, C in enumerate(mats):
            for e in ("1", "0"):
                os.environ["SCC_EIG_FSI_ENGINE"] = e
                n = C.shape[0]
                Cd = torch.tensor(C, dtype=torch.float64, device="cuda:0")
                Z = torch.zeros(n * 16, dtype=torch.float64, device="cuda:0")
                W = torch.zeros(16, dtype=torch.float64, device="cuda:0")
                path = ctypes.c_int(-1)
                L.scc_diag_eigen_topk(ctypes.c_void_p(Cd.data_ptr()), n, n, 15, ctypes.c_void_p(Z.data_ptr()),
                                      ctypes.c_void_p(W.data_ptr()), ctypes.byref(path))
                print(f"it={it} mat={mi} engine={e} path={path.value}", flush=True)


if __name__ == "__main__":
    what = sys.argv[1]
    if what == "repeat":
        repeat()
    elif what == "stamps":
        stamps()
    elif what == "eig":
        eig()
    elif what == "guard":
        guard()
    elif what == "guard1":
        guard_case(sys.argv[2])
