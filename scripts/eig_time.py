"""Eigen-stage timing on synthetic Grams of size n (two-stage vs one-stage),
with the distance checked against the exact SVD.  Usage:
    python scripts/eig_time.py 323,562,845 [reps]"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "oracle"))
import torch  # noqa: E402,F401

import oracle as O  # noqa: E402
from scconsensus_amd import _native as nat  # noqa: E402

sizes = [int(x) for x in (sys.argv[1] if len(sys.argv) > 1 else "323,562,845").split(",")]
reps = int(sys.argv[2]) if len(sys.argv) > 2 else 5
eng = nat.Engine(0, profile=True)
for n in sizes:
    rng = np.random.default_rng(n)
    N = 2000
    X = rng.standard_normal((n, N)) * np.linspace(3.0, 0.5, n)[:, None]
    X[:12] += rng.standard_normal((12, 1)) * rng.standard_normal((1, N)) * 4.0
    ds = eng.dataset_dense(X)
    g = np.arange(n)
    ref = O.dist_euclidean(O.pca_scores(X, g))
    for sbr in ["1", "0"]:
        os.environ["SCC_EIG_SBR"] = sbr
        dist = eng.distance(ds, g, nat.SCC_DIST_PCA_EUCLID)
        err = float(np.max(np.abs(dist - ref)))
        eng.synchronize()
        eng.reset_timers()
        for _ in range(reps):
            eng.distance(ds, g, nat.SCC_DIST_PCA_EUCLID, device_out_ptr=0)
        eng.synchronize()
        t = {f: eng.kernel_time(f) for f in ["eigen", "eig_tridiag", "eig_vec", "eig_fin"]}
        print(f"n {n} sbr {sbr}: " + " ".join(f"{k} {v[0] / max(v[1], 1):.3f}" for k, v in t.items())
              + f"  dist err {err:.2e}", flush=True)
    ds.close()
