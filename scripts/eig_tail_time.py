"""Tridiagonalisation time with the one-workgroup register tail (default) vs
the hand-off kernel for every column (SCC_EIG_TAIL=0), on synthetic Grams of
size n, plus the eigenvalue error against numpy.
Usage: python scripts/eig_tail_time.py 100,256,323 [reps]"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "oracle")]
import torch  # noqa: E402,F401

from scconsensus_amd import _native as nat  # noqa: E402

sizes = [int(x) for x in (sys.argv[1] if len(sys.argv) > 1 else "100,200,256,323").split(",")]
reps = int(sys.argv[2]) if len(sys.argv) > 2 else 5
eng = nat.Engine(0, profile=True)
os.environ["SCC_EIG_SI"] = "0"
for n in sizes:
    rng = np.random.default_rng(n)
    N = 2000
    X = rng.standard_normal((n, N)) * np.linspace(3.0, 0.5, n)[:, None]
    ds = eng.dataset_dense(X)
    g = np.arange(n)
    Xc = X - X.mean(axis=1, keepdims=True)
    lam = np.linalg.eigvalsh(Xc @ Xc.T)[::-1][:15]
    out = []
    for tail in ["1", "0"]:
        os.environ["SCC_EIG_TAIL"] = tail
        eng.distance(ds, g, nat.SCC_DIST_PCA_EUCLID, device_out_ptr=0)
        eng.synchronize()
        eng.reset_timers()
        for _ in range(reps):
            eng.distance(ds, g, nat.SCC_DIST_PCA_EUCLID, device_out_ptr=0)
        eng.synchronize()
        tt = eng.kernel_time("eig_tridiag")
        te = eng.kernel_time("eigen")
        ev = (eng.last_pca_scores(N) ** 2).sum(axis=0)[:15]
        out.append((tt[0] / max(tt[1], 1), te[0] / max(te[1], 1), float(np.max(np.abs(ev - lam) / lam))))
    print(f"n {n}: tail tridiag {out[0][0]:.3f} ms eigen {out[0][1]:.3f} ms relerr {out[0][2]:.1e} | "
          f"hand-off tridiag {out[1][0]:.3f} ms eigen {out[1][1]:.3f} ms relerr {out[1][2]:.1e}", flush=True)
    ds.close()
