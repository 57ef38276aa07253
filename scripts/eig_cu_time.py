"""Tridiagonalisation time, one-CU kernel (SCC_EIG_CU=1) vs the multi-workgroup
kernel, on synthetic Grams of size n.  Usage: python scripts/eig_cu_time.py 100,180,323 [reps]"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import torch  # noqa: E402,F401

from scconsensus_amd import _native as nat  # noqa: E402

sizes = [int(x) for x in (sys.argv[1] if len(sys.argv) > 1 else "100,180,250,323").split(",")]
reps = int(sys.argv[2]) if len(sys.argv) > 2 else 5
eng = nat.Engine(0, profile=True)
os.environ["SCC_EIG_SBR"] = "0"
for n in sizes:
    rng = np.random.default_rng(n)
    N = 2000
    X = rng.standard_normal((n, N)) * np.linspace(3.0, 0.5, n)[:, None]
    ds = eng.dataset_dense(X)
    g = np.arange(n)
    out = []
    for cu in ["1", "0"]:
        os.environ["SCC_EIG_CU"] = cu
        eng.distance(ds, g, nat.SCC_DIST_PCA_EUCLID, device_out_ptr=0)
        eng.synchronize()
        eng.reset_timers()
        for _ in range(reps):
            eng.distance(ds, g, nat.SCC_DIST_PCA_EUCLID, device_out_ptr=0)
        eng.synchronize()
        v = eng.kernel_time("eig_tridiag")
        out.append(v[0] / max(v[1], 1))
    print(f"n {n}: one-CU {out[0]:.3f} ms ({1e3 * out[0] / max(n - 1, 1):.2f} us/col)  multi-WG {out[1]:.3f} ms", flush=True)
    ds.close()
