"""Eigen-stage time (whole stage: subspace attempt + any fallback) with the
subspace iteration on (default) and off, on a many-cluster spectrum and on a
smooth one.  Usage: python scripts/eig_si_time.py 450,845 [reps]"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import torch  # noqa: E402,F401

from scconsensus_amd import _native as nat  # noqa: E402

sizes = [int(x) for x in (sys.argv[1] if len(sys.argv) > 1 else "450,845").split(",")]
reps = int(sys.argv[2]) if len(sys.argv) > 2 else 3
eng = nat.Engine(0, profile=True)
for n in sizes:
    for kind in ["spiky", "smooth"]:
        rng = np.random.default_rng(n)
        N = 3000
        if kind == "spiky":
            X = rng.standard_normal((n, N)) * 0.5
            lab = rng.integers(0, 40, N)
            X += (rng.standard_normal((n, 40)) * np.linspace(4.0, 1.5, 40)[None, :])[:, lab]
        else:
            X = rng.standard_normal((n, N)) * np.linspace(3.0, 0.5, n)[:, None]
        ds = eng.dataset_dense(X)
        g = np.arange(n)
        out = []
        for si in ["1", "0"]:
            os.environ["SCC_EIG_SI"] = si
            eng.distance(ds, g, nat.SCC_DIST_PCA_EUCLID, device_out_ptr=0)
            eng.synchronize()
            eng.reset_timers()
            for _ in range(reps):
                eng.distance(ds, g, nat.SCC_DIST_PCA_EUCLID, device_out_ptr=0)
            eng.synchronize()
            v = eng.kernel_time("eigen")
            out.append(v[0] / max(v[1], 1))
        print(f"n {n} {kind}: eigen with subspace attempt {out[0]:.3f} ms, direct only {out[1]:.3f} ms", flush=True)
        ds.close()
