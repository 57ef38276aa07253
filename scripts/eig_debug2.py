"""Eigensolver: sizes x workgroup counts against numpy (LDS vs global row store)."""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "oracle"))
import oracle as O  # noqa: E402
from scconsensus_amd import _native as nat  # noqa: E402

eng = nat.Engine(0)
for n, N, nwgs in [(700, 900, [70, 256]), (1500, 1200, [150, 40]), (2100, 1200, [210, 256, 100])]:
    rng = np.random.default_rng(11)
    X = rng.standard_normal((n, N)) * np.linspace(3.0, 0.5, n)[:, None]
    X[:20] += rng.standard_normal((20, 1)) * rng.standard_normal((1, N)) * 4.0
    ds = eng.dataset_dense(X)
    g = np.arange(n)
    ref = O.dist_euclidean(O.pca_scores(X, g))
    for nwg in nwgs:
        os.environ["SCC_EIG_NWG"] = str(nwg)
        d = eng.distance(ds, g, nat.SCC_DIST_PCA_EUCLID)
        print(n, nwg, "max err", float(np.max(np.abs(d - ref))), flush=True)
