"""Eigensolver debug: tiny PCA cases against numpy (prints GPU W/Z via SCC_EIG_DUMP)."""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "oracle"))
os.environ["SCC_EIG_DUMP"] = "1"
import oracle as O  # noqa: E402
from scconsensus_amd import _native as nat  # noqa: E402

eng = nat.Engine(0)
X = np.array([[0.0, 1.0, 3.0, 6.0], [0.0, 0.0, 0.0, 0.0], [1.0, 1.0, 1.0, 1.0]])
ds = eng.dataset_dense(X)
print("tiny", eng.distance(ds, np.array([0, 2]), nat.SCC_DIST_PCA_EUCLID), flush=True)
rng = np.random.default_rng(0)
for n in [2, 3, 4, 5, 8, 17, 40]:
    X = rng.standard_normal((n, 30))
    ds = eng.dataset_dense(X)
    g = np.arange(n)
    d = eng.distance(ds, g, nat.SCC_DIST_PCA_EUCLID)
    ref = O.dist_euclidean(O.pca_scores(X, g))
    print(n, "max err", float(np.max(np.abs(d - ref))), flush=True)
