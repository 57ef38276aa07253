"""Phase stamps of the register-tail tridiagonalisation (SCC_STAMPS=1) at a
few sizes.  Usage: SCC_STAMPS=1 python scripts/eig_tail_stamps.py 64,256"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import torch  # noqa: E402,F401

from scconsensus_amd import _native as nat  # noqa: E402

os.environ["SCC_EIG_SI"] = "0"
eng = nat.Engine(0)
for n in [int(x) for x in (sys.argv[1] if len(sys.argv) > 1 else "64,256").split(",")]:
    X = np.random.default_rng(n).standard_normal((n, 1500))
    ds = eng.dataset_dense(X)
    for _ in range(2):
        eng.distance(ds, np.arange(n), nat.SCC_DIST_PCA_EUCLID, device_out_ptr=0)
    eng.synchronize()
    print(f"n {n} done", flush=True)
    ds.close()
