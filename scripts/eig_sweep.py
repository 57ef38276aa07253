"""Sweep the eigensolver's workgroup count on the config-B union (timing only)."""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from scconsensus_amd import _native as nat  # noqa: E402
from scconsensus_amd import api, synth  # noqa: E402

cfg = sys.argv[1] if len(sys.argv) > 1 else "B"
d = synth.generate(cfg)
names, code = api.select_clusters(d.labels, 10)
eng = nat.Engine(0, profile=True)
ds = eng.dataset_csc(d.indptr, d.indices, d.data, d.G, d.N)
r = eng.de_run(ds, code, len(names), nat.SCC_DE_FAST, fetch="union")
print(f"union {len(r.union)}", flush=True)
ref = None
for nwg in [int(x) for x in (sys.argv[2].split(",") if len(sys.argv) > 2 else ["8", "16", "24", "33", "48", "64", "128"])]:
    os.environ["SCC_EIG_NWG"] = str(nwg)
    eng.distance(ds, r.union, nat.SCC_DIST_PCA_EUCLID, device_out_ptr=0)
    eng.synchronize()
    eng.reset_timers()
    for _ in range(3):
        eng.distance(ds, r.union, nat.SCC_DIST_PCA_EUCLID, device_out_ptr=0)
    eng.synchronize()
    t = {f: eng.kernel_time(f) for f in ["eig_tridiag", "eig_vec", "eig_fin", "eigen", "gram", "dist"]}
    S = eng.last_pca_scores(d.N)
    if ref is None:
        ref = S
    dev = float(np.max(np.abs(np.abs(S) - np.abs(ref))))
    print(f"nwg {nwg}: " + " ".join(f"{k} {v[0] / max(v[1], 1):.3f}" for k, v in t.items()) + f"  |S| dev {dev:.2e}",
          flush=True)
