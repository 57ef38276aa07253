"""Distance-kernel tile-shape sweep at config B (SCC_DIST_TILE variants of
scc_launch_dist_euclid), HBM-resident output; prints ms and TB/s."""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import torch  # noqa: E402

from scconsensus_amd import _native as nat  # noqa: E402
from scconsensus_amd import api, synth  # noqa: E402

d = synth.generate(sys.argv[1] if len(sys.argv) > 1 else "B")
names, code = api.select_clusters(d.labels, 10)
eng = nat.Engine(0, profile=True)
ds = eng.dataset_csc(d.indptr, d.indices, d.data, d.G, d.N)
r = eng.de_run(ds, code, len(names), nat.SCC_DE_FAST, fetch="union")
out = torch.empty(d.N * (d.N - 1) // 2, dtype=torch.float64, device="cuda:0")
ref = None
for v in (sys.argv[2].split(",") if len(sys.argv) > 2 else ["0", "1", "2", "3", "4", "5"]):
    os.environ["SCC_DIST_TILE"] = v
    eng.distance(ds, r.union, nat.SCC_DIST_PCA_EUCLID, device_out_ptr=out.data_ptr())
    eng.synchronize()
    if ref is None:
        ref = out[::9973].clone()
    else:
        assert torch.equal(ref, out[::9973])
    eng.reset_timers()
    for _ in range(5):
        eng.distance(ds, r.union, nat.SCC_DIST_PCA_EUCLID, device_out_ptr=out.data_ptr())
    eng.synchronize()
    t, c = eng.kernel_time("dist")
    ms = t / max(c, 1)
    print(f"tile {v}: dist {ms:.3f} ms  {out.numel() * 8 / ms / 1e9:.2f} TB/s", flush=True)
