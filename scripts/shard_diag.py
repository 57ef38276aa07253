"""dev: single-GPU distance vs the world-1 sharded route at config A, per eigen path"""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from scconsensus_amd import _native as nat  # noqa: E402
from scconsensus_amd import api, parallel, sharded, synth  # noqa: E402

d = synth.generate("A")
names, code = api.select_clusters(d.labels, 10)
for fsi in ("1", "0"):
    os.environ["SCC_EIG_FSI"] = fsi
    eng = nat.Engine(0)
    ds = eng.dataset_csc(d.indptr, d.indices, d.data, d.G, d.N)
    union = eng.de_run(ds, code, len(names), nat.SCC_DE_FAST, fetch="union").union
    full = sharded.pca_sharded(eng, ds, union, parallel.Dist(), torch.device("cuda:0")).cpu().numpy().reshape(-1, 16)
    dist1 = eng.distance(ds, union)
    S1 = eng.last_pca_scores(d.N)
    k = S1.shape[1]
    print(f"fsi={fsi} |U|={len(union)} k={k} max|S_shard - S_single| = {np.max(np.abs(full[:, :k] - S1)):.3g} "
          f"max|S| {np.max(np.abs(S1)):.3g}", flush=True)
    ds.close()
    eng.close()
