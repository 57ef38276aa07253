"""Time scc_silhouette on the config-B distance vector (HBM-resident)."""
import json
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
eng.distance(ds, r.union, device_out_ptr=0)
for _ in range(2):
    eng.silhouette(d.N, code)
eng.synchronize()
eng.reset_timers()
for _ in range(5):
    w, ca = eng.silhouette(d.N, code)
ms = eng.kernel_time("silhouette")
t = ms[0] / ms[1]
stored = 8.0 * d.N * (d.N - 1) / 2
print(json.dumps({"config": cfg, "cells": d.N, "clusters": int(len(np.unique(code))), "silhouette_ms": t,
                  "stored_dist_GBps": stored / t / 1e6, "read_GBps_both_halves": 2 * stored / t / 1e6,
                  "SI": float(np.mean(ca))}), flush=True)
