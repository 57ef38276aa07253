"""The cold call's distance leg into a fresh pageable buffer, per engine
context: first and repeat call, the streamed-output wall time (`d2h` timer)
beside the whole call.  python scripts/cold_d2h.py [B] (run it once per
SCC_D2H_KERNEL setting, in separate processes)."""
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from scconsensus_amd import _native as nat  # noqa: E402
from scconsensus_amd import api, synth  # noqa: E402

cfg = sys.argv[1] if len(sys.argv) > 1 else "B"
d = synth.generate(cfg)
names, code = api.select_clusters(d.labels, 10)
K = len(names)
warm = nat.Engine(0)  # HIP initialised, as in the bench's process
warm.close()
for ctx in range(2):
    eng = nat.Engine(0, profile=True)
    for tag in ("first", "repeat"):
        ds = eng.dataset_csc(d.indptr, d.indices, d.data, d.G, d.N)
        r = eng.de_run(ds, code, K, nat.SCC_DE_FAST, fetch="nodg")
        eng.reset_timers()
        host = np.empty(d.N * (d.N - 1) // 2, np.float64)
        t0 = time.perf_counter()
        eng.distance(ds, r.union, nat.SCC_DIST_PCA_EUCLID, out=host)
        t1 = time.perf_counter()
        t, n = eng.kernel_time("d2h")
        print(f"SCC_D2H_KERNEL={os.environ.get('SCC_D2H_KERNEL', '1')} context {ctx} {tag}: "
              f"distance {1e3 * (t1 - t0):.1f} ms, streamed output {t:.1f} ms", flush=True)
        ds.close()
        del host
    eng.close()
