"""Save the config-B DE-gene union (GPU run) for offline spectrum studies."""
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
eng = nat.Engine(0)
ds = eng.dataset_csc(d.indptr, d.indices, d.data, d.G, d.N)
r = eng.de_run(ds, code, len(names), nat.SCC_DE_FAST, fetch="union")
os.makedirs(os.path.join(ROOT, "gpurun_out"), exist_ok=True)
np.save(os.path.join(ROOT, "gpurun_out", f"union_{cfg}.npy"), np.asarray(r.union, np.int32))
print("union", len(r.union))
