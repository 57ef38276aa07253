"""GPU diagnostics (not a test): run one DE configuration with stage-level
synchronisation (SCC_DEBUG_SYNC=1) and compare with the oracle.

usage: python scripts/diag_gpu.py {forced|B|C|D|E}"""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "oracle")]
import numpy as np  # noqa: E402

import oracle as O  # noqa: E402
from scconsensus_amd import _native as nat  # noqa: E402
from scconsensus_amd import api, synth  # noqa: E402


def log(*a):
    print(f"[{time.strftime('%H:%M:%S')}]", *a, flush=True)


def main(which):
    if which in ("C", "D", "E"):
        import torch  # torch's HIP runtime first (the synthetic matrix is generated with it)
        torch.zeros(1, device="cuda:0")
    eng = nat.Engine(0)
    if which == "forced":
        d = synth.generate("A")
        names, code = api.select_clusters(d.labels, 10)
        ds = eng.dataset_csc(d.indptr, d.indices, d.data, d.G, d.N)
        log("run forced caps", {k: v for k, v in os.environ.items() if k.startswith("SCC_")})
        g = eng.de_run(ds, code, len(names), nat.SCC_DE_FAST, fetch="rows")
        log("gpu done; oracle...")
        o = O.de_fast(d.dense(), code, len(names))
        log("rows equal", np.array_equal(g.rows.gene, o.row_gene), "u2 equal",
            np.array_equal(g.rows.u2, np.round(2 * o.row_W).astype(np.int64)), "union equal",
            np.array_equal(g.union, o.union))
    elif which == "B":
        d = synth.generate("B")
        log("generated B")
        names, code = api.select_clusters(d.labels, 10)
        ds = eng.dataset_csc(d.indptr, d.indices, d.data, d.G, d.N)
        log("uploaded")
        g = eng.de_run(ds, code, len(names), nat.SCC_DE_FAST, fetch="rows")
        log("DE done: union", len(g.union), "rows", len(g.rows.gene), "tested/pair max", g.rows.pair_tested.max())
        dist = eng.distance(ds, g.union, nat.SCC_DIST_PCA_EUCLID, device_out_ptr=0)
        log("dist done")
    elif which in ("C", "D", "E"):
        import torch
        d = synth.generate_device(which, "cuda:0")
        torch.cuda.synchronize()
        log("generated", which, "nnz", d.nnz)
        names, code = api.select_clusters(d.labels, 10)
        ds = eng.dataset_csc_device(d.indptr.data_ptr(), d.indices.data_ptr(), d.data.data_ptr(), d.G, d.N, d.nnz)
        for rep in range(2):
            t0 = time.perf_counter()
            g = eng.de_run(ds, code, len(names), nat.SCC_DE_FAST, fetch="rows")
            log("DE done in", round(time.perf_counter() - t0, 4), "s: union", len(g.union), "rows", len(g.rows.gene),
                "tested/pair max", g.rows.pair_tested.max())
    else:
        raise SystemExit(2)


if __name__ == "__main__":
    main(sys.argv[1])
