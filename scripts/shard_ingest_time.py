"""Per-rank ingest of a gene shard (1/W of the genes) on a validated dataset:
range read (k_ing_hist rng) vs every entry (SCC_INGEST_FULL=1), and the whole
per-rank DE stage times.  python scripts/shard_ingest_time.py D 8"""
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from scconsensus_amd import _native as nat  # noqa: E402
from scconsensus_amd import api, sharded, synth  # noqa: E402

cfg = sys.argv[1] if len(sys.argv) > 1 else "D"
W = int(sys.argv[2]) if len(sys.argv) > 2 else 8
if cfg in ("C", "D"):
    d = synth.generate_device(cfg, "cuda:0", layout="csc")
    torch.cuda.synchronize()
else:
    d = synth.generate(cfg)
names, code = api.select_clusters(d.labels, 10)
K = len(names)
P = K * (K - 1) // 2
eng = nat.Engine(0, profile=True)
if cfg in ("C", "D"):
    ds = eng.dataset_csc_device(d.indptr.data_ptr(), d.indices.data_ptr(), d.data.data_ptr(), d.G, d.N, d.nnz)
    w = torch.bincount(d.indices.to(torch.int64), minlength=d.G).cpu().numpy()
else:
    ds = eng.dataset_csc(d.indptr, d.indices, d.data, d.G, d.N)
    w = np.bincount(d.indices, minlength=d.G)
eng.de_run(ds, code, K, nat.SCC_DE_FAST, fetch="union")  # validates the dataset
fams = ["ingest", "gene_stats", "gene_rank", "pair_test"]
for full in ("1", "0"):
    os.environ["SCC_INGEST_FULL"] = full
    out = {}
    for r in range(W):
        lo, hi = sharded.gene_shard(d.G, r, W, w)
        cap = max(1, P * (hi - lo))
        buf = torch.empty(cap * 8, dtype=torch.int64, device="cuda:0")
        eng.de_run_shard_records(ds, code, K, lo, hi, buf.data_ptr(), cap)  # warm-up
        eng.synchronize()
        eng.reset_timers()
        for _ in range(3):
            eng.de_run_shard_records(ds, code, K, lo, hi, buf.data_ptr(), cap)
        eng.synchronize()
        for f in fams:
            t, n = eng.kernel_time(f)
            out.setdefault(f, []).append(t / max(n, 1))
        del buf
    print(f"config {cfg}, {W} gene shards, {'full read' if full == '1' else 'range read'}: "
          + ", ".join(f"{f} max {max(v):.3f} mean {np.mean(v):.3f} ms" for f, v in out.items()), flush=True)
