"""Eigenvalues of the union-gene Gram (the PCA step's matrix) of a config, for
the eigensolver choice: python scripts/gram_spectrum.py D  -> gpurun_out/spec_D.npy"""
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from scconsensus_amd import _native as nat  # noqa: E402
from scconsensus_amd import api, synth  # noqa: E402

cfg = sys.argv[1] if len(sys.argv) > 1 else "D"
dev = "cuda:0"
if cfg in ("C", "D"):
    d = synth.generate_device(cfg, dev, layout="csc")
    torch.cuda.synchronize()
else:
    d = synth.generate(cfg)
names, code = api.select_clusters(d.labels, 10)
eng = nat.Engine(0)
if cfg in ("C", "D"):
    ds = eng.dataset_csc_device(d.indptr.data_ptr(), d.indices.data_ptr(), d.data.data_ptr(), d.G, d.N, d.nnz)
else:
    ds = eng.dataset_csc(d.indptr, d.indices, d.data, d.G, d.N)
r = eng.de_run(ds, code, len(names), nat.SCC_DE_FAST, fetch="union")
genes = np.asarray(r.union, np.int32)
nu = len(genes)
f64 = dict(dtype=torch.float64, device=dev)
part = torch.zeros(2 * nu + 1, **f64)
eng.pca_shard_colsum(ds, genes, 0, d.N, part.data_ptr())
gram = torch.zeros(nu * nu + 1, **f64)
eng.pca_shard_gram(part.data_ptr(), 1, gram.data_ptr())
torch.cuda.synchronize()
C = gram[: nu * nu].reshape(nu, nu).cpu().numpy()
w = np.linalg.eigvalsh(C)[::-1]
os.makedirs(os.path.join(ROOT, "gpurun_out"), exist_ok=True)
np.save(os.path.join(ROOT, "gpurun_out", f"spec_{cfg}.npy"), w)
w = w / w[0]
print(cfg, "nu", nu, "K", len(names))
print("top 20:", np.round(w[:20], 5).tolist())
for b in [16, 24, 32, 48, 64]:
    print(f"lambda_{b + 1}/lambda_15 = {w[b] / w[14]:.4f}")
print("lambda_16/lambda_15 =", w[15] / w[14])
