"""Where does the GPU distance differ from the exact SVD?  Splits the error of
`dist` into the PCA part (engine scores vs exact SVD scores) and the distance
kernel part (engine dist vs pdist of the engine's own scores)."""
import sys

import numpy as np
from scipy.spatial.distance import pdist

sys.path[:0] = [".", "oracle"]
import oracle as O  # noqa: E402
from scconsensus_amd import _native as nat  # noqa: E402
from scconsensus_amd import api, synth  # noqa: E402

cfg = sys.argv[1] if len(sys.argv) > 1 else "A"
d = synth.generate(cfg)
names, code = api.select_clusters(d.labels, 10)
eng = nat.Engine(0)
ds = eng.dataset_csc(d.indptr, d.indices, d.data, d.G, d.N)
uni = eng.de_run(ds, code, len(names), nat.SCC_DE_FAST, fetch="union").union
gd = eng.distance(ds, uni)
Sg = eng.last_pca_scores(d.N)
Xu = d.scipy_csc().tocsr()[uni].toarray()
So = O.pca_scores(Xu, np.arange(len(uni)))
k = So.shape[1]
print("N", d.N, "|U|", len(uni), "k", k)
ev_o = (So ** 2).sum(0)
ev_g = (Sg ** 2).sum(0)
print("eigenvalues exact  ", ev_o)
print("rel eig err        ", (ev_g - ev_o) / ev_o)
# per component agreement up to sign
for q in range(k):
    s = np.sign(np.dot(Sg[:, q], So[:, q])) or 1.0
    print(f"comp {q:2d} max |Sg - So| {np.max(np.abs(s * Sg[:, q] - So[:, q])):.3e}")
# subspace agreement
Qg, _ = np.linalg.qr(Sg)
Qo, _ = np.linalg.qr(So)
sv = np.linalg.svd(Qg.T @ Qo, compute_uv=False)
print("subspace: min cos", sv.min(), "sin(max angle)", np.sqrt(max(0.0, 1 - sv.min() ** 2)))
pg = pdist(Sg)
po = pdist(So)
print("dist kernel err  max |gpu dist - pdist(Sg)|", np.max(np.abs(gd - pg)))
print("PCA err          max |pdist(Sg) - pdist(So)|", np.max(np.abs(pg - po)))
print("total            max |gpu dist - pdist(So)|", np.max(np.abs(gd - po)), "max dist", po.max())
