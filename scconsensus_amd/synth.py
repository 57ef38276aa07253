"""Deterministic synthetic scRNA-seq inputs of the BASELINE.json shapes.

SURVEY.md §8(d): X = log1p(count / lib * 1e4), count ~ NB(r=2, mu = base_g *
mult_{a,g} * s_c), base_g ~ Gamma(0.3) * 0.5, 5 % marker genes per cluster with
mult ~ U(2, 8), s_c ~ LogNormal(0, 0.3).  The output is a genes x cells CSC
matrix over cells (the R ``dgCMatrix`` layout: per cell, ascending gene rows),
i.e. exactly what ``reclusterDEConsensusFast(dataMatrix = <dgCMatrix>)``
receives, plus consensus labels as strings.

Configs (BASELINE.json ``configs``): A 3k cells x 2k genes K=8; B 26k x 10k
K=12 (PBMC cluster-size profile from the reference's
images/Contingency_Table_Final.png row totals); C 100k x 15k K=30; D 200k x 20k
K=50; E 1M x 20k K=100.  Seeds A=1 ... E=5.
"""
from __future__ import annotations

from dataclasses import dataclass

import numpy as np

# WGCNA::labels2colors-style names (no "grey": the reference drops those).
COLOR_NAMES = [
    "turquoise", "blue", "brown", "yellow", "green", "red", "black", "pink", "magenta",
    "purple", "greenyellow", "tan", "salmon", "cyan", "midnightblue", "lightcyan",
    "lightgreen", "lightyellow", "royalblue", "darkred", "darkgreen", "darkturquoise",
    "orange", "darkorange", "white", "skyblue", "saddlebrown", "steelblue",
    "paleturquoise", "violet", "darkolivegreen", "darkmagenta",
]

PBMC_SIZES = [5484, 4719, 4006, 2631, 2562, 2556, 2099, 1160, 77, 59]

CONFIGS = {
    "A": dict(G=2000, N=3000, K=8, seed=1, sizes="dirichlet"),
    "B": dict(G=10000, N=26000, K=12, seed=2, sizes="pbmc"),
    "C": dict(G=15000, N=100000, K=30, seed=3, sizes="zipf"),
    "D": dict(G=20000, N=200000, K=50, seed=4, sizes="zipf"),
    "E": dict(G=20000, N=1000000, K=100, seed=5, sizes="zipf"),
}


@dataclass
class Dataset:
    G: int
    N: int
    indptr: np.ndarray   # int64 [N+1]   (CSC over cells)
    indices: np.ndarray  # int32 [nnz]   gene row of each stored value
    data: np.ndarray     # float64 [nnz]
    labels: np.ndarray   # object/str [N] consensus labels
    gene_names: list
    cell_names: list

    @property
    def nnz(self) -> int:
        return int(self.indptr[-1])

    def dense(self) -> np.ndarray:
        """Gene-major dense G x N (for the oracle / small configs only)."""
        X = np.zeros((self.G, self.N), np.float64)
        cells = np.repeat(np.arange(self.N), np.diff(self.indptr))
        X[self.indices, cells] = self.data
        return X

    def scipy_csc(self):
        import scipy.sparse as sp
        return sp.csc_matrix((self.data, self.indices, self.indptr), shape=(self.G, self.N))


def label_names(K: int):
    if K <= len(COLOR_NAMES):
        return list(COLOR_NAMES[:K])
    return [f"cl{a:03d}" for a in range(K)]


def cluster_sizes(kind: str, N: int, K: int, rng) -> np.ndarray:
    if kind == "pbmc":
        base = list(PBMC_SIZES)
        extra = K - len(base)
        rest = N - sum(base)
        if extra > 0:
            mids = np.full(extra, rest // extra)
            mids[: rest - mids.sum()] += 1
            base += list(mids)
        sizes = np.array(base[:K], np.int64)
        sizes[0] += N - sizes.sum()
        return sizes
    if kind == "dirichlet":
        floor = 30
        w = rng.dirichlet(np.full(K, 2.0))
        sizes = floor + np.floor(w * (N - floor * K)).astype(np.int64)
    else:  # zipf-like with min 200
        w = 1.0 / np.arange(1, K + 1) ** 0.8
        w /= w.sum()
        floor = min(200, N // (2 * K))
        sizes = floor + np.floor(w * (N - floor * K)).astype(np.int64)
    sizes[0] += N - sizes.sum()
    return sizes


def generate(name: str = "A", *, G=None, N=None, K=None, seed=None, sizes=None,
             block_genes: int = 256) -> Dataset:
    cfg = dict(CONFIGS[name])
    G = cfg["G"] if G is None else G
    N = cfg["N"] if N is None else N
    K = cfg["K"] if K is None else K
    seed = cfg["seed"] if seed is None else seed
    rng = np.random.default_rng(seed)
    sz = cluster_sizes(cfg["sizes"] if sizes is None else sizes, N, K, rng)
    lab_idx = np.repeat(np.arange(K), sz)
    rng.shuffle(lab_idx)
    names = np.array(label_names(K), dtype=object)
    base = rng.gamma(0.3, 1.0, G) * 0.5
    mult = np.ones((K, G))
    nmark = max(1, int(0.05 * G))
    for a in range(K):
        idx = rng.choice(G, nmark, replace=False)
        mult[a, idx] = rng.uniform(2.0, 8.0, nmark)
    s = rng.lognormal(0.0, 0.3, N)
    rows, cols, vals = [], [], []
    for g0 in range(0, G, block_genes):
        g1 = min(G, g0 + block_genes)
        mu = base[g0:g1, None] * mult[:, g0:g1].T[:, lab_idx] * s[None, :]
        lam = rng.gamma(2.0, mu / 2.0)
        cnt = rng.poisson(lam)
        r, c = np.nonzero(cnt)
        rows.append((r + g0).astype(np.int32))
        cols.append(c.astype(np.int64))
        vals.append(cnt[r, c].astype(np.float64))
    rows = np.concatenate(rows)
    cols = np.concatenate(cols)
    vals = np.concatenate(vals)
    lib = np.bincount(cols, weights=vals, minlength=N)
    lib[lib == 0] = 1.0
    x = np.log1p(vals / lib[cols] * 1e4)
    order = np.lexsort((rows, cols))
    rows, cols, x = rows[order], cols[order], x[order]
    indptr = np.zeros(N + 1, np.int64)
    np.cumsum(np.bincount(cols, minlength=N), out=indptr[1:])
    return Dataset(G, N, indptr, rows.astype(np.int32), x, names[lab_idx],
                   [f"gene{g:05d}" for g in range(G)], [f"cell{c:07d}" for c in range(N)])


def from_dense(X: np.ndarray, labels) -> Dataset:
    """Wrap a gene-major dense matrix (tests / edge fixtures)."""
    X = np.asarray(X, np.float64)
    G, N = X.shape
    Xc = X.T  # cells x genes: per cell, ascending genes
    cols, rows = np.nonzero(Xc)
    indptr = np.zeros(N + 1, np.int64)
    np.cumsum(np.bincount(cols, minlength=N), out=indptr[1:])
    return Dataset(G, N, indptr, rows.astype(np.int32), Xc[cols, rows].copy(),
                   np.asarray(labels, dtype=object), [f"gene{g:05d}" for g in range(G)],
                   [f"cell{c:07d}" for c in range(N)])


def edge_fixture(seed: int = 11) -> Dataset:
    """SURVEY §8(d) edge cases in one small matrix: a 20-cell cluster with genes
    that are tie-free (exact p), a "grey" cluster and a "grey60" cluster, a
    cluster of <= 10 cells, constant genes, a gene with pct exactly 20 %
    (n=15, c=3), negative values and explicit ties between clusters."""
    rng = np.random.default_rng(seed)
    sizes = {"turquoise": 60, "blue": 45, "brown": 20, "yellow": 15, "grey": 25, "grey60": 12,
             "tiny": 8, "green": 35}
    labels = np.concatenate([[k] * v for k, v in sizes.items()]).astype(object)
    perm = rng.permutation(len(labels))
    labels = labels[perm]
    N = len(labels)
    G = 120
    X = np.zeros((G, N))
    dens = rng.uniform(0.05, 0.9, G)
    for g in range(G):
        m = rng.random(N) < dens[g]
        X[g, m] = np.log1p(rng.gamma(2.0, 1.0 + (g % 7), m.sum()))
    # cluster-specific markers
    for k, (lab, _) in enumerate(sizes.items()):
        g = 10 + k
        sel = labels == lab
        X[g, sel] = np.log1p(rng.gamma(5.0, 3.0, sel.sum())) + 1.0
    # tie-free genes on the small clusters (exact test branch): all distinct, nonzero
    for g in range(30, 36):
        X[g, :] = rng.permutation(N) / 7.0 + 0.5 + g
    # constant genes
    X[40, :] = 1.25
    X[41, :] = 0.0
    # pct exactly 20 % in "yellow" (n=15 -> 3 cells), zero elsewhere
    X[42, :] = 0.0
    yel = np.nonzero(labels == "yellow")[0]
    X[42, yel[:3]] = [2.0, 2.5, 3.0]
    # a gene with 21 % in yellow-sized... and ties across clusters (integer-like values)
    X[43, :] = rng.integers(0, 4, N).astype(float)
    X[44, :] = np.round(rng.gamma(1.0, 1.0, N), 1)
    # negative values (scaled data is allowed by the math)
    X[45, :] = rng.normal(0.0, 1.0, N)
    X[46, :] = np.where(rng.random(N) < 0.5, -rng.gamma(2.0, 1.0, N), 0.0)
    return from_dense(X, labels)


# ---------------------------------------------------------------- on the GPU
@dataclass
class DeviceDataset:
    """The same generator's matrix built in HBM with torch (synthetic-data
    plumbing for the large configs C/D/E, whose host generation would take
    minutes).  ``layout`` "csc": per cell, ascending gene rows (dgCMatrix);
    "csr": per gene, ascending cells (a gene-major CSR).  The arrays are torch
    tensors on the device; ``labels`` is a host array."""
    G: int
    N: int
    layout: str
    indptr: object   # torch int64 [N+1] (csc) or [G+1] (csr)
    indices: object  # torch int32 [nnz]: gene row (csc) or cell column (csr)
    data: object     # torch float64 [nnz]
    labels: np.ndarray

    @property
    def nnz(self) -> int:
        return int(self.data.numel())

    def to_host(self) -> Dataset:
        """Host CSC copy (the CPU baseline's sample reads it)."""
        import torch
        if self.layout == "csc":
            ip, ix, x = self.indptr.cpu().numpy(), self.indices.cpu().numpy(), self.data.cpu().numpy()
        else:
            rows = torch.repeat_interleave(torch.arange(self.G, device=self.data.device, dtype=torch.int32),
                                           torch.diff(self.indptr))
            key = self.indices.to(torch.int64) * self.G + rows
            order = torch.argsort(key)
            ix = rows[order].cpu().numpy()
            x = self.data[order].cpu().numpy()
            ip = np.zeros(self.N + 1, np.int64)
            np.cumsum(np.bincount(self.indices.cpu().numpy(), minlength=self.N), out=ip[1:])
        return Dataset(self.G, self.N, ip, ix.astype(np.int32), x, self.labels,
                       [f"gene{g:05d}" for g in range(self.G)], [f"cell{c:07d}" for c in range(self.N)])


# Mean-expression scale per config: E's 1M-cell CSR is generated at the
# SURVEY §8(d) E density (~5 %, about 1e9 stored values); the others at the
# generator's natural ~11 %.
DEVICE_BASE_SCALE = {"E": 0.2}


def generate_device(name: str, device, *, seed=None, layout: str = "csc", block_genes: int = 0) -> DeviceDataset:
    """SURVEY §8(d) generator on the GPU: cluster sizes, labels, base, marker
    multipliers and size factors from the host numpy stream (as `generate`);
    the NB(r=2) counts as Poisson(mu/2 * (E1 + E2)) (a shape-2 gamma is the
    sum of two unit exponentials) from a seeded torch generator, gene block
    by gene block; X = log1p(count / lib * 1e4)."""
    import torch
    cfg = dict(CONFIGS[name])
    G, N, K = cfg["G"], cfg["N"], cfg["K"]
    seed = cfg["seed"] if seed is None else seed
    rng = np.random.default_rng(seed)
    sz = cluster_sizes(cfg["sizes"], N, K, rng)
    lab_idx = np.repeat(np.arange(K), sz)
    rng.shuffle(lab_idx)
    names = np.array(label_names(K), dtype=object)
    base = rng.gamma(0.3, 1.0, G) * 0.5 * DEVICE_BASE_SCALE.get(name, 1.0)
    mult = np.ones((K, G))
    nmark = max(1, int(0.05 * G))
    for a in range(K):
        idx = rng.choice(G, nmark, replace=False)
        mult[a, idx] = rng.uniform(2.0, 8.0, nmark)
    s = rng.lognormal(0.0, 0.3, N)
    dev = torch.device(device)
    gen = torch.Generator(device=dev)
    gen.manual_seed(int(seed) * 7919 + 17)
    t_base = torch.tensor(base, dtype=torch.float32, device=dev)
    t_multT = torch.tensor(mult.T.copy(), dtype=torch.float32, device=dev)  # [G, K]
    t_lab = torch.tensor(lab_idx, dtype=torch.int64, device=dev)
    t_s = torch.tensor(s, dtype=torch.float32, device=dev)
    if block_genes <= 0:
        block_genes = max(1, min(G, (1 << 28) // N))
    rows, cols, cnts = [], [], []
    for g0 in range(0, G, block_genes):
        g1 = min(G, g0 + block_genes)
        mu = t_base[g0:g1, None] * t_multT[g0:g1][:, t_lab] * t_s[None, :]
        u = torch.rand((2, g1 - g0, N), generator=gen, device=dev, dtype=torch.float32).clamp_(min=1e-30)
        lam = mu.mul_(-0.5).mul_(torch.log(u[0] * u[1]))
        del u
        cnt = torch.poisson(lam, generator=gen)
        del lam
        nz = torch.nonzero(cnt)  # row-major: gene-major, ascending cells
        rows.append((nz[:, 0] + g0).to(torch.int32))
        cols.append(nz[:, 1].to(torch.int32))
        cnts.append(cnt[nz[:, 0], nz[:, 1]])
        del cnt, nz
    rows = torch.cat(rows)
    cols = torch.cat(cols)
    v = torch.cat(cnts).to(torch.float64)
    del cnts
    lib = torch.zeros(N, dtype=torch.float64, device=dev).index_add_(0, cols.to(torch.int64), v)
    lib[lib == 0] = 1.0
    x = torch.log1p(v / lib[cols.to(torch.int64)] * 1e4)
    del v, lib
    if layout == "csr":
        indptr = torch.zeros(G + 1, dtype=torch.int64, device=dev)
        indptr[1:] = torch.cumsum(torch.bincount(rows.to(torch.int64), minlength=G), 0)
        return DeviceDataset(G, N, "csr", indptr, cols, x, names[lab_idx])
    key = cols.to(torch.int64) * G + rows.to(torch.int64)
    order = torch.argsort(key)
    del key
    indptr = torch.zeros(N + 1, dtype=torch.int64, device=dev)
    indptr[1:] = torch.cumsum(torch.bincount(cols.to(torch.int64), minlength=N), 0)
    return DeviceDataset(G, N, "csc", indptr, rows[order].contiguous(), x[order].contiguous(), names[lab_idx])
