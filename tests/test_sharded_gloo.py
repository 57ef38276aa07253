"""CPU, world_size 2 (gloo): the sharded-job orchestration and the
bench launcher, with the engine replaced by a numpy stand-in that follows the
C ABI's buffer contracts (include/scc.h: scc_de_run_shard_records /
scc_de_finish_records, scc_pca_shard_*).  The GPU path itself is covered by
tests/test_gpu_shard.py and tests/test_gpu_shard_ranks.py."""
import json
import os
import socket
import subprocess
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

WORKER = r'''
import ctypes, json, os, sys
import numpy as np
import torch
sys.path.insert(0, os.environ["SCC_ROOT"])
sys.path.insert(0, os.path.join(os.environ["SCC_ROOT"], "oracle"))
from scconsensus_amd import _native as nat, parallel, sharded

REC = np.dtype([("pair", "<i4"), ("gene", "<i4"), ("p", "<f8"), ("lfc", "<f8"), ("pct1", "<f8"), ("pct2", "<f8"),
                ("u2", "<i8"), ("ties", "<i8"), ("flags", "<u4"), ("res", "<u4")])
assert REC.itemsize == 64

def view(ptr, n, dtype):
    dt = np.dtype(dtype)
    return np.frombuffer((ctypes.c_char * (n * dt.itemsize)).from_address(ptr), dtype=dt)

class DS:
    def __init__(self, X):
        self.X = X
        self.G, self.N = X.shape

class Stand:
    """numpy stand-in for the engine (CPU tensors)."""
    def __init__(self, fail):
        self.fail = fail
    def tested(self, K, G):
        P = K * (K - 1) // 2
        return [(p, g) for p in range(P) for g in range(G) if (g + 2 * p) % 3 == 0]
    def de_run_shard_records(self, ds, code, K, lo, hi, ptr, cap, **kw):
        if self.fail == "de":
            raise nat.SccError(5, "R stop() on this rank's genes")
        cells = [(p, g) for p, g in self.tested(K, ds.G) if lo <= g < hi]
        out = view(ptr, cap, REC)
        for i, (p, g) in enumerate(cells):
            out[i] = (p, g, (g + 1) / (ds.G + 1), 0.5 - p, 10.0, 20.0, 2 * g, p, 1, 0)
        return len(cells)
    def de_finish_records(self, ds, code, K, ptr, counts, stride, fetch, **kw):
        got = []
        for b, c in enumerate(counts):
            blk = view(ptr + 64 * b * stride, int(c), REC)
            got += [(int(r["pair"]), int(r["gene"]), int(r["u2"])) for r in blk]
        return sorted(got)
    def de_finish_records_pairs(self, ds, code, K, ptr, counts, stride, plo, phi, first_ptr, **kw):
        if self.fail == "select":
            raise nat.SccError(7, "selection failed on this rank")
        self.pairs_seen = [plo, phi]
        got = self.de_finish_records(ds, code, K, ptr, counts, stride, "union")
        first = view(first_ptr, ds.G, np.int64)
        first[:] = -1
        for p in range(plo, phi):  # "selected": the pair's first three tested genes; key (pair, rank)
            for rank, g in enumerate(sorted(g for pp, g, _ in got if pp == p)[:3]):
                key = (p << 32) | rank
                if first[g] == -1 or key < first[g]:
                    first[g] = key
    def de_union_first_occ(self, first_ptr, G):
        first = view(first_ptr, G, np.int64)
        return np.array([g for _, g in sorted((int(first[g]), g) for g in range(G) if first[g] != -1)], np.int32)
    def pca_shard_colsum(self, ds, genes, lo, hi, part_ptr):
        if self.fail == "pca":
            raise nat.SccError(3, "out of memory on this rank")
        self.genes, self.lo, self.hi, self.ds = genes, lo, hi, ds
        s = ds.X[genes][:, lo:hi].sum(axis=1)
        part = view(part_ptr, 2 * len(genes), np.float64)
        part[0::2] = s
        part[1::2] = 0.0
    def pca_shard_gram(self, parts_ptr, world, gram_ptr):
        if not hasattr(self, "genes"):  # the engine: SCC_ERR_INVALID "call scc_pca_shard_colsum first"
            raise nat.SccError(1, "scc_pca_shard_gram: call scc_pca_shard_colsum first")
        nu = len(self.genes)
        parts = view(parts_ptr, world * 2 * nu, np.float64).reshape(world, 2 * nu)
        mean = (parts[:, 0::2] + parts[:, 1::2]).sum(axis=0) / self.ds.N
        self.Xc = self.ds.X[self.genes][:, self.lo:self.hi].T - mean
        view(gram_ptr, nu * nu, np.float64)[:] = (self.Xc.T @ self.Xc).ravel()
    def pca_shard_eigen(self, gram_ptr, vecs_ptr, ncomp):
        if not hasattr(self, "Xc"):
            raise nat.SccError(1, "scc_pca_shard_eigen: call scc_pca_shard_gram first")
        nu = len(self.genes)
        self.eigen_calls = getattr(self, "eigen_calls", 0) + 1
        if self.fail == "eigen":
            raise nat.SccError(6, "eigensolver hand-off timed out")
        C = view(gram_ptr, nu * nu, np.float64).reshape(nu, nu)
        w, V = np.linalg.eigh(C)
        k = ncomp or min(nu, 15)
        Z = view(vecs_ptr, nu * 16, np.float64).reshape(nu, 16)
        Z[:, :k] = V[:, ::-1][:, :k]
    def pca_shard_project(self, vecs_ptr, scores_ptr, ncomp):
        if not hasattr(self, "Xc"):
            raise nat.SccError(1, "scc_pca_shard_project: call scc_pca_shard_gram first")
        nu = len(self.genes)
        k = ncomp or min(nu, 15)
        Z = view(vecs_ptr, nu * 16, np.float64).reshape(nu, 16)
        S = view(scores_ptr, self.ds.N * 16, np.float64).reshape(self.ds.N, 16)
        S[self.lo:self.hi, :k] = self.Xc @ Z[:, :k]
    def synchronize(self):
        pass

d = parallel.init("gloo")
rng = np.random.default_rng(3)
X = rng.gamma(1.0, 1.0, (40, 300)) * (rng.random((40, 300)) < 0.6)
X[:5] *= np.linspace(4.0, 1.0, 300)  # a few strong directions
ds = DS(X)
fail = os.environ.get("SCC_FAIL_RANK_STAGE", "")
eng = Stand(fail.split(":")[1] if fail and int(fail.split(":")[0]) == d.rank else None)
res = {"rank": d.rank}
try:
    w = np.arange(1, ds.G + 1, dtype=float)  # stored values per gene: later genes heavier
    got = sharded.de_sharded(eng, ds, None, 4, d, torch.device("cpu"), fetch="union", weights=w, pair_split=False)
    res["de_ok"] = got == sorted((p, g, 2 * g) for p, g in eng.tested(4, ds.G))
    # pair-split selection: each rank selects its pairs, first occurrences MIN-combined
    r2 = sharded.de_sharded(eng, ds, None, 4, d, torch.device("cpu"), fetch="union", weights=w)
    want = []
    for p in range(6):
        for g in sorted(g for pp, g in eng.tested(4, ds.G) if pp == p)[:3]:
            if g not in want:
                want.append(g)
    res["union_ok"] = [int(g) for g in r2.union] == want
    res["pairs_seen"] = eng.pairs_seen
    res["genes"] = list(sharded.gene_shard(ds.G, d.rank, d.world, w))
    genes = np.arange(0, 40, 2)
    S = sharded.pca_sharded(eng, ds, genes, d, torch.device("cpu")).numpy().reshape(ds.N, 16)
    import oracle as O
    R = O.pca_scores(X, genes)
    from scipy.spatial.distance import pdist
    res["dist_err"] = float(np.max(np.abs(pdist(S[:, :R.shape[1]]) - pdist(R))))
    res["eigen_calls"] = getattr(eng, "eigen_calls", 0)
except sharded.ShardError as e:
    res["error"] = e.code
print(json.dumps(res))
d.close()
'''


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _run(extra_env=None, script=WORKER):
    port = _free_port()
    procs = []
    for r in range(2):
        env = dict(os.environ, RANK=str(r), WORLD_SIZE="2", LOCAL_RANK=str(r), MASTER_ADDR="127.0.0.1",
                   MASTER_PORT=str(port), SCC_ROOT=ROOT, **(extra_env or {}))
        procs.append(subprocess.Popen([sys.executable, "-c", script], env=env, stdout=subprocess.PIPE,
                                      stderr=subprocess.PIPE, text=True))
    out = []
    for p in procs:
        o, e = p.communicate(timeout=240)
        assert p.returncode == 0, e[-3000:]
        out.append(json.loads(o.strip().splitlines()[-1]))
    return sorted(out, key=lambda r: r["rank"])


def test_sharded_job_two_ranks():
    """Records exchange gives every rank every tested cell; gene shards are
    balanced by weight; the sharded PCA (column sums all-gathered in rank
    order, Gram all-reduced, disjoint score rows) gives the exact-SVD
    distances."""
    res = _run()
    for r in res:
        assert r["de_ok"], r
        assert r["dist_err"] < 1e-9, r
    assert res[0]["genes"][0] == 0 and res[0]["genes"][1] == res[1]["genes"][0] and res[1]["genes"][1] == 40
    assert res[0]["genes"][1] > 20  # weights 1..40: the lighter genes make the bigger block
    # one eigensolve (rank 0), its vectors broadcast to every rank
    assert [r["eigen_calls"] for r in res] == [1, 0]
    # pair-split selection: pairs [0, 3) and [3, 6), the union equals the all-pairs one
    assert all(r["union_ok"] for r in res), res
    assert [r["pairs_seen"] for r in res] == [[0, 3], [3, 6]]


def test_error_on_one_rank_raises_everywhere():
    """a failure one rank alone sees (an R stop() on its genes, an
    OOM) must raise on every rank, not leave the other blocked in a collective."""
    for rank, stage, code in ((1, "de", 5), (1, "pca", 3), (0, "eigen", 6), (1, "select", 7)):
        res = _run({"SCC_FAIL_RANK_STAGE": f"{rank}:{stage}"})
        assert [r.get("error") for r in res] == [code, code], (stage, res)


def test_weighted_range():
    from scconsensus_amd.parallel import weighted_range
    for w in (np.ones(10), np.arange(1, 101.0), np.r_[np.zeros(5), 100.0, np.ones(50)], np.zeros(7)):
        for world in (1, 2, 3, 8):
            parts = [weighted_range(w, r, world) for r in range(world)]
            assert parts[0][0] == 0 and parts[-1][1] == len(w)
            assert all(parts[i][1] == parts[i + 1][0] for i in range(world - 1))
    w = np.arange(1, 101.0)
    a, b = weighted_range(w, 0, 2), weighted_range(w, 1, 2)
    assert abs(w[a[0]:a[1]].sum() - w[b[0]:b[1]].sum()) <= w.max()


def test_bench_launcher_two_ranks():
    """`bench.py --gpus 2` (no WORLD_SIZE in the environment) starts its own 2
    ranks through torch.distributed.run; the line reports n_gpus 2 and shard2."""
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    p = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--dry-run", "--steps", "2",
                        "--warmup", "1"], env=env, capture_output=True, text=True, timeout=240)
    assert p.returncode == 0, p.stderr[-3000:]
    line = json.loads([ln for ln in p.stdout.splitlines() if ln.startswith("{")][-1])
    assert line["n_gpus"] == 2 and line["config"]["parallelism"] == "shard2" and line["scaling"] == "strong"
    p = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--dry-run", "--mode", "jobs",
                        "--steps", "2", "--warmup", "1"], env=env, capture_output=True, text=True, timeout=240)
    line = json.loads([ln for ln in p.stdout.splitlines() if ln.startswith("{")][-1])
    assert line["config"]["parallelism"] == "jobs2" and line["scaling"] == "weak"
