"""CPU, world_size 2 (gloo): the multi-process path bench.py takes for N > 1
(rank discovery, barrier, max-over-ranks step time, per-rank job seeds,
balanced shards) runs correctly on 2 ranks."""
import os
import socket
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

WORKER = r'''
import json, os, sys, time
sys.path.insert(0, os.environ["SCC_ROOT"])
from scconsensus_amd import parallel, synth
d = parallel.init("gloo")
assert d.world == 2
d.barrier()
t = 0.5 + d.rank                       # rank 1 is the slow one
mx = d.max_over_ranks(t)
tot = d.sum_over_ranks(1.0)
seed = parallel.job_seed(2, d.rank)
ds = synth.generate("A", G=50, N=200, K=4, seed=seed)
lo, hi = parallel.shard_range(10007, d.rank, d.world)
print(json.dumps({"rank": d.rank, "max": mx, "tot": tot, "seed": seed, "nnz": int(ds.nnz), "lo": lo, "hi": hi}))
d.close()
'''


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def test_two_rank_gloo():
    port = _free_port()
    procs = []
    for r in range(2):
        env = dict(os.environ, RANK=str(r), WORLD_SIZE="2", LOCAL_RANK=str(r), MASTER_ADDR="127.0.0.1",
                   MASTER_PORT=str(port), SCC_ROOT=ROOT)
        procs.append(subprocess.Popen([sys.executable, "-c", WORKER], env=env, stdout=subprocess.PIPE,
                                      stderr=subprocess.PIPE, text=True))
    outs = []
    for p in procs:
        o, e = p.communicate(timeout=240)
        assert p.returncode == 0, e
        outs.append(o.strip().splitlines()[-1])
    import json
    res = sorted((json.loads(o) for o in outs), key=lambda r: r["rank"])
    assert all(r["max"] == 1.5 for r in res)          # step time = max over ranks
    assert all(r["tot"] == 2.0 for r in res)
    assert res[0]["seed"] != res[1]["seed"]            # independent jobs (weak scaling)
    assert res[0]["nnz"] != res[1]["nnz"]
    assert res[0]["lo"] == 0 and res[0]["hi"] == res[1]["lo"] and res[1]["hi"] == 10007


def test_shard_range_balanced():
    from scconsensus_amd.parallel import shard_range
    for n in (0, 1, 7, 10000, 10007):
        for w in (1, 2, 3, 8):
            parts = [shard_range(n, r, w) for r in range(w)]
            assert parts[0][0] == 0 and parts[-1][1] == n
            assert all(parts[i][1] == parts[i + 1][0] for i in range(w - 1))
            sizes = [b - a for a, b in parts]
            assert max(sizes) - min(sizes) <= 1


SHARD_WORKER = r'''
import ctypes, json, os, sys
import numpy as np
import torch
sys.path.insert(0, os.environ["SCC_ROOT"])
from scconsensus_amd import parallel, sharded

class Fake:
    """Stands in for the engine: a shard writes its genes' cells (g + 1 in
    every pair row) and leaves the rest zero, as scc_de_run_shard does."""
    P = 3
    def de_shard_bytes(self, K, G):
        return 8 * self.P * G
    def de_run_shard(self, ds, code, K, lo, hi, ptr, **kw):
        a = np.ctypeslib.as_array((ctypes.c_int64 * (self.P * ds.G)).from_address(ptr)).reshape(self.P, ds.G)
        a[:] = 0
        a[:, lo:hi] = np.arange(lo, hi) + 1
        self.kw = kw
    def synchronize(self):
        pass
    def de_finish(self, ds, code, K, ptr, fetch, **kw):
        return np.ctypeslib.as_array((ctypes.c_int64 * (self.P * ds.G)).from_address(ptr)).reshape(self.P, ds.G).copy()

class DS:
    G, N = 1001, 50

d = parallel.init("gloo")
eng = Fake()
out = sharded.de_sharded(eng, DS(), None, 3, d, torch.device("cpu"), fetch="union", exchange="dense",
                         min_per_cent=7.0, top_n=5)
ok = bool((out == np.arange(DS.G) + 1).all())
print(json.dumps({"rank": d.rank, "ok": ok, "kw": sorted(eng.kw), "cols": sharded.column_shard(DS.N, d.rank, d.world),
                  "genes": sharded.gene_shard(DS.G, d.rank, d.world)}))
d.close()
'''


def test_sharded_de_orchestration_two_ranks():
    """The sharded-DE exchange on 2 gloo ranks: every rank ends
    with the exact union of both ranks' shards (the engine is faked; the GPU
    path is covered by tests/test_gpu_shard.py)."""
    port = _free_port()
    procs = []
    for r in range(2):
        env = dict(os.environ, RANK=str(r), WORLD_SIZE="2", LOCAL_RANK=str(r), MASTER_ADDR="127.0.0.1",
                   MASTER_PORT=str(port), SCC_ROOT=ROOT)
        procs.append(subprocess.Popen([sys.executable, "-c", SHARD_WORKER], env=env, stdout=subprocess.PIPE,
                                      stderr=subprocess.PIPE, text=True))
    import json
    res = []
    for p in procs:
        o, e = p.communicate(timeout=240)
        assert p.returncode == 0, e
        res.append(json.loads(o.strip().splitlines()[-1]))
    res.sort(key=lambda r: r["rank"])
    assert all(r["ok"] for r in res)
    assert res[0]["kw"] == ["min_per_cent", "top_n"]
    assert res[0]["genes"] == [0, 501] and res[1]["genes"] == [501, 1001]
    assert res[0]["cols"][0] == 0 and res[0]["cols"][1] == res[1]["cols"][0] and res[1]["cols"][1] == 50


def test_column_shard_balanced():
    from scconsensus_amd.sharded import column_shard
    for n in (2, 3, 10, 1000, 26000, 200000):
        for w in (1, 2, 3, 8):
            parts = [column_shard(n, r, w) for r in range(w)]
            assert parts[0][0] == 0 and parts[-1][1] == n
            assert all(parts[i][1] == parts[i + 1][0] for i in range(w - 1))
            cnt = [b * (2 * n - b - 1) // 2 - a * (2 * n - a - 1) // 2 for a, b in parts]
            assert sum(cnt) == n * (n - 1) // 2
            if n >= 1000:
                assert max(cnt) - min(cnt) <= 2 * n  # each boundary within one column of the ideal split
