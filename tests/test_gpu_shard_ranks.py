"""GPU, 2 processes: the sharded job through a real process
group.  Both ranks share the one MI355X of the test box (gloo carries the
collectives; on a node each rank owns a GPU and RCCL carries them).  Every
rank must end with the unsharded union and rows (bit for bit: the record
exchange is exact), and its distance column slice -- from the PCA sharded
over cell blocks -- must equal the same slice of the unsharded distance
within 1e-6 (the Gram's partial sums are added in another order and config A's PC 15 is near-degenerate)."""
import json
import os
import socket
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

WORKER = r'''
import json, os, sys
import numpy as np
import torch
sys.path.insert(0, os.environ["SCC_ROOT"])
from scconsensus_amd import _native as nat, api, parallel, sharded, synth
d = parallel.init("gloo")
eng = nat.Engine(0)
data = synth.generate("A")
names, code = api.select_clusters(data.labels, 10)
K = len(names)
ds = eng.dataset_csc(data.indptr, data.indices, data.data, data.G, data.N)
got = sharded.de_sharded(eng, ds, code, K, d, torch.device("cuda:0"), fetch="rows")
lo, hi, part = sharded.distance_sharded(eng, ds, got.union, d, torch.device("cuda:0"), device_out_ptr=None)
ref = eng.de_run(ds, code, K, nat.SCC_DE_FAST, fetch="rows")
full = eng.distance(ds, ref.union)
N = data.N
s0, s1 = lo * (2 * N - lo - 1) // 2, hi * (2 * N - hi - 1) // 2
print(json.dumps({"rank": d.rank, "union": bool(np.array_equal(got.union, ref.union)),
                  "p": bool(np.array_equal(got.rows.p, ref.rows.p)), "u2": bool(np.array_equal(got.rows.u2, ref.rows.u2)),
                  "dist": bool(np.max(np.abs(part - full[s0:s1])) < 1e-6), "lo": lo, "hi": hi, "n": len(got.union)}))
d.close()
'''


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def test_two_rank_sharded_job():
    port = _free_port()
    procs = []
    for r in range(2):
        env = dict(os.environ, RANK=str(r), WORLD_SIZE="2", LOCAL_RANK=str(r), MASTER_ADDR="127.0.0.1",
                   MASTER_PORT=str(port), SCC_ROOT=ROOT, SCC_SHARE_GPU="1")
        procs.append(subprocess.Popen([sys.executable, "-c", WORKER], env=env, stdout=subprocess.PIPE,
                                      stderr=subprocess.PIPE, text=True))
    res = []
    for p in procs:
        o, e = p.communicate(timeout=300)
        assert p.returncode == 0, e[-3000:]
        res.append(json.loads(o.strip().splitlines()[-1]))
    res.sort(key=lambda r: r["rank"])
    for r in res:
        assert r["union"] and r["p"] and r["u2"] and r["dist"], r
    assert res[0]["lo"] == 0 and res[0]["hi"] == res[1]["lo"] and res[1]["hi"] == 3000
    assert res[0]["n"] > 50
