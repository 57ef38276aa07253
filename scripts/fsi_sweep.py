"""Filtered subspace iteration: segments x degree sweep on one configuration's
Gram (the distance stage's eigensolve, Fast:398).  Each setting runs in its
own child process (the engine's graphs are keyed on the context, not on the
knobs); the parent never touches the GPU.
python scripts/fsi_sweep.py B "5,8 4,10 3,12"  ->  eigen ms per call, path, flag"""
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

CHILD = r"""
import os, sys, time
import numpy as np
sys.path.insert(0, %r)
from scconsensus_amd import _native as nat, api, synth
cfg = sys.argv[1]
d = synth.generate(cfg)
names, code = api.select_clusters(d.labels, 10)
eng = nat.Engine(0, profile=True)
ds = eng.dataset_csc(d.indptr, d.indices, d.data, d.G, d.N)
u = eng.de_run(ds, code, len(names), fetch="union").union
for _ in range(3):
    eng.distance(ds, u, nat.SCC_DIST_PCA_EUCLID, device_out_ptr=0)
eng.synchronize()
eng.reset_timers()
reps = 10
for _ in range(reps):
    eng.distance(ds, u, nat.SCC_DIST_PCA_EUCLID, device_out_ptr=0)
eng.synchronize()
t, n = eng.kernel_time("eigen")
print(f"RESULT eigen {t / max(n, 1):.4f} ms path {int(eng.lib.scc_diag_eig_last_path())} |U| {len(u)}", flush=True)
""" % ROOT

cfg = sys.argv[1] if len(sys.argv) > 1 else "B"
combos = (sys.argv[2] if len(sys.argv) > 2 else "5,8 4,10 4,9 3,12 6,7 5,7").split()
for cb in combos:
    s, m = cb.split(",")
    env = dict(os.environ, SCC_EIG_FSI_SEG=s, SCC_EIG_FSI_DEG=m, SCC_EIG_SI_LOG="1")
    r = subprocess.run([sys.executable, "-c", CHILD, cfg], env=env, capture_output=True, text=True, timeout=300)
    res = [ln for ln in r.stdout.splitlines() if ln.startswith("RESULT")]
    logs = [ln for ln in r.stderr.splitlines() if ln.startswith("[scc fsi] n=")]
    print(f"{cfg} seg={s} deg={m}: {res[-1] if res else 'no result (rc %d)' % r.returncode} | "
          f"{logs[-1] if logs else ''}", flush=True)
