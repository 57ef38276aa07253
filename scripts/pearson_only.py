"""Run only the Pearson distance (config B shape: the DE union of config B)
a few times, for rocprofv3 passes on k_pearson_mfma.  Prints per-launch ms."""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from scconsensus_amd import _native as nat  # noqa: E402
from scconsensus_amd import api, synth  # noqa: E402

cfg = sys.argv[1] if len(sys.argv) > 1 else "B"
reps = int(sys.argv[2]) if len(sys.argv) > 2 else 5
f32 = os.environ.get("SCC_PEARSON_F32") == "1"
d = synth.generate(cfg)
names, code = api.select_clusters(d.labels, 10)
eng = nat.Engine(0, profile=True)
ds = eng.dataset_csc(d.indptr, d.indices, d.data, d.G, d.N)
uni = eng.de_run(ds, code, len(names), nat.SCC_DE_FAST, fetch="union").union
for _ in range(2):
    eng.distance(ds, uni, nat.SCC_DIST_PEARSON, device_out_ptr=0, f32=f32)
eng.synchronize()
eng.reset_timers()
t0 = time.perf_counter()
for _ in range(reps):
    eng.distance(ds, uni, nat.SCC_DIST_PEARSON, device_out_ptr=0, f32=f32)
eng.synchronize()
ms, n = eng.kernel_time("pearson")
flops = float(d.N) * (d.N - 1) * len(uni)
print(f"N={d.N} |U|={len(uni)} f32out={f32} pearson {ms / n:.3f} ms/launch  {flops / (ms / n) / 1e9:.1f} TF/s "
      f"(wall {(time.perf_counter() - t0) / reps * 1e3:.2f} ms/call)", flush=True)
