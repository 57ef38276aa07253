"""Time the DE stage under rank-kernel variants (env knobs), config B."""
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
variants = [a.split("=") for a in sys.argv[1:]] or [["SCC_RANK_WIDE", "0"], ["SCC_RANK_WIDE", "1"]]
for k, v in variants:
    env = dict(os.environ, **{k: v})
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--no-cpu-baseline", "--steps", "5"],
                       env=env, capture_output=True, text=True, timeout=300)
    import json
    line = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    if not line:
        print(k, v, "FAILED", r.stderr[-2000:], flush=True)
        continue
    j = json.loads(line[-1])
    sm = j["stage_ms"]
    print(f"{k}={v}: step {j['ms_per_step']:.3f} ms  rank {sm['gene_rank']:.3f}  stats {sm['gene_stats']:.3f}", flush=True)
