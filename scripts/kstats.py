"""Per-kernel summary of a rocprofv3 `--stats` kernel_stats.csv, libscc kernels
only (torch's synthetic-data generators dropped), per step:
    python scripts/kstats.py KSTATS.csv [steps] [limit]"""
import csv
import sys

path = sys.argv[1]
steps = float(sys.argv[2]) if len(sys.argv) > 2 else 1.0
lim = int(sys.argv[3]) if len(sys.argv) > 3 else 40
rows = []
for r in csv.DictReader(open(path)):
    name = r["Name"].strip('"')
    if "at::" in name or "rocprim" in name or "rocclr" in name:
        continue
    short = name.split("(")[0].replace("void ", "")
    rows.append((float(r["TotalDurationNs"]) / 1e3, int(r["Calls"]), float(r["AverageNs"]) / 1e3, short))
rows.sort(reverse=True)
tot = sum(r[0] for r in rows)
print(f"{'calls':>6} {'avg_us':>10} {'per_step_us':>12}  kernel   (libscc total per step {tot / steps:.1f} us)")
for t, n, avg, name in rows[:lim]:
    print(f"{n:6d} {avg:10.1f} {t / steps:12.1f}  {name[:90]}")
