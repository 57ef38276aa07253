"""Per-kernel summary of a rocprofv3 --kernel-trace sqlite output: python scripts/kstats.py DB [limit]"""
import sqlite3
import sys

c = sqlite3.connect(sys.argv[1])
lim = int(sys.argv[2]) if len(sys.argv) > 2 else 30
rows = c.execute("select name, count(*), avg(end-start)/1000.0, sum(end-start)/1000.0 from kernels "
                 "group by name order by 4 desc limit ?", (lim,)).fetchall()
print(f"{'calls':>6} {'avg_us':>10} {'total_us':>11}  kernel")
for r in rows:
    print(f"{r[1]:6d} {r[2]:10.1f} {r[3]:11.1f}  {r[0][:100]}")
