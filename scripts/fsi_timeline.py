"""Per-kernel timeline of one filtered-subspace eigensolve from a rocprofv3
kernel trace (run_kernel_trace.csv): the window from k_fsi_coef0 to the
kernel before the next non-eigen kernel, with each kernel's duration and the
gap before it, summed by kernel name.

    python scripts/fsi_timeline.py gpurun_out/proffsi/run_kernel_trace.csv [window index]
"""
import csv
import sys
from collections import defaultdict

EIG = ("k_fsi", "k_si_", "k_sig", "k_small_syev", "__amd_rocclr_fill")


def main():
    path = sys.argv[1]
    which = int(sys.argv[2]) if len(sys.argv) > 2 else -1
    rows = sorted(csv.DictReader(open(path)), key=lambda r: int(r["Start_Timestamp"]))
    names = [r["Kernel_Name"].split("(")[0].replace("void ", "") for r in rows]
    starts = [i for i, n in enumerate(names) if n.startswith("k_fsi_coef0")]
    if not starts:
        print("no FSI window")
        return
    i0 = starts[which]
    i1 = i0
    while i1 + 1 < len(rows) and names[i1 + 1].startswith(EIG):
        i1 += 1
    t0 = int(rows[i0]["Start_Timestamp"])
    agg = defaultdict(lambda: [0, 0.0, 0.0])
    prev = t0
    for i in range(i0, i1 + 1):
        s, e = int(rows[i]["Start_Timestamp"]), int(rows[i]["End_Timestamp"])
        a = agg[names[i]]
        a[0] += 1
        a[1] += (e - s) / 1e3
        a[2] += max(0, s - prev) / 1e3
        prev = e
    total = (prev - t0) / 1e3
    busy = sum(a[1] for a in agg.values())
    print(f"window: {i1 - i0 + 1} kernels, {total:.1f} us wall, {busy:.1f} us in kernels, {total - busy:.1f} us gaps")
    for n, (c, d, g) in sorted(agg.items(), key=lambda x: -x[1][1] - x[1][2]):
        print(f"  {n[:40]:40s} x{c:3d}  kernels {d:8.1f} us ({d / c:6.2f} each)  gaps {g:7.1f} us")


if __name__ == "__main__":
    main()
