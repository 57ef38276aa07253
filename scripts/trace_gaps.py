"""Idle gaps between kernels in a rocprofv3 kernel trace (one process, one
GPU): the union of kernel busy intervals vs the wall span of the last `steps`
bench steps (a step starts at each k_ing_hist launch), and the largest gaps
with the kernels on either side.
Usage: python scripts/trace_gaps.py gpurun_out/prof/run_kernel_trace.csv [steps]"""
import csv
import sys

path = sys.argv[1]
steps = int(sys.argv[2]) if len(sys.argv) > 2 else 3
rows = []
for r in csv.DictReader(open(path)):
    rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"].split("(")[0][:48]))
rows.sort()
starts = [i for i, r in enumerate(rows) if r[2].startswith("void k_ing_hist") or r[2].startswith("k_ing_hist")]
if len(starts) < steps + 1:
    sys.exit(f"only {len(starts)} steps in the trace")
# the HBM-resident steps: no large copy (the transfer-inclusive steps stream
# the distance to the host)
clean = [s for s in range(len(starts) - 1)
         if not any(r[2].startswith("__amd_rocclr_copyBuffer") and r[1] - r[0] > 100_000
                    for r in rows[starts[s]:starts[s + 1]])]
for s in clean[-steps:]:
    seg = rows[starts[s]:starts[s + 1]]
    t0, t1 = seg[0][0], seg[-1][1]
    busy, cur_s, cur_e, end_name = 0, seg[0][0], seg[0][1], seg[0][2]
    gaps = []
    for a, b, name in seg[1:]:
        if a > cur_e:
            busy += cur_e - cur_s
            gaps.append((a - cur_e, end_name, name))
            cur_s, cur_e, end_name = a, b, name
        elif b > cur_e:
            cur_e, end_name = b, name
    busy += cur_e - cur_s
    gaps.sort(reverse=True)
    print(f"step: wall {(t1 - t0) / 1e3:.1f} us, busy {busy / 1e3:.1f} us, idle {(t1 - t0 - busy) / 1e3:.1f} us "
          f"in {len(gaps)} gaps")
    for g, a, b in gaps[:8]:
        print(f"   {g / 1e3:7.1f} us  after {a}  before {b}")
