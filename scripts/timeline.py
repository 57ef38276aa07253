"""Timeline of one DE step's libscc kernels from a rocprofv3 --kernel-trace
CSV: for the LAST occurrence of a marker kernel (default k_de_clear, the
step's first), every libscc kernel that started after it up to the next
stage marker, with its start/end relative to the marker, its queue and its
duration (us).  Shows which launches overlap and what the critical path is.
Usage: timeline.py <run_kernel_trace.csv> [first_kernel] [last_kernel_prefix]"""
import csv
import sys


def main():
    path = sys.argv[1]
    first = sys.argv[2] if len(sys.argv) > 2 else "k_de_clear"
    last = sys.argv[3] if len(sys.argv) > 3 else "k_pair_test"
    rows = []
    for r in csv.DictReader(open(path)):
        name = r["Kernel_Name"].replace("void ", "").split("(")[0]
        rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), name, r.get("Queue_Id", "?")))
    rows.sort()
    starts = [i for i, r in enumerate(rows) if r[2].startswith(first)]
    if len(starts) < 1:
        sys.exit(f"no {first}")
    i0 = starts[-2] if len(starts) > 1 else starts[-1]  # the second-to-last step (the last may be truncated)
    t0 = rows[i0][0]
    for s, e, n, q in rows[i0:]:
        print(f"{(s - t0) / 1e3:10.1f} {(e - t0) / 1e3:10.1f} {(e - s) / 1e3:9.1f}  q{q:>3}  {n[:70]}")
        if n.startswith(last):
            break


if __name__ == "__main__":
    main()
