"""Per-kernel HBM traffic per launch from the rocprofv3 PMC passes of
scripts/pmc_traffic.sh.  gfx950 correction (MI355X_MICROARCH.md, HBM): FETCH_SIZE
reports half the bytes of wide coalesced streaming reads, so it is doubled;
WRITE_SIZE is exact for 16-B streaming stores.  Both counters are in KiB."""
import collections
import csv
import glob
import json
import os
import sys


def per_kernel(path):
    acc = collections.defaultdict(float)
    disp = collections.defaultdict(set)
    for f in glob.glob(os.path.join(path, "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            k = r["Kernel_Name"].split("(")[0].replace("void ", "")
            acc[k] += float(r["Counter_Value"])
            disp[k].add(r["Dispatch_Id"])
    return {k: (acc[k], len(disp[k])) for k in acc}


root = sys.argv[1]
fe = per_kernel(os.path.join(root, "FETCH_SIZE"))
wr = per_kernel(os.path.join(root, "WRITE_SIZE"))
out = {}
for k in sorted(set(fe) | set(wr)):
    f, nf = fe.get(k, (0.0, 1))
    w, nw = wr.get(k, (0.0, 1))
    fb = 2.0 * f * 1024 / max(nf, 1)
    wb = w * 1024 / max(nw, 1)
    out[k] = {"fetch_bytes_per_launch_corrected": fb, "write_bytes_per_launch": wb,
              "traffic_bytes_per_launch": fb + wb, "launches": max(nf, nw)}
print(json.dumps({"source": "rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE, separate passes over `python3 bench.py "
                            "--config <cfg> --no-cpu-baseline --no-transfers --no-pearson --steps 2 --warmup 2` "
                            "(scripts/pmc_traffic.sh); FETCH_SIZE x2 (gfx950)",
                  "kernels": out}, indent=1))
