"""Per-kernel sums of the PMC passes of scripts/pmc_mfma.sh (per launch)."""
import collections
import csv
import glob
import json
import os
import sys

root = sys.argv[1]
out = {}
for pas in sorted(os.listdir(root)):
    d = os.path.join(root, pas)
    if not os.path.isdir(d):
        continue
    acc = collections.defaultdict(lambda: collections.defaultdict(float))
    disp = collections.defaultdict(set)
    for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            k = r["Kernel_Name"].split("(")[0].replace("void ", "")
            acc[k][r["Counter_Name"]] += float(r["Counter_Value"])
            disp[k].add(r["Dispatch_Id"])
    keep = ("gram", "pearson", "dist_euclid", "ing_", "gather", "rank_waves", "rank_split", "tridiag", "gene_stats")
    out[pas] = {k: {c: v / max(len(disp[k]), 1) for c, v in cs.items()} | {"launches": len(disp[k])}
                for k, cs in acc.items() if any(s in k for s in keep)}
print(json.dumps(out, indent=1))
