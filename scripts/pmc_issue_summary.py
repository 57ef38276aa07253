"""Per-kernel issue/wait breakdown from scripts/pmc_issue.sh: per launch, the
fractions of wave-cycles spent issuing (ACTIVE_INST_ANY), parked on a wait
counter or barrier (WAIT_ANY) and stalled at issue (WAIT_INST_ANY), VALU and
LDS instructions per wave, LDS bank conflicts per LDS instruction.
(SQ_*_CYCLES / SQ_WAIT_* / SQ_ACTIVE_* count quad-cycles; ratios need no scale.)"""
import collections
import csv
import glob
import json
import os
import sys

root = sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/pmci"
acc = collections.defaultdict(lambda: collections.defaultdict(float))
disp = collections.defaultdict(set)
for f in glob.glob(os.path.join(root, "**", "*counter_collection.csv"), recursive=True):
    for r in csv.DictReader(open(f)):
        k = r["Kernel_Name"].split("(")[0].replace("void ", "")
        acc[k][r["Counter_Name"]] += float(r["Counter_Value"])
        disp[k].add((f, r["Dispatch_Id"]))
out = {}
for k, c in acc.items():
    wc = c.get("SQ_WAVE_CYCLES", 0.0)
    if wc <= 0:
        continue
    waves = c.get("SQ_WAVES", 0.0)
    lds = c.get("SQ_INSTS_LDS", 0.0)
    out[k] = {
        "wave_cycles_total": wc,
        "active_inst_any_frac": c.get("SQ_ACTIVE_INST_ANY", 0.0) / wc,
        "wait_any_frac": c.get("SQ_WAIT_ANY", 0.0) / wc,
        "wait_inst_any_frac": c.get("SQ_WAIT_INST_ANY", 0.0) / wc,
        "active_valu_frac": c.get("SQ_ACTIVE_INST_VALU", 0.0) / wc,
        "active_lds_frac": c.get("SQ_ACTIVE_INST_LDS", 0.0) / wc,
        "valu_insts_per_wave": c.get("SQ_INSTS_VALU", 0.0) / waves if waves else None,
        "lds_insts_per_wave": lds / waves if waves else None,
        "lds_bank_conflict_per_lds_inst": c.get("SQ_LDS_BANK_CONFLICT", 0.0) / lds if lds else None,
        "gui_active_cycles": c.get("GRBM_GUI_ACTIVE", None),
    }
top = sorted(out.items(), key=lambda kv: -kv[1]["wave_cycles_total"])
print(json.dumps({"source": "rocprofv3 --pmc, two passes over `python3 bench.py --no-cpu-baseline --no-pearson "
                            "--no-transfers --steps 2 --warmup 1` (config B), scripts/pmc_issue.sh",
                  "kernels": dict(top[:25])}, indent=1))
