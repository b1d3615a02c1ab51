"""Summarise rocprofv3 --pmc CSVs: per kernel (name substring), the median over
dispatches of each counter summed over its per-XCD/per-SE instances.
    python tools/pmc_summary.py <dir> [kernel substring] [--last N]
--last N keeps each pass's last N dispatches of the kernel (a steady regime
after a warm-up)."""
import collections
import csv
import glob
import json
import statistics
import sys

args = sys.argv[1:]
last = 0
if "--last" in args:
    i = args.index("--last")
    last = int(args[i + 1])
    del args[i:i + 2]
root = args[0]
kern = args[1] if len(args) > 1 else "eval_tile"
per = collections.defaultdict(lambda: collections.defaultdict(float))
meta = {}
for f in sorted(glob.glob(f"{root}/**/*counter_collection.csv", recursive=True)):
    for r in csv.DictReader(open(f)):
        if kern not in r["Kernel_Name"]:
            continue
        key = (f, r["Dispatch_Id"])
        per[key][r["Counter_Name"]] += float(r["Counter_Value"])
        meta = {k: r[k] for k in ("Kernel_Name", "Grid_Size", "Workgroup_Size", "LDS_Block_Size", "VGPR_Count",
                                  "Accum_VGPR_Count", "SGPR_Count", "Scratch_Size")}
if last:
    keep = []
    for f in {k[0] for k in per}:
        keep += sorted((k for k in per if k[0] == f), key=lambda k: int(k[1]))[-last:]
    per = {k: per[k] for k in keep}
vals = collections.defaultdict(list)
for d in per.values():
    for c, v in d.items():
        vals[c].append(v)
out = {"kernel": meta, "dispatches": {c: len(v) for c, v in vals.items()},
       "median": {c: statistics.median(v) for c, v in sorted(vals.items())}}
print(json.dumps(out, indent=1))
