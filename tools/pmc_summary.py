"""Summarise rocprofv3 --pmc CSVs: per kernel (name substring), the median over
dispatches of each counter summed over its per-XCD/per-SE instances."""
import collections
import csv
import glob
import json
import statistics
import sys

root = sys.argv[1]
kern = sys.argv[2] if len(sys.argv) > 2 else "eval_tile"
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
vals = collections.defaultdict(list)
for d in per.values():
    for c, v in d.items():
        vals[c].append(v)
out = {"kernel": meta, "dispatches": {c: len(v) for c, v in vals.items()},
       "median": {c: statistics.median(v) for c, v in sorted(vals.items())}}
print(json.dumps(out, indent=1))
