"""Kernel time per GA generation over the last N generations of a rocprofv3
kernel trace (profiling only): the window starts at the N-th last launch of the
local-search kernel; prints per-kernel microseconds per generation and shares.

    python tools/trace_window.py gpurun_out/r03_s19/ga_trace/run_kernel_trace.csv 20
"""
import collections
import csv
import json
import sys

path, n = sys.argv[1], int(sys.argv[2])
rows = list(csv.DictReader(open(path)))
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
ls = [r for r in rows if "local_search_kernel" in r["Kernel_Name"]]
t0 = int(ls[-n]["Start_Timestamp"])
win = [r for r in rows if int(r["Start_Timestamp"]) >= t0]
acc = collections.defaultdict(int)
for r in win:
    name = r["Kernel_Name"].split("(")[0].replace("void ", "")
    acc[name] += int(r["End_Timestamp"]) - int(r["Start_Timestamp"])
total = sum(acc.values())
span = max(int(r["End_Timestamp"]) for r in win) - t0
out = {"generations": n, "kernel_us_per_gen": round(total / n / 1e3, 1), "wall_us_per_gen": round(span / n / 1e3, 1),
       "kernels": {k: {"us_per_gen": round(v / n / 1e3, 2), "share": round(v / total, 4)}
                   for k, v in sorted(acc.items(), key=lambda x: -x[1])}}
print(json.dumps(out, indent=1))
