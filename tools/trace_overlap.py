"""Stream overlap in a rocprofv3 kernel trace (--kernel-trace CSV): for the
local-search kernels of the last N dispatches, the union of their busy time,
the sum of their durations and the time two or more ran at once, per stream.

    python tools/trace_overlap.py run_kernel_trace.csv [--kernel local_search_kernel] [--last 40]
"""
import argparse
import csv
import json

ap = argparse.ArgumentParser()
ap.add_argument("trace")
ap.add_argument("--kernel", default="local_search_kernel")
ap.add_argument("--last", type=int, default=40)
a = ap.parse_args()
rows = [r for r in csv.DictReader(open(a.trace)) if a.kernel in r["Kernel_Name"]]
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
rows = rows[-a.last:]
iv = [(int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Stream_Id"]) for r in rows]
ev = sorted([(s, 1) for s, _, _ in iv] + [(e, -1) for _, e, _ in iv])
live, prev, union, multi = 0, None, 0, 0
for t, d in ev:
    if prev is not None and live > 0:
        union += t - prev
        if live > 1:
            multi += t - prev
    live += d
    prev = t
total = sum(e - s for s, e, _ in iv)
span = max(e for _, e, _ in iv) - min(s for s, _, _ in iv)
print(json.dumps({"kernels": len(iv), "streams": sorted({s for _, _, s in iv}), "span_ms": span / 1e6,
                  "busy_union_ms": union / 1e6, "sum_of_durations_ms": total / 1e6,
                  "overlapped_ms": multi / 1e6, "overlap_fraction_of_union": multi / union if union else 0.0,
                  "mean_kernel_ms": total / len(iv) / 1e6}, indent=1))
