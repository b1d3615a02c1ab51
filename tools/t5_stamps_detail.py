"""Per-round and per-XCD workgroup times of eval_tile5 from the raw stamps
written by tools/t5_stamps.py --raw (profiling build): which workgroups are
slow (first or second of a CU's slot, XCD), and how much slot time each CU
loses at its end (one slot idle while the other finishes).

    python tools/t5_stamps_detail.py raw.npz [--slots 2]
"""
import json
import sys

import numpy as np

st = np.load(sys.argv[1])["stamps"]                 # [launch][block][10]
slots = 2
out = {"launches": st.shape[0], "workgroups": st.shape[1]}
rounds, xccs, cu_idle, cu_span = [], {}, [], []
for li in range(st.shape[0]):
    ts, hw, we = st[li, :, 0], st[li, :, 1], st[li, :, 2:]
    te = we.max(axis=1)
    T1 = te.max()
    xcc, hid = hw >> 32, hw & 0xFFFFFFFF
    key = xcc * 4096 + ((hid >> 13) & 7) * 512 + ((hid >> 12) & 1) * 256 + ((hid >> 8) & 15)
    dur = (te - ts) * 1e-2
    for k in np.unique(key):
        m = np.where(key == k)[0]
        o = m[np.argsort(ts[m])]
        for r, b in enumerate(o):
            rounds.append((r, dur[b]))
        ends = np.sort(te[m])
        cu_span.append((ends[-1] - ts[m].min()) * 1e-2)
        cu_idle.append((ends[-1] - ends[-2]) * 1e-2 if len(ends) > 1 else 0.0)   # last slot alone
    for x in np.unique(xcc):
        xccs.setdefault(int(x), []).extend(dur[xcc == x].tolist())
rr = {}
for r, d in rounds:
    rr.setdefault(r, []).append(d)
out["wg_us_by_start_order_on_cu"] = {int(r): {"median": float(np.median(v)), "p10": float(np.percentile(v, 10)),
                                               "p90": float(np.percentile(v, 90)), "n": len(v)} for r, v in rr.items()}
out["wg_us_by_xcc"] = {x: float(np.median(v)) for x, v in sorted(xccs.items())}
out["cu_last_workgroup_alone_us"] = {"median": float(np.median(cu_idle)), "p90": float(np.percentile(cu_idle, 90))}
out["cu_span_us"] = {"median": float(np.median(cu_span)), "min": float(np.min(cu_span)), "max": float(np.max(cu_span))}
print(json.dumps(out, indent=1))
