"""Where the headline eval_tile5 launch spends its time between workgroups:
per-workgroup stamps (s_memrealtime, 10 ns: wave 0's start, every wave's end)
and the CU each workgroup ran on, from the profiling build (libttga_prof.so,
-DTT_T5_STAMP), over back-to-back launches of the bench workload (med,
P = 65,536, bench.py's population; the launch index rides in variant bits
12..14).

Per launch: span (first start -> last end) and the gap to the next launch,
workgroup times, and how full the CUs' workgroup slots are:
  slot_util   = sum of workgroup times / (CUs x slots per CU x span)
  ramp_us     = first start -> every CU holds its full slots
  tail_us     = the first CU out of work -> the last end
  idle_tail   = slot-time idle after the first CU runs out of work / slot-time
  refill_us   = a workgroup's start minus the latest end on its CU before it
                (how long a freed slot waits for the next workgroup), median / p90
  wave_skew_us= per workgroup, last wave end minus first wave end (the slot is
                held until the slowest wave ends), median
    python tools/t5_stamps.py [--config med] [--pop 65536] [--launches 8]
"""
import argparse
import ctypes
import json
import pathlib
import sys
import time

REPO = pathlib.Path(__file__).resolve().parent.parent
sys.path.insert(0, str(REPO / "timetabling-ga-mpi-openmp_amd"))
import numpy as np  # noqa: E402
import torch  # noqa: E402

import ttga  # noqa: E402
from ttga import native  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--config", default="med")
ap.add_argument("--pop", type=int, default=65536)
ap.add_argument("--launches", type=int, default=8)
ap.add_argument("--slots", type=int, default=2, help="resident workgroups per CU")
ap.add_argument("--variant", type=int, default=8)
ap.add_argument("--raw", default=None, help="write the raw stamps (npz)")
a = ap.parse_args()
lib = native.load(REPO / "timetabling-ga-mpi-openmp_amd" / "libttga_prof.so")
native._lib = lib
lib.tt_t5_stamp_read.argtypes = [ctypes.c_void_p, ctypes.c_int]
lib.tt_t5_stamp_read.restype = ctypes.c_int
NL, NB, NWD = 8, 16384, 10                       # kT5Launches, kT5MaxBlocks, kT5Words

inst = ttga.config_instance(a.config)
dp = native.DeviceProblem(inst)
P = a.pop
g = torch.from_numpy(ttga.population_seeds(12345, P)).cuda()
s = torch.empty((P, inst.E), dtype=torch.uint8, device="cuda")
r = torch.empty_like(s)
dp.random_init(g, s, r)
out = [torch.empty(P, dtype=t, device="cuda") for t in (torch.int32, torch.int32, torch.uint8, torch.int32)]
t0 = time.perf_counter()
while time.perf_counter() - t0 < 0.3:
    for _ in range(20):
        dp.eval(s, r, variant=a.variant, out=out)
    torch.cuda.synchronize()
buf = np.zeros(NL * NB * NWD, dtype=np.uint64)
lib.tt_t5_stamp_read(buf.ctypes.data, 1)
L = min(a.launches, NL)
e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
e0.record()
for li in range(L):
    dp.eval(s, r, variant=a.variant | (li << 12), out=out)
e1.record()
torch.cuda.synchronize()
ev_ms = e0.elapsed_time(e1) / L
lib.tt_t5_stamp_read(buf.ctypes.data, 0)
grid = (P + 63) // 64
nw = 4 if a.variant == 7 else 8                   # stamped waves (at most 8)
st = buf.reshape(NL, NB, NWD).astype(np.int64)[:L, :grid]
if a.raw:
    np.savez_compressed(a.raw, stamps=st)
t_s, hw, wend = st[:, :, 0], st[:, :, 1], st[:, :, 2:2 + nw]
t_e = wend.max(axis=2)
assert (t_s > 0).all() and (t_e >= t_s).all(), "missing stamps"
xcc, hid = hw >> 32, hw & 0xFFFFFFFF
cu_key = xcc * 4096 + ((hid >> 13) & 7) * 512 + ((hid >> 12) & 1) * 256 + ((hid >> 8) & 15)
rows, spans = [], []
for li in range(L):
    ts, te, ck = t_s[li], t_e[li], cu_key[li]
    T0, T1 = ts.min(), te.max()
    spans.append((T0, T1))
    keys = np.unique(ck)
    ncu = keys.size
    span = (T1 - T0) * 1e-2
    dur = (te - ts) * 1e-2
    last_end, full_at, refill, per_cu = [], [], [], []
    for k in keys:
        m = ck == k
        s_k, e_k = ts[m], te[m]
        o = np.argsort(s_k)
        s_k, e_k = s_k[o], e_k[o]
        per_cu.append(int(m.sum()))
        last_end.append(e_k.max())
        full_at.append(s_k[min(a.slots, s_k.size) - 1])
        for i in range(a.slots, s_k.size):              # workgroups that waited for a freed slot
            prev = e_k[:i][e_k[:i] <= s_k[i]]
            if prev.size:
                refill.append((s_k[i] - prev.max()) * 1e-2)
    first_out = min(last_end)
    tail = (T1 - first_out) * 1e-2
    busy_tail = np.clip(te - np.maximum(ts, first_out), 0, None).sum() * 1e-2
    skew = (wend[li].max(axis=1) - wend[li].min(axis=1)) * 1e-2
    rows.append({"launch": li, "span_us": float(span), "cus": int(ncu),
                 "wg_per_cu_min": int(min(per_cu)), "wg_per_cu_max": int(max(per_cu)),
                 "wg_median_us": float(np.median(dur)), "wg_p10_us": float(np.percentile(dur, 10)),
                 "wg_p90_us": float(np.percentile(dur, 90)),
                 "slot_util": float(dur.sum() / (ncu * a.slots * span)),
                 "ramp_us": float((max(full_at) - T0) * 1e-2), "tail_us": float(tail),
                 "idle_tail": float((ncu * a.slots * tail - busy_tail) / (ncu * a.slots * span)),
                 "refill_median_us": float(np.median(refill)) if refill else None,
                 "refill_p90_us": float(np.percentile(refill, 90)) if refill else None,
                 "wave_skew_median_us": float(np.median(skew))})
gaps = [float((spans[i + 1][0] - spans[i][1]) * 1e-2) for i in range(L - 1)]
res = {"config": a.config, "P": P, "variant": a.variant, "workgroups": grid, "event_ms_per_launch": ev_ms,
       "stamp_period_us": float((spans[-1][1] - spans[0][0]) * 1e-2 / L), "gap_us": gaps, "launches": rows}
for k in rows[0]:
    if k != "launch" and rows[0][k] is not None:
        res["median_" + k] = float(np.median([x[k] for x in rows]))
print(json.dumps(res, indent=1))
