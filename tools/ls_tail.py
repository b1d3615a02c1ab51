"""Where a GA generation's local-search launch spends its tail (profiling build
libttga_prof.so, per-wave records of -DTT_LS_PROF): an island is run to the
warm state of tools/bench_ga.py, one generation's children are bred, evaluated
and ordered longest-expected first (hcv descending, as ttga.ga.Island does),
and their search is launched in that order. Reported: the launch span, how
busy the wave slots were, the slowest waves (duration, start offset, position
in the dispatch order, hcv) and how well hcv ranks the durations; plus the
span list scheduling would give with the measured durations in the hcv order
and in the ideal (duration) order, with the launch's own concurrency.

    python tools/ls_tail.py --config comp15 [--children 8192] [--steps 1000]
"""
import argparse
import ctypes
import json
import pathlib
import sys

REPO = pathlib.Path(__file__).resolve().parent.parent
sys.path.insert(0, str(REPO / "timetabling-ga-mpi-openmp_amd"))
import heapq  # noqa: E402

import numpy as np  # noqa: E402
import torch  # noqa: E402

import ttga  # noqa: E402
from ttga import native  # noqa: E402
from ttga.ga import Island  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--config", default="comp15")
ap.add_argument("--pop", type=int, default=65536)
ap.add_argument("--children", type=int, default=8192)
ap.add_argument("--steps", type=int, default=1000)
ap.add_argument("--warm-gens", type=int, default=96)
ap.add_argument("--warm-feasible", type=float, default=0.6)
ap.add_argument("--dump", default=None, help="npz of per-child durations, trials and features for offline study")
a = ap.parse_args()

lib = native.load(native.PKG_DIR / "libttga_prof.so")
native._lib = lib
lib.tt_ls_wave_read.argtypes = [ctypes.c_void_p, ctypes.c_int]
inst = ttga.config_instance(a.config)
dp = native.DeviceProblem(inst)
isl = Island(dp, pop_size=a.pop, children=a.children, max_steps=a.steps, seed=42, lpt=True)
isl.initialize()
gens = 0
while gens < a.warm_gens and float(isl.pop["feasible"].float().mean().item()) < a.warm_feasible:
    isl.step()
    gens += 1
c = isl.child
dp.ga_breed(isl.pop["slot"], isl.pop["room"], isl.pop["penalty"], isl.rng_child, c["slot"], c["room"], isl.flags,
            isl.p_cross, isl.p_mut, isl.skip)
isl._evaluate(c)
hcv = c["hcv"].cpu().numpy().copy()
c_slot0, c_room0 = c["slot"].cpu().numpy().copy(), c["room"].cpu().numpy().copy()
order = dp.lpt_order(c["hcv"], isl.work)
n = a.children
buf = np.zeros(4 * 65536, dtype=np.uint64)
lib.tt_ls_wave_read(buf.ctypes.data, 1)
torch.cuda.synchronize()
dp.local_search(c["slot"], c["room"], isl.rng_child, a.steps, 1.0, 1.0, 0.0, order=order)
torch.cuda.synchronize()
lib.tt_ls_wave_read(buf.ctypes.data, 0)
rec = buf.reshape(-1, 4)[:n].astype(np.float64)
start, end, cyc, trials = rec[:, 0], rec[:, 1], rec[:, 2], rec[:, 3]
t0, t1 = start.min(), end.max()
dur = end - start                                          # 10 ns units
span = t1 - t0
pos = np.empty(n, dtype=np.int64)
pos[order.cpu().numpy()] = np.arange(n)
# concurrency: the most waves alive at once
ev = sorted([(s, 1) for s in start] + [(e, -1) for e in end])
live = peak = 0
for _, d in ev:
    live += d
    peak = max(peak, live)


def list_schedule(durs, slots):
    h = [0.0] * slots
    heapq.heapify(h)
    fin = 0.0
    for d in durs:
        t = heapq.heappop(h)
        heapq.heappush(h, t + d)
        fin = max(fin, t + d)
    return fin


ordered = dur[order.cpu().numpy()]
slow = np.argsort(-dur)[: max(1, n // 100)]
rank = lambda x: np.argsort(np.argsort(x))  # noqa: E731
rho = float(np.corrcoef(rank(hcv), rank(dur))[0, 1])
out = {"config": a.config, "children": n, "warm_gens": gens,
       "span_us": span / 100.0, "mean_wave_us": float(dur.mean()) / 100.0, "max_wave_us": float(dur.max()) / 100.0,
       "slot_busy": float(dur.sum() / (span * peak)), "peak_waves": peak,
       "spearman_hcv_duration": rho,
       "slowest_1pct": {"dur_us_mean": float(dur[slow].mean()) / 100.0,
                         "start_offset_us_mean": float((start[slow] - t0).mean()) / 100.0,
                         "order_position_median": float(np.median(pos[slow])),
                         "hcv_median": float(np.median(hcv[slow])), "hcv_median_all": float(np.median(hcv)),
                         "trials_mean": float(trials[slow].mean()), "trials_mean_all": float(trials.mean())},
       "list_schedule_us": {"hcv_order": list_schedule(ordered, peak) / 100.0,
                            "duration_order": list_schedule(np.sort(dur)[::-1], peak) / 100.0,
                            "index_order": list_schedule(dur, peak) / 100.0},
       "note": "durations in s_memrealtime units (10 ns); list schedules use the measured durations and the "
               "launch's peak concurrency, so they ignore that a wave runs faster when fewer share its SIMD"}
if a.dump:
    # per-child features of the children as searched (their slots and rooms before the search)
    sl = c_slot0.astype(np.int64)
    rm = c_room0.astype(np.int64)
    sn, corr, poss = dp.derived()
    corr = corr.astype(bool)
    np.fill_diagonal(corr, False)
    E, R = inst.E, inst.R
    cell = sl * R + rm
    n_cell = np.zeros((n, 45 * R), np.int64)
    np.add.at(n_cell, (np.arange(n)[:, None], cell), 1)
    room_pairs = (n_cell * (n_cell - 1) // 2).sum(1)
    n_slot = np.zeros((n, 45), np.int64)
    np.add.at(n_slot, (np.arange(n)[:, None], sl), 1)
    overfull = np.maximum(n_slot - R, 0).sum(1)
    unsuit = (poss[np.arange(E)[None, :], rm] == 0).sum(1)
    corr_ev = np.zeros((n, E), np.int64)
    for i in range(n):
        same = sl[i][:, None] == sl[i][None, :]
        corr_ev[i] = (same & corr).sum(1)
    cell_ev = np.take_along_axis(n_cell, cell, 1) - 1
    ehcv = corr_ev + cell_ev
    np.savez_compressed(a.dump, dur=dur, trials=trials, hcv=hcv, room_pairs=room_pairs, corr_pairs=corr_ev.sum(1) // 2,
                        unsuit=unsuit, overfull=overfull, nhot=(ehcv > 0).sum(1), order_pos=pos)
print(json.dumps(out, indent=1))
