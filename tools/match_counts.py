"""Operation counts of the room matcher (Solution.cpp:836-891) on random rows of
an instance, replayed on the host: per slot, the lane-serial replay's event
expansions, room expansions and dad writes, and the wave matcher's searches,
room-stage steps and augmenting-path steps (csrc/tt_match.h wave_match_slot).
Profiling aid for DESIGN.md §Room assignment; not a checker.

    python tools/match_counts.py [syn] [rows]
"""
import heapq
import pathlib
import sys

import numpy as np

sys.path.insert(0, str(pathlib.Path(__file__).resolve().parent.parent / "timetabling-ga-mpi-openmp_amd"))
import ttga  # noqa: E402


def possible_rooms(inst):
    sn = inst.student_events.sum(axis=0)
    out = []
    for e in range(inst.E):
        ok = (inst.room_size >= sn[e]) & ~((inst.event_features[e][None, :] == 1) & (inst.room_features == 0)).any(axis=1)
        out.append(sum(1 << r for r in range(inst.R) if ok[r]))
    return out


def lane_replay(pl):
    """The reference's lowest-index-first search, step by step."""
    n = dict(searches=0, ev_exp=0, room_exp=0, dad_w=0, path=0)
    N = len(pl)
    mr, rm, unm, rmatched = [None] * N, {}, set(range(N)), 0
    while True:
        n["searches"] += 1
        evq = sorted(unm)
        heapq.heapify(evq)
        sr = fr = 0
        dad, sink = {}, None
        while True:
            if evq:
                i = heapq.heappop(evq)
                n["ev_exp"] += 1
                nr = pl[i] & ~sr
                sr |= nr
                fr |= nr
                j = 0
                while nr:
                    if nr & 1:
                        dad[j] = i
                        n["dad_w"] += 1
                    nr >>= 1
                    j += 1
                continue
            if fr:
                j = (fr & -fr).bit_length() - 1
                fr &= fr - 1
                n["room_exp"] += 1
                if not (rmatched >> j) & 1:
                    sink = j
                    break
                heapq.heappush(evq, rm[j])
                continue
            break
        if sink is None:
            return n
        j = sink
        while True:
            n["path"] += 1
            i = dad[j]
            prev, mr[i], rm[j] = mr[i], j, i
            rmatched |= 1 << j
            if prev is None:
                unm.discard(i)
                break
            j = prev


def wave_counts(pl, R):
    """The wave matcher's stages: closed-form first stage, bulk room pops."""
    n = dict(searches=0, room_steps=0, path=0)
    N = len(pl)
    mr, rm, unm, rmatched = [None] * N, {}, set(range(N)), 0
    while True:
        n["searches"] += 1
        sr, dad = 0, {}
        for i in sorted(unm):
            nr = pl[i] & ~sr
            sr |= nr
            for j in range(R):
                if (nr >> j) & 1:
                    dad[j] = i
        fr, sink = sr, None
        while True:
            n["room_steps"] += 1
            free = fr & ~rmatched
            M = fr & (((free & -free) - 1) if free else (1 << 64) - 1)
            disc = [j for j in range(R) if (M >> j) & 1 and (pl[rm[j]] & ~sr)]
            if not disc:
                if free:
                    sink = (free & -free).bit_length() - 1
                break
            j = disc[0]
            fr &= ~(M & ((2 << j) - 1))
            nr = pl[rm[j]] & ~sr
            sr |= nr
            fr |= nr
            for k in range(R):
                if (nr >> k) & 1:
                    dad[k] = rm[j]
        if sink is None:
            return n
        j = sink
        while True:
            n["path"] += 1
            i = dad[j]
            prev, mr[i], rm[j] = mr[i], j, i
            rmatched |= 1 << j
            if prev is None:
                unm.discard(i)
                break
            j = prev


def main():
    cfg = sys.argv[1] if len(sys.argv) > 1 else "syn"
    rows = int(sys.argv[2]) if len(sys.argv) > 2 else 20
    inst = ttga.config_instance(cfg)
    poss = possible_rooms(inst)
    rng = np.random.default_rng(1)
    lane, wave, events = {}, {}, 0
    for _ in range(rows):
        sl = rng.integers(0, 45, inst.E)
        for t in range(45):
            pl = [poss[e] for e in np.nonzero(sl == t)[0]]
            events += len(pl)
            for k, v in lane_replay(pl).items():
                lane[k] = lane.get(k, 0) + v
            for k, v in wave_counts(pl, inst.R).items():
                wave[k] = wave.get(k, 0) + v
    slots = rows * 45
    print({"config": cfg, "rows": rows, "events_per_slot": events / slots,
           "mean_possible_rooms": float(np.mean([bin(p).count("1") for p in poss])),
           "lane_replay_per_slot": {k: v / slots for k, v in lane.items()},
           "wave_matcher_per_slot": {k: v / slots for k, v in wave.items()}})


if __name__ == "__main__":
    main()
