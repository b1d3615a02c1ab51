"""checksln-style validator: recompute a printed timetable's cost from scratch.

    python -m ttga.validate instance.tim [output.jsonl | -]

reads the JSON lines of a run (ga.cpp's `solution` lines, ga.cpp:169-197, from
ttga-ga, `python -m ttga.islands` or the reference itself), recomputes hcv,
scv and feasibility of every printed timetable from the instance alone, and
checks the printed `totalBest` and `feasible` against them. Exit status 0 when
every line agrees, 1 otherwise (one JSON report line per solution either way).

The cost is the reference's (Solution.cpp:63-160), evaluated here with numpy
from the definitions, independently of the kernels and of the oracle:
  hcv = sum over (slot, room) cells of C(n, 2)               (Solution.cpp:148-150)
      + #{i < j : slot_i == slot_j and corr(i, j)}            (:151-153)
      + #{e : room_e not possible for e}                      (:155-156)
  scv = sum_e [slot_e % 9 == 8] * studentNumber[e]            (:93-96)
      + sum over students, days of max(0, run - 2) per run of consecutive attended slots   (:98-117)
      + #{(student, day) with exactly one attended slot}      (:119-137)
  feasible <=> hcv == 0                                       (:63-84)
"""
from __future__ import annotations

import json
import sys

import numpy as np

SLOTS, PER_DAY, DAYS = 45, 9, 5


def evaluate(inst, timeslots, rooms) -> dict:
    """hcv, scv and their parts for one timetable (event -> slot, room)."""
    t = np.asarray(timeslots, dtype=np.int64).reshape(-1)
    r = np.asarray(rooms, dtype=np.int64).reshape(-1)
    E, R = inst.E, inst.R
    if t.size != E or r.size != E:
        raise ValueError(f"timetable has {t.size} slots / {r.size} rooms for {E} events")
    if t.min(initial=0) < 0 or t.max(initial=0) >= SLOTS or r.min(initial=0) < 0 or r.max(initial=0) >= R:
        raise ValueError("slot outside 0..44 or room outside 0..R-1")
    A = inst.student_events.astype(np.int64)
    sn = A.sum(axis=0)
    X = np.zeros((E, SLOTS), np.int64)
    X[np.arange(E), t] = 1
    # hard constraints
    cells = np.bincount(t * R + r, minlength=SLOTS * R)
    room_pairs = int((cells * (cells - 1) // 2).sum())
    corr = (A.T @ A) > 0
    same = X @ X.T                                         # [slot_i == slot_j]
    corr_pairs = int(np.triu(same * corr, k=1).sum())
    possible = inst.possible_rooms()
    unsuitable = int((possible[np.arange(E), r] == 0).sum())
    hcv = room_pairs + corr_pairs + unsuitable
    # soft constraints
    occ = (A @ X) > 0                                      # student attends something in slot
    days = occ.reshape(inst.S, DAYS, PER_DAY)
    last = int(sn[t % PER_DAY == PER_DAY - 1].sum())
    consec = int((days[:, :, :-2] & days[:, :, 1:-1] & days[:, :, 2:]).sum())
    single = int((days.sum(axis=2) == 1).sum())
    scv = last + consec + single
    return {"hcv": hcv, "scv": scv, "feasible": hcv == 0, "penalty": scv if hcv == 0 else 1000000 + hcv,
            "room_pairs": room_pairs, "corr_pairs": corr_pairs, "unsuitable": unsuitable,
            "last_slot": last, "consecutive": consec, "single_class": single}


def check_line(inst, line: str) -> dict | None:
    """Report for one JSON line if it is a `solution` line, else None.
    Feasible lines carry the timetable (ga.cpp:173-187); infeasible ones only
    the cost, which is then reported unchecked."""
    try:
        obj = json.loads(line)
    except ValueError:
        return None
    sol = obj.get("solution") if isinstance(obj, dict) else None
    if not isinstance(sol, dict):
        return None
    rep = {"procID": sol.get("procID"), "claimed_feasible": sol.get("feasible"), "claimed": sol.get("totalBest")}
    if "timeslots" not in sol or "rooms" not in sol:
        rep.update(checked=False, ok=not sol.get("feasible", False))
        return rep
    ev = evaluate(inst, sol["timeslots"], sol["rooms"])
    value = ev["scv"] if ev["feasible"] else ev["hcv"] * 1000000 + ev["scv"]
    rep.update(checked=True, hcv=ev["hcv"], scv=ev["scv"], feasible=ev["feasible"], value=value,
               ok=bool(ev["feasible"] == bool(sol.get("feasible")) and value == sol.get("totalBest")))
    return rep


def check_text(inst, text: str) -> list[dict]:
    return [r for r in (check_line(inst, ln) for ln in text.splitlines() if ln.startswith("{")) if r is not None]


def main(argv=None) -> int:
    from .instance import read_tim
    argv = sys.argv[1:] if argv is None else argv
    if not argv or len(argv) > 2:
        sys.stderr.write("usage: python -m ttga.validate instance.tim [output.jsonl | -]\n")
        return 2
    inst = read_tim(argv[0])
    text = sys.stdin.read() if len(argv) == 1 or argv[1] == "-" else open(argv[1]).read()
    reps = check_text(inst, text)
    for r in reps:
        print(json.dumps(r, sort_keys=True))
    return 0 if reps and all(r["ok"] for r in reps) else 1


if __name__ == "__main__":
    sys.exit(main())
