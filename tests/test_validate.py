"""The checksln-style validators (ttga.validate, host/ttga_check.cpp) against
the reference: its golden evaluations, and the reference PROGRAM's own
printed timetable (oracle/_ref/timetabling.ga.uk.2, ga.cpp with its own main,
run as a singleton MPI process), whose printed totalBest the validators
re-derive from the instance (the reference's crossover children
carry stale slot lists, so it may print a totalBest its timetable does not
have). No GPU."""
import json
import pathlib
import subprocess

import numpy as np
import pytest

import ttga
from oracle_lib import ref
from ttga.validate import check_text, evaluate

REPO = pathlib.Path(__file__).resolve().parent.parent
CHECK = REPO / "timetabling-ga-mpi-openmp_amd" / "ttga-check"
REF_BIN = REPO / "oracle" / "_ref" / "timetabling.ga.uk.2"
TAGS = [("canon", "slots", "rooms"), ("rand", "slots", "rand_rooms"), ("skew", "skew_slots", "skew_rooms"),
        ("ls3", "ls3_slots", "ls3_rooms")]


def load(name):
    z = np.load(REPO / "tests" / "golden" / f"{name}.npz")
    E, R, F, S = (int(x) for x in z["dims"])
    return ttga.Instance(E, R, F, S, z["room_size"], z["student_events"], z["room_features"], z["event_features"]), z


def solution_line(slots, rooms, feasible, value, proc=0):
    return json.dumps({"solution": {"feasible": bool(feasible), "procID": proc, "rooms": [int(x) for x in rooms],
                                    "threadID": 0, "timeslots": [int(x) for x in slots], "totalBest": int(value),
                                    "totalTime": 1.0}}, separators=(",", ":"), sort_keys=True)


@pytest.mark.parametrize("name", ["sm", "med", "tight"])
def test_python_validator_vs_reference_goldens(name):
    inst, z = load(name)
    for tag, sk, rk in TAGS:
        for i in range(z[sk].shape[0]):
            ev = evaluate(inst, z[sk][i], z[rk][i])
            assert ev["hcv"] == z[f"eval_{tag}_hcv"][i] and ev["scv"] == z[f"eval_{tag}_scv"][i], (tag, i)
            assert ev["feasible"] == bool(z[f"eval_{tag}_feasible"][i])
            assert ev["penalty"] == z[f"eval_{tag}_penalty"][i]


@pytest.mark.parametrize("name", ["sm", "med", "tight"])
def test_native_validator_vs_reference_goldens(tmp_path, name):
    if not CHECK.exists():
        pytest.skip("ttga-check not built")
    inst, z = load(name)
    tim = tmp_path / f"{name}.tim"
    ttga.write_tim(inst, tim)
    lines, want = [], []
    for tag, sk, rk in TAGS:
        for i in range(z[sk].shape[0]):
            h, s = int(z[f"eval_{tag}_hcv"][i]), int(z[f"eval_{tag}_scv"][i])
            lines.append(solution_line(z[sk][i], z[rk][i], h == 0, s if h == 0 else h * 1000000 + s, len(lines)))
            want.append((h, s))
    bad = solution_line(z["slots"][0], z["rooms"][0], True, 0, len(lines))      # tampered claim
    out = subprocess.run([str(CHECK), str(tim), "-"], input="\n".join(lines + [bad]) + "\n", capture_output=True,
                         text=True, timeout=120)
    reps = [json.loads(x) for x in out.stdout.splitlines()]
    assert out.returncode == 1 and len(reps) == len(lines) + 1
    assert [(r["hcv"], r["scv"]) for r in reps[:-1]] == want and all(r["ok"] for r in reps[:-1])
    assert not reps[-1]["ok"]
    assert check_text(inst, "\n".join(lines))[0]["ok"]


def test_validators_on_reference_program_output(tmp_path):
    """The reference program's own run on the sm instance (one rank, one
    thread): both validators recompute its printed timetable to the
    reference's own Solution::computeHcv/computeScv of that timetable; the
    printed totalBest is reported as agreeing or not (F2)."""
    R = ref()
    if R is None or not REF_BIN.exists():
        pytest.skip("reference build oracle/_ref not present")
    inst, _ = load("sm")
    tim = tmp_path / "sm.tim"
    ttga.write_tim(inst, tim)
    run = subprocess.run([str(REF_BIN), "-i", str(tim), "-s", "42", "-c", "1", "-p", "1"], capture_output=True,
                         text=True, timeout=300, cwd=str(tmp_path))
    assert run.returncode == 0, run.stderr[-2000:]
    objs = [json.loads(x) for x in run.stdout.splitlines() if x.startswith("{")]
    kinds = [tuple(sorted(next(iter(o.values())).keys())) for o in objs]
    assert ("best", "procID", "threadID", "time") in kinds
    assert kinds[-1] == ("procsNum", "threadsNum", "totalTime")
    sol = [o["solution"] for o in objs if "solution" in o][0]
    assert sol["feasible"]
    h, s, f, p = R.problem(inst).eval(np.array(sol["timeslots"], np.uint8)[None], np.array(sol["rooms"], np.uint8)[None])
    py = check_text(inst, run.stdout)[0]
    assert (py["hcv"], py["scv"]) == (int(h[0]), int(s[0]))
    out = subprocess.run([str(CHECK), str(tim), "-"], input=run.stdout, capture_output=True, text=True, timeout=60)
    nat = json.loads(out.stdout.splitlines()[0])
    assert (nat["hcv"], nat["scv"], nat["ok"]) == (py["hcv"], py["scv"], py["ok"])
    assert py["ok"] == (int(s[0]) == sol["totalBest"])
