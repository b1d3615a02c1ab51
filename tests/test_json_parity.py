"""Driver output and GA selection pinned to the reference's OWN ga.cpp and
jsoncpp (tests/golden/ga_ref.json, written by oracle/gen_golden_ga.py through
oracle/_ref/libttref_ga.so): the four JSON line kinds of ga.cpp:169-257,603-609
reproduced byte for byte (wall-clock times masked) by the Python driver's line
builders and by the native driver (`ttga-ga --replay-log`), jsoncpp's
rendering of doubles, selection5 (ga.cpp:129-145) and the sort of ga.cpp:583
through the oracle's GA primitives. No GPU."""
import json
import pathlib
import re
import subprocess

import numpy as np
import pytest

import ttga
from oracle_lib import oracle
from ttga.ga import CostLog, json_line, run_best_line, run_final_line, solution_line
from ttga.rng import ParkMiller

REPO = pathlib.Path(__file__).resolve().parent.parent
GOLD = json.loads((REPO / "tests" / "golden" / "ga_ref.json").read_text())
EXE = REPO / "timetabling-ga-mpi-openmp_amd" / "ttga-ga"
TIME = re.compile(r'"(time|totalTime)":[-+0-9.eE]+')


def mask(lines):
    return [TIME.sub(r'"\1":T', ln) for ln in lines]


def sm_instance():
    z = np.load(REPO / "tests" / "golden" / "sm.npz")
    E, R, F, S = (int(x) for x in z["dims"])
    return ttga.Instance(E, R, F, S, z["room_size"], z["student_events"], z["room_features"], z["event_features"])


def members(run):
    """(feasible, scv, hcv) of each pop[0] of a golden run, by the oracle."""
    o = oracle().problem(sm_instance())
    sl, rm = np.array(run["slots"], np.uint8), np.array(run["rooms"], np.uint8)
    h, s, f, _ = o.eval(sl, rm)
    return sl, rm, [(bool(a), int(b), int(c)) for a, b, c in zip(f, s, h)]


@pytest.mark.parametrize("k", range(len(GOLD["doubles"])))
def test_doubles_like_jsoncpp(k):
    d = GOLD["doubles"][k]
    assert json_line({"x": float.fromhex(d["value"])}) == d["line"]


@pytest.mark.parametrize("r", range(len(GOLD["logs"])))
def test_log_lines_python_driver(r):
    run = GOLD["logs"][r]
    sl, rm, ms = members(run)
    log = CostLog(run["proc"], None, 0.0)
    got = [x for x in (log.offer(f, s, h, t, 0.0) for (f, s, h), t in zip(ms, run["tids"])) if x]
    f, s, h = ms[-1]
    if run["proc"] == 0:
        got.append(run_best_line(f, s if f else h * 1000000 + s))
    got.append(solution_line({"feasible": f, "scv": s, "hcv": h, "slot": sl[-1], "room": rm[-1]}, run["proc"], 0.0))
    got.append(run_final_line(1, run["threads"], 0.5))
    assert mask(got) == mask(run["lines"])


@pytest.mark.parametrize("r", range(len(GOLD["logs"])))
def test_log_lines_native_driver(tmp_path, r):
    if not EXE.exists():
        pytest.skip("ttga-ga not built")
    run = GOLD["logs"][r]
    sl, rm, ms = members(run)
    E = sl.shape[1]
    rows = [f"{run['proc']} {run['threads']} {len(ms)} {E}"]
    rows += [f"{int(f)} {s} {h} {t}" for (f, s, h), t in zip(ms, run["tids"])]
    rows += [" ".join(map(str, sl[-1])), " ".join(map(str, rm[-1]))]
    (tmp_path / "replay.txt").write_text("\n".join(rows) + "\n")
    out = subprocess.run([str(EXE), "--replay-log", str(tmp_path / "replay.txt")], capture_output=True, text=True,
                         timeout=60)
    assert out.returncode == 0, out.stderr
    assert mask(out.stdout.splitlines()) == mask(run["lines"])


def selection_case_expectations(case):
    """For child k of a breed batch, the stream that continues the golden
    tournament sequence: seed = the Park-Miller state after 10k draws (two
    selection5 of 5 draws each per child)."""
    pm = ParkMiller(case["seed"])
    seeds = []
    for k in range(len(case["winners"]) // 2):
        seeds.append(pm.seed)
        for _ in range(10):
            pm.next()
    return np.array(seeds, np.int64)


@pytest.mark.parametrize("c", range(len(GOLD["selection5"])))
def test_selection5_oracle_vs_reference(c):
    """The oracle's tt_ga_breed restatement draws the same tournaments as the
    reference's selection5: with crossover always on, each child's slots
    follow parent a = winner 2k and parent b = winner 2k+1 per the next E draws."""
    case = GOLD["selection5"][c]
    inst = sm_instance()
    o = oracle().problem(inst)
    N = case["N"]
    rng = np.random.default_rng(c)
    pop_slot = rng.integers(0, 45, (N, inst.E), dtype=np.uint8)
    pop_room = rng.integers(0, inst.R, (N, inst.E), dtype=np.uint8)
    seeds = selection_case_expectations(case)
    pen = np.array(case["penalty"], np.int32)
    cs, cr, fl, st = o.ga_breed(pop_slot, pop_room, pen, seeds, seeds.size, 1.0, 0.0, 0)
    w = np.array(case["winners"])
    for k in range(seeds.size):
        pm = ParkMiller(int(seeds[k]))
        for _ in range(11):                       # two tournaments, the crossover draw
            pm.next()
        take_a = np.array([pm.next() < 0.5 for _ in range(inst.E)])
        exp = np.where(take_a, pop_slot[w[2 * k]], pop_slot[w[2 * k + 1]])
        assert np.array_equal(cs[k], exp), k
    assert fl.tolist() == [1] * seeds.size


@pytest.mark.parametrize("c", range(len(GOLD["sort"])))
def test_sort_vs_reference(c):
    case = GOLD["sort"][c]
    inst = sm_instance()
    o = oracle().problem(inst)
    pen = np.array(case["penalty"], np.int32)
    N = pen.size
    pop = dict(slot=np.zeros((N, inst.E), np.uint8), room=np.zeros((N, inst.E), np.uint8),
               hcv=np.zeros(N, np.int32), scv=np.zeros(N, np.int32), feasible=np.zeros(N, np.uint8), penalty=pen)
    got = o.ga_replace(pop, {k: v[:0] for k, v in pop.items()})
    assert got["penalty"].tolist() == case["sorted"]
