"""Statistical comparison of whole GA runs: the reference PROGRAM against the
device GA on 400-event instances (north star: "Full-GA trajectories, whose
RNG differs, are compared statistically on best-scv and feasibility rate over
fixed seeds").

Reference side (CPU, where oracle/_ref/timetabling.ga.uk.2 was built from
/root/reference's own sources):

    python tools/ga_quality_program.py reference --config med --seeds 16 -p 2 \
        --out profiles/r03_ga_refprog_med.json

runs `timetabling.ga.uk.2 -i <config>.tim -s <seed> -p 2 -c 1` once per seed
(one MPI rank, one OpenMP thread: pop 10, one child per generation, 2001
generations, maxSteps 1000, ga.cpp:389-397,490-588), in parallel processes,
and keeps each run's printed best. Because of SURVEY F2 the printed totalBest
of a feasible run can differ from the true cost of the printed timetable, so
the timetable is re-evaluated from the instance (ttga.validate, the
Solution.cpp:63-160 definitions) and that value is the run's outcome.

Device side (GPU; needs the reference JSON only):

    python tools/ga_quality_program.py device --ref profiles/r03_ga_refprog_med.json \
        --out profiles/r03_ga_quality_med.json

runs ttga.ga.Island(pop 10, children 1, maxSteps from -p) for the same seeds
and generation count (islands on separate streams, several at a time) and
compares: feasibility counts (Fisher exact test) and the final values
(Mann-Whitney U, two-sided), plus the best scv among feasible runs.
"""
from __future__ import annotations

import argparse
import json
import os
import pathlib
import subprocess
import sys
import tempfile
import time
from concurrent.futures import ThreadPoolExecutor

REPO = pathlib.Path(__file__).resolve().parent.parent
sys.path.insert(0, str(REPO / "timetabling-ga-mpi-openmp_amd"))
import numpy as np  # noqa: E402

import ttga  # noqa: E402
from ttga.ga import max_steps_for  # noqa: E402
from ttga.validate import evaluate  # noqa: E402

REF_BIN = REPO / "oracle" / "_ref" / "timetabling.ga.uk.2"
GENS = 2001          # ga.cpp:510, generations 0..2000 with one thread


def run_reference(tim: str, seed: int, ptype: int, inst) -> dict:
    t0 = time.perf_counter()
    r = subprocess.run([str(REF_BIN), "-i", tim, "-s", str(seed), "-p", str(ptype), "-c", "1"], capture_output=True,
                       text=True, timeout=7200, cwd=tempfile.gettempdir())
    wall = time.perf_counter() - t0
    if r.returncode != 0:
        raise RuntimeError(f"reference seed {seed}: rc {r.returncode}: {r.stderr[-500:]}")
    objs = [json.loads(ln) for ln in r.stdout.splitlines() if ln.startswith("{")]
    sol = [o["solution"] for o in objs if "solution" in o][-1]
    run = [o["runEntry"] for o in objs if "runEntry" in o and "totalBest" in o["runEntry"]][-1]
    log = [o["logEntry"]["best"] for o in objs if "logEntry" in o]
    out = {"seed": seed, "wall_s": wall, "printed_feasible": bool(sol["feasible"]),
           "printed_totalBest": int(sol["totalBest"]), "run_totalBest": int(run["totalBest"]),
           "log_entries": len(log), "first_logged": log[0] if log else None}
    if "timeslots" in sol:
        ev = evaluate(inst, sol["timeslots"], sol["rooms"])
        out.update(recomputed_hcv=ev["hcv"], recomputed_scv=ev["scv"], feasible=bool(ev["feasible"]),
                   value=ev["scv"] if ev["feasible"] else ev["hcv"] * 1000000 + ev["scv"])
    else:      # an infeasible best carries no timetable (ga.cpp:173-187): the printed value stands
        out.update(feasible=False, value=int(sol["totalBest"]))
    out["printed_matches_timetable"] = out["value"] == out["printed_totalBest"]
    return out


def reference(a):
    if not REF_BIN.exists():
        raise SystemExit(f"{REF_BIN} missing (make -C oracle ref-bin where /root/reference exists)")
    inst = ttga.config_instance(a.config)
    seeds = list(range(a.first_seed, a.first_seed + a.seeds))
    with tempfile.TemporaryDirectory() as d:
        tim = os.path.join(d, f"{a.config}.tim")
        ttga.write_tim(inst, tim)
        with ThreadPoolExecutor(a.jobs) as ex:
            runs = list(ex.map(lambda s: run_reference(tim, s, a.p, inst), seeds))
    res = {"config": a.config, "E": inst.E, "R": inst.R, "F": inst.F, "S": inst.S, "pop_size": 10,
           "children_per_generation": 1, "generations": GENS, "problem_type": a.p, "max_steps": max_steps_for(a.p),
           "seeds": seeds, "program": "oracle/_ref/timetabling.ga.uk.2 (ga.cpp + Solution/Problem/Random/Control/"
                                      "jsoncpp compiled unmodified from the reference), -c 1, one MPI rank",
           "runs": runs, "feasible": int(sum(r["feasible"] for r in runs)),
           "printed_differs_from_timetable": int(sum(not r["printed_matches_timetable"] for r in runs))}
    _dump(res, a.out)


def device(a):
    import torch

    from ttga import native
    from ttga.ga import Island
    ref = json.loads(pathlib.Path(a.ref).read_text())
    inst = ttga.config_instance(ref["config"])
    dp = native.DeviceProblem(inst)
    seeds, steps = ref["seeds"], ref["max_steps"]
    gens = a.gens or ref["generations"]
    finals, feas = {}, {}
    t0 = time.perf_counter()
    for i in range(0, len(seeds), a.concurrent):
        group = seeds[i:i + a.concurrent]
        streams = [torch.cuda.Stream() for _ in group]
        isls = []
        for s, st in zip(group, streams):
            with torch.cuda.stream(st):
                isl = Island(dp, pop_size=10, children=1, max_steps=steps, seed=int(s))
                isl.initialize()
            isls.append(isl)
        for _ in range(gens):
            for isl, st in zip(isls, streams):
                with torch.cuda.stream(st):
                    isl.step()
        torch.cuda.synchronize()
        for s, isl in zip(group, isls):
            f, scv, hcv, _ = isl.member_meta(0)
            feas[s] = bool(f)
            finals[s] = scv if f else hcv * 1000000 + scv
        print(f"seeds {group[0]}..{group[-1]} done, {time.perf_counter() - t0:.1f} s", flush=True)
    wall = time.perf_counter() - t0
    from scipy import stats
    rv = np.array([r["value"] for r in ref["runs"]])
    rf = np.array([r["feasible"] for r in ref["runs"]])
    dv = np.array([finals[s] for s in seeds])
    df = np.array([feas[s] for s in seeds])
    n = len(seeds)
    table = [[int(df.sum()), n - int(df.sum())], [int(rf.sum()), n - int(rf.sum())]]
    res = {"config": ref["config"], "generations": gens, "max_steps": steps, "seeds": seeds,
           "reference": {"feasible": int(rf.sum()), "values": rv.tolist(),
                         "median_value": float(np.median(rv)),
                         "best_scv_feasible": (int(rv[rf].min()) if rf.any() else None),
                         "median_scv_feasible": (float(np.median(rv[rf])) if rf.any() else None),
                         "mean_wall_s_per_run": float(np.mean([r["wall_s"] for r in ref["runs"]]))},
           "device": {"feasible": int(df.sum()), "values": dv.tolist(), "median_value": float(np.median(dv)),
                      "best_scv_feasible": (int(dv[df].min()) if df.any() else None),
                      "median_scv_feasible": (float(np.median(dv[df])) if df.any() else None),
                      "wall_s_all_runs": wall, "concurrent_islands": a.concurrent,
                      "note": "ttga.ga.Island(pop 10, children 1), islands on separate HIP streams"},
           "tests": {"feasibility_fisher_p": float(stats.fisher_exact(table)[1]),
                     "final_value_mannwhitney_p": float(stats.mannwhitneyu(dv, rv, alternative="two-sided").pvalue)}}
    if rf.any() and df.any():
        res["tests"]["feasible_scv_mannwhitney_p"] = float(
            stats.mannwhitneyu(dv[df], rv[rf], alternative="two-sided").pvalue)
    _dump(res, a.out)


def _dump(res, out):
    print(json.dumps(res), flush=True)
    if out:
        pathlib.Path(out).write_text(json.dumps(res, indent=1) + "\n")


def main():
    ap = argparse.ArgumentParser()
    sub = ap.add_subparsers(dest="mode", required=True)
    r = sub.add_parser("reference")
    r.add_argument("--config", default="med")
    r.add_argument("--seeds", type=int, default=16)
    r.add_argument("--first-seed", type=int, default=1)
    r.add_argument("-p", type=int, default=2, help="problem type: maxSteps 200 / 1000 / 2000 (ga.cpp:389-397)")
    r.add_argument("--jobs", type=int, default=max(1, (os.cpu_count() or 2) - 1))
    r.add_argument("--out")
    d = sub.add_parser("device")
    d.add_argument("--ref", required=True)
    d.add_argument("--gens", type=int, default=0, help="0: the reference's 2001")
    d.add_argument("--concurrent", type=int, default=8)
    d.add_argument("--out")
    a = ap.parse_args()
    reference(a) if a.mode == "reference" else device(a)


if __name__ == "__main__":
    main()
