"""Statistical comparison of whole-GA trajectories: the device GA against the
reference's own GA, same parameters, fixed seeds.

The device engine's random streams differ from the reference's (SURVEY F6:
one Park-Miller stream per individual instead of one shared stream), and it
crosses into a fresh child (no F2), so single trajectories cannot be compared
bit for bit (the per-operator kernels are: tests/test_gpu_parity.py). What is
compared is the distribution of outcomes over K fixed seeds:

* reference: ga.cpp with one MPI rank and one OpenMP thread (-c 1), i.e. the
  steady-state GA of pop_size members with one child per generation, run by
  oracle/_ref's ref_ga_run around the reference's own Solution objects, as is
  (F2 included) and with the crossover child fresh (as_is = 0);
* device: ttga.ga.Island(pop_size, children=1), the same generation count.

Per run the outcome is the value ga.cpp's setGlobalCost reports for pop[0]
(scv if feasible, else hcv*1e6 + scv, ga.cpp:234-257). Reported: feasibility
rate (Fisher exact test), best-scv distribution (Mann-Whitney U, two-sided),
medians of the logged best at generation checkpoints, and wall time per run.

    python tools/ga_quality.py [--config sm] [--seeds 16] [--gens 2001] [--steps 200] [--pop 10]
"""
import argparse
import json
import os
import pathlib
import sys
import time

REPO = pathlib.Path(__file__).resolve().parent.parent
sys.path.insert(0, str(REPO / "timetabling-ga-mpi-openmp_amd"))
sys.path.insert(0, str(REPO / "tests"))
import numpy as np  # noqa: E402

import ttga  # noqa: E402


def summarize(final, feas, trace, checkpoints):
    fs = final[feas.astype(bool)]
    return {
        "feasible_rate": float(feas.mean()),
        "best_scv_feasible": {"median": float(np.median(fs)) if fs.size else None,
                              "mean": float(fs.mean()) if fs.size else None,
                              "min": int(fs.min()) if fs.size else None, "max": int(fs.max()) if fs.size else None},
        "final_log_value": [int(v) for v in final],
        "median_logged_best_at_generation": {str(g): float(np.median(trace[:, g])) for g in checkpoints},
    }


def device_runs(inst, seeds, pop, gens, steps, children=1, schedule="batch"):
    import torch

    from ttga import native
    from ttga.ga import Island
    dp = native.DeviceProblem(inst)
    final = np.zeros(len(seeds), np.int64)
    feas = np.zeros(len(seeds), np.uint8)
    trace = np.zeros((len(seeds), gens + 1), np.int64)
    secs = []
    for k, s in enumerate(seeds):
        isl = Island(dp, pop_size=pop, children=children, max_steps=steps, seed=int(s), schedule=schedule)
        tr = torch.zeros(gens + 1, dtype=torch.int64, device="cuda")
        p = isl.pop

        def log(g):      # setCurrentCost's value for pop[0], kept on the device (no per-generation sync)
            h, c = p["hcv"][0].to(torch.int64), p["scv"][0].to(torch.int64)
            tr[g] = torch.where(p["feasible"][0] != 0, c, h * 1000000 + c)

        torch.cuda.synchronize()
        t0 = time.perf_counter()
        isl.initialize()
        log(0)
        for g in range(gens):
            isl.step()
            log(g + 1)
        isl.flush()                      # staggered: the pending sub-batches replaced
        log(gens)
        torch.cuda.synchronize()
        secs.append(time.perf_counter() - t0)
        trace[k] = tr.cpu().numpy()
        feas[k] = 1 if isl.member_meta(0)[0] else 0
        final[k] = trace[k, -1]
    return final, feas, trace, float(np.mean(secs))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="sm")
    ap.add_argument("--seeds", type=int, default=16)
    ap.add_argument("--first-seed", type=int, default=1)
    ap.add_argument("--gens", type=int, default=2001, help="ga.cpp runs generations 0..2000")
    ap.add_argument("--steps", type=int, default=200, help="maxSteps (-p 1: 200, -p 2: 1000, else 2000)")
    ap.add_argument("--pop", type=int, default=10)
    ap.add_argument("--threads", type=int, default=0)
    ap.add_argument("--no-device", action="store_true")
    ap.add_argument("--device-children", type=int, default=1, help="children per device generation")
    ap.add_argument("--device-gens", type=int, default=0, help="device generations (0: --gens)")
    ap.add_argument("--device-schedule", choices=["batch", "staggered"], default="batch")
    ap.add_argument("--no-ref-as-is", action="store_true", help="skip the reference run with F2")
    ap.add_argument("--out", default=None)
    a = ap.parse_args()
    from scipy import stats

    import threading
    t_start = time.perf_counter()

    def heartbeat():                     # the long reference runs print nothing for minutes
        while True:
            time.sleep(30)
            print(f"[ga_quality] running {time.perf_counter() - t_start:.0f} s", file=sys.stderr, flush=True)
    threading.Thread(target=heartbeat, daemon=True).start()

    from oracle_lib import ref
    inst = ttga.config_instance(a.config)
    seeds = list(range(a.first_seed, a.first_seed + a.seeds))
    threads = a.threads or int(os.environ.get("OMP_NUM_THREADS", "0")) or min(16, os.cpu_count() or 1)
    checkpoints = sorted({0, 100, 500, 1000, a.gens // 2, a.gens} & set(range(a.gens + 1)))
    res = {"config": a.config, "E": inst.E, "R": inst.R, "F": inst.F, "S": inst.S, "pop_size": a.pop,
           "children_per_generation": 1, "generations": a.gens, "max_steps": a.steps, "seeds": seeds,
           "runs": {}}
    R = ref()
    if R is None:
        raise SystemExit("oracle/_ref/libttref.so is missing (build it where /root/reference exists)")
    h = R.problem(inst)
    for name, as_is in ((("reference_as_is", 1),) if not a.no_ref_as_is else ()) + (("reference_fresh_child", 0),):
        hcv, scv, feas, pen, trace, secs = h.ga_run(seeds, a.pop, a.gens, a.steps, as_is, threads)
        final = trace[:, -1]
        res["runs"][name] = summarize(final, feas, trace, checkpoints)
        res["runs"][name]["seconds_per_run"] = secs * threads / len(seeds) if len(seeds) >= threads else secs
        res["runs"][name]["note"] = ("ref_ga_run, OpenMP over seeds (%d threads); seconds_per_run = wall x "
                                     "threads / runs" % threads)
    if not a.no_device:
        dg = a.device_gens or a.gens
        final, feas, trace, secs = device_runs(inst, seeds, a.pop, dg, a.steps, a.device_children, a.device_schedule)
        res["runs"]["device"] = summarize(final, feas, trace, sorted({0, dg // 2, dg}))
        res["runs"]["device"]["seconds_per_run"] = secs
        res["runs"]["device"]["note"] = (f"ttga.ga.Island(pop_size, children={a.device_children}, schedule="
                                         f"{a.device_schedule}), {dg} generations ({dg * a.device_children} children; "
                                         f"the reference: {a.gens}), one island at a time on cuda:0")
        tests = {}
        for name in [n for n in ("reference_as_is", "reference_fresh_child") if n in res["runs"]]:
            r = res["runs"][name]
            fa = np.array([v < 1000000 for v in r["final_log_value"]])
            fd = feas.astype(bool)
            table = [[int(fd.sum()), int((~fd).sum())], [int(fa.sum()), int((~fa).sum())]]
            fisher_p = float(stats.fisher_exact(table)[1])
            vd = np.array(res["runs"]["device"]["final_log_value"])
            vr = np.array(r["final_log_value"])
            mw = stats.mannwhitneyu(vd, vr, alternative="two-sided")
            tests["device_vs_" + name] = {"feasibility_fisher_p": fisher_p, "final_value_mannwhitney_p": float(mw.pvalue),
                                          "median_device": float(np.median(vd)), "median_reference": float(np.median(vr))}
        res["tests"] = tests
    line = json.dumps(res)
    print(line, flush=True)
    if a.out:
        pathlib.Path(a.out).write_text(json.dumps(res, indent=1) + "\n")


if __name__ == "__main__":
    main()
