"""Full-GA throughput (BASELINE configs[2]: ITC-2002-like comp instances,
population 65,536, full GA on one MI355X vs the host-CPU reference).

GPU: one island (ttga.ga.Island) with N members and C children per generation;
a generation is breed (selection5 x2, crossover p 0.8 / copy, mutation p 0.5)
+ localSearch(maxSteps) + evaluation + replace-worst + sort, all batched on the
device. Metric: children per second over G timed generations (after the
initial population is built and one warm-up generation).

CPU: the reference's own per-child path of ga.cpp:543-577 (three
RandomInitialSolution, two selection5, copies, crossover/copy, mutation,
localSearch, computePenalty) on the host cores, OpenMP over children
(oracle/_ref ref_ga_children), on a sample of children bred from the
population at the start of the timed generations, on the streams the device
gives its first children of the next generation. The reference's replace-worst
+ sort of its 10-member population is omitted from its timing (negligible
there).

Bit-exactness: the same sample of children is bred, searched and evaluated on
the device from the same population snapshot and streams (tt_ga_breed ->
tt_local_search -> tt_eval) and compared with the reference's children:
slots, rooms, hcv, scv, feasible, penalty and final RNG states
("children_match_reference").

    python tools/bench_ga.py [--config comp01] [--pop 65536] [--children 65536]
                             [--gens 3] [--steps 200] [--cpu-sample 512]
                             [--warm-gens N] [--warm-feasible F]

--warm-gens / --warm-feasible run untimed generations first, until a fraction F
of the population is feasible (or N generations), so the timed generations
are the GA's phase-2 regime (feasible parents, localSearch phase 2), where the
reference spends most of a run.
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
import torch  # noqa: E402

import ttga  # noqa: E402
from ttga import native  # noqa: E402
from ttga.ga import Island  # noqa: E402

sys.path.insert(0, str(REPO))
from bench import host_cores  # noqa: E402  (every core this job may use + the CPU model)
from ttga.islands import rank_seed  # noqa: E402

import hashlib  # noqa: E402

from oracle_lib import ref  # noqa: E402


def parser():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="comp01")
    ap.add_argument("--pop", type=int, default=65536)
    ap.add_argument("--children", type=int, default=65536)
    ap.add_argument("--gens", type=int, default=3)
    ap.add_argument("--min-seconds", type=float, default=0.0,
                    help="keep running timed generations until at least this much time has passed")
    ap.add_argument("--steps", type=int, default=200, help="maxSteps (-p 1: 200, -p 2: 1000, else 2000)")
    ap.add_argument("--seed", type=int, default=42)
    ap.add_argument("--cpu-sample", type=int, default=512)
    ap.add_argument("--warm-gens", type=int, default=0, help="at most this many untimed generations first")
    ap.add_argument("--warm-feasible", type=float, default=1.1, help="stop warming once this fraction is feasible")
    ap.add_argument("--lpt", choices=["auto", "on", "off"], default="auto",
                    help="longest-expected-first dispatch of the children's local search (Island default: auto)")
    ap.add_argument("--lib", default=None, help="profiling: an A/B build (tools/ab_build.sh) instead of the in-tree library")
    ap.add_argument("--schedule", choices=["batch", "staggered"], default="batch",
                    help="Island schedule: whole generations, or two half-batches on two streams bred one "
                         "half-batch behind (ttga.ga.Island)")
    ap.add_argument("--parts", type=int, default=2, help="sub-batches of the staggered schedule")
    ap.add_argument("--islands", type=int, default=1,
                    help="K independent islands of --pop members on this GPU, each on its own stream (ttga.islands "
                         "--islands K between migrations); children/s over all K")
    return ap


def run_ga(a):
    """One island on the in-tree (or --lib) library; returns the JSON record."""
    inst = ttga.config_instance(a.config)
    dp = native.DeviceProblem(inst)
    K = max(1, a.islands)
    # island k's seed as ttga.islands gives it (ga.cpp:412); one island: --seed, no stream of its own
    seeds = [a.seed] + [rank_seed(a.seed, k) for k in range(1, K)]
    isls = [Island(dp, pop_size=a.pop, children=a.children, max_steps=a.steps, seed=seeds[k],
                   lpt=None if a.lpt == "auto" else a.lpt == "on", stream=torch.cuda.Stream() if K > 1 else None,
                   schedule=a.schedule, parts=a.parts)
            for k in range(K)]
    isl = isls[0]
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for i in isls:
        i.initialize()
    torch.cuda.synchronize()
    init_s = time.perf_counter() - t0
    for i in isls:
        i.step()                                # warm-up generation
    torch.cuda.synchronize()
    warm = 1

    def feasible_fraction():
        torch.cuda.synchronize()
        return min(float(i.pop["feasible"].float().mean().item()) for i in isls)
    while warm < a.warm_gens and feasible_fraction() < a.warm_feasible:
        for i in isls:
            i.step()
        warm += 1
    feas_start = feasible_fraction()
    torch.cuda.synchronize()
    # snapshot of the population and child streams the CPU sample (and its device replay) breed from
    pop_slot, pop_room = isl.pop["slot"].cpu().numpy().copy(), isl.pop["room"].cpu().numpy().copy()
    pop_pen = isl.pop["penalty"].cpu().numpy().copy()
    snap = {k: v.clone() for k, v in isl.pop.items()}
    snap_rng = isl.rng_child.clone()
    t0 = time.perf_counter()
    gens = 0
    while gens < a.gens or time.perf_counter() - t0 < a.min_seconds:
        for i in isls:                          # K > 1: the islands' streams overlap
            i.step()
        gens += 1
        # the generations are stream-ordered and need no host round trip; the clock is
        # checked against the device every 8 generations (a sync after every one left
        # the GPU idle while the host enqueued the next generation's launches)
        if gens >= a.gens and gens % 8 == 0:
            torch.cuda.synchronize()
    for i in isls:
        i.flush()                               # staggered: the last half-batch replaced inside the clock
    torch.cuda.synchronize()
    gpu_s = time.perf_counter() - t0
    feas, scv, hcv, pen = isl.member_meta(0)
    ph2, allsteps = dp.local_search_stats(isl.stream)      # the last generation's children (diagnostics)
    # digest of the final population (slots, rooms, penalties): equal runs, equal digests
    _h = hashlib.sha256()
    for _k in ("slot", "room", "penalty"):
        _h.update(isl.pop[_k].cpu().numpy().tobytes())
    pop_digest = _h.hexdigest()[:16]
    pf = isl.pop["feasible"].bool()
    out = {"config": a.config, "E": inst.E, "R": inst.R, "F": inst.F, "S": inst.S, "pop": a.pop,
           "children_per_gen": a.children, "islands": K, "schedule": a.schedule,
           "parts": isl.parts, "gens": gens, "max_steps": a.steps, "lpt_dispatch": isl.lpt,
           "init_seconds": init_s,
           "ls_phase2_step_share": ph2 / allsteps if allsteps else None,
           "warm_gens": warm, "feasible_fraction_at_start": feas_start,
           "pop_digest": pop_digest, "gpu_seconds": gpu_s, "gpu_children_per_s": K * a.children * gens / gpu_s,
           "best_scv_feasible": int(isl.pop["scv"][pf].min().item()) if bool(pf.any()) else None,
           "best": {"feasible": feas, "scv": scv, "hcv": hcv, "penalty": pen},
           "feasible_fraction": float(isl.pop["feasible"].float().mean().item())}

    R = ref()
    if R is not None and a.cpu_sample > 0:
        n = min(a.cpu_sample, a.children)
        threads, total, model = host_cores()
        h = R.problem(inst)
        seeds = snap_rng[:n].cpu().numpy().copy()
        res = {}
        for as_is in (1, 0):       # as_is = 0 last: its children are the ones compared
            ref_children, ref_rng, res[as_is] = h.ga_children(pop_slot, pop_room, pop_pen, seeds, a.steps, threads, as_is)
        # the device replay of the same children from the snapshot
        c = {k: torch.empty_like(v[:n]) for k, v in snap.items()}
        g = torch.from_numpy(seeds).cuda()
        fl = torch.zeros(n, dtype=torch.uint8, device="cuda")
        dp.ga_breed(snap["slot"], snap["room"], snap["penalty"], g, c["slot"], c["room"], fl, isl.p_cross, isl.p_mut, True)
        dp.local_search(c["slot"], c["room"], g, a.steps)
        dp.eval(c["slot"], c["room"], out=(c["hcv"], c["scv"], c["feasible"], c["penalty"]))
        torch.cuda.synchronize()
        mism = [k for k in ("slot", "room", "hcv", "scv", "feasible", "penalty")
                if not np.array_equal(c[k].cpu().numpy(), ref_children[k])]
        if not np.array_equal(g.cpu().numpy(), ref_rng):
            mism.append("rng")
        out["children_match_reference"] = {"children": n, "match": not mism, "mismatched": mism,
                                           "feasible_children": int(ref_children["feasible"].sum())}
        out["cpu_baseline"] = {"kind": "reference", "cores": threads, "cpu_model": model, "host_cores_total": total,
                               "sample_children": n, "seconds": res[0],
                               "children_per_s": n / res[0],
                               "what": "ga.cpp:543-577 per child (3x RandomInitialSolution, 2x selection5, copies, "
                                       "crossover into a fresh child / copy, mutation, localSearch, computePenalty), "
                                       "OpenMP over children",
                               "as_is_children_per_s": n / res[1],
                               "as_is_note": "crossover into the child that already holds a random solution, as "
                                             "ga.cpp:543-563 does (SURVEY F2); its doubled slot lists change the "
                                             "local search's work; context only, not used for the speedup"}
        out["speedup_vs_cpu"] = out["gpu_children_per_s"] / out["cpu_baseline"]["children_per_s"]
    return out


if __name__ == "__main__":
    args = parser().parse_args()
    if args.lib:
        native._lib = native.load(pathlib.Path(args.lib).resolve())
    print(json.dumps(run_ga(args)))
