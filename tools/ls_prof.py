"""Section profile of the local-search kernel (profiling build libttga_prof.so,
-DTT_LS_PROF): shader-clock totals over all waves of one batch, per trial and
per wave. Same workload as tools/bench_ls.py (med, pop 4096, maxSteps 200 from
RandomInitialSolution)."""
import argparse
import ctypes
import json
import pathlib
import sys

REPO = pathlib.Path(__file__).resolve().parent.parent
sys.path.insert(0, str(REPO / "timetabling-ga-mpi-openmp_amd"))
import torch  # noqa: E402

import ttga  # noqa: E402
from ttga import native  # noqa: E402

NAMES = ["init", "build_and_match", "match_task_wave", "corr_in_set", "scv_terms", "sync_accept", "feasible_now",
         "total", "trials", "event_visits", "waves", "scramble", "match_calls", "match_events", "match_steps",
         "p2_move1", "p2_move1_corr_ok", "p2_move1_match_ok", "p2_move2", "p2_move2_corr_ok", "p2_move2_match_ok",
         "p1_move2_quick", "p1_move2_lb_ok", "p1_move1_matched", "p1_move1_accepted", "p1_move1_kept_task",
         "visit_setup_p1", "move1_loop_p1", "move2_loop_p1", "phase1", "phase2", "visit_setup_p2", "move1_loop_p2",
         "move2_loop_p2", "skip_p1", "hot_flags_p1", "max_total", "p1_move1_bound_rejects",
         "p1_move2_bound_rejects", "pair_bound_init", "p1_move2_rejected_after_task0", "p1_move2_accepted"]

ap = argparse.ArgumentParser()
ap.add_argument("--config", default="med")
ap.add_argument("--pop", type=int, default=4096)
ap.add_argument("--steps", type=int, default=200)
ap.add_argument("--pre-steps", type=int, default=0, help="untimed localSearch steps first (phase 2 start)")
ap.add_argument("--from-ga", type=float, default=0.0,
                help="profile the localSearch of GA children: an island (pop --pop, --children) is run until "
                     "this fraction of it is feasible, then one generation's bred children are searched")
ap.add_argument("--children", type=int, default=32768)
ap.add_argument("--warm-gens", type=int, default=400, help="--from-ga: at most this many generations first")
ap.add_argument("--lib", default=None, help="a profiling A/B build (tools/ab_build_one.sh with -DTT_LS_PROF)")
a = ap.parse_args()

lib = native.load(pathlib.Path(a.lib).resolve() if a.lib else native.PKG_DIR / "libttga_prof.so")
native._lib = lib
lib.tt_ls_prof_read.argtypes = [ctypes.c_void_p, ctypes.c_int]
lib.tt_ls_prof_read.restype = ctypes.c_int
inst = ttga.config_instance(a.config)
dp = native.DeviceProblem(inst)
P, E = a.pop, inst.E
s = torch.empty((P, E), dtype=torch.uint8, device="cuda")
r = torch.empty_like(s)
if a.from_ga > 0:
    from ttga.ga import Island
    isl = Island(dp, pop_size=P, children=a.children, max_steps=a.steps, seed=42)
    isl.initialize()
    gens = 0
    while float(isl.pop["feasible"].float().mean().item()) < a.from_ga and gens < a.warm_gens:
        isl.step()
        gens += 1
    c = isl.child
    dp.ga_breed(isl.pop["slot"], isl.pop["room"], isl.pop["penalty"], isl.rng_child, c["slot"], c["room"],
                isl.flags, isl.p_cross, isl.p_mut, isl.skip)
    s, r, P = c["slot"], c["room"], a.children
else:
    dp.random_init(torch.from_numpy(ttga.population_seeds(1000, P)).cuda(), s, r)
if a.pre_steps:
    dp.local_search(s, r, torch.from_numpy(ttga.population_seeds(5000, P)).cuda(), a.pre_steps)
g = torch.from_numpy(ttga.population_seeds(9000, P)).cuda()
buf = (ctypes.c_ulonglong * 64)()
lib.tt_ls_prof_read(buf, 1)
dp.local_search(s, r, g, a.steps)
torch.cuda.synchronize()
n = lib.tt_ls_prof_read(buf, 1)
v = {NAMES[i]: int(buf[i]) for i in range(n)}
trials, waves = max(v["trials"], 1), max(v["waves"], 1)
out = {"config": a.config, "pop": P, "max_steps": a.steps, "from_ga": a.from_ga,
       "ga_generations": gens if a.from_ga > 0 else 0,
       "feasible_at_start": float(isl.pop["feasible"].float().mean().item()) if a.from_ga > 0 else None, "raw": v,
       "cycles_per_trial": {k: v[k] / trials for k in NAMES[:7]},
       "cycles_per_wave": {k: v[k] / waves for k in NAMES[:8] + ["scramble", "visit_setup_p1", "move1_loop_p1",
                                                                  "move2_loop_p1", "phase1", "phase2", "visit_setup_p2",
                                                                  "move1_loop_p2", "move2_loop_p2", "skip_p1",
                                                                  "hot_flags_p1", "pair_bound_init"]},
       "trials_per_wave": v["trials"] / waves, "visits_per_wave": v["event_visits"] / waves,
       "slowest_wave_cycles": v["max_total"], "slowest_over_mean": v["max_total"] / max(v["total"] / waves, 1),
       "note": "s_memtime deltas summed over waves that finished in the first launch; sections nest "
               "(match_task_wave and corr_in_set inside build_and_match/deltas)"}
print(json.dumps(out, indent=1))
