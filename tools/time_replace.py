"""tt_ga_replace cost by case (ga.cpp:582-583 for C children at once), HIP
events on the launch stream, comp01 rows (E = 355):

* sorted: survivors already in key order (every generation after the first):
  merge path;
* init: C = 0 on an unsorted population (the initial sort, ga.cpp:433-434);
* migrant: C = 1 with an out-of-order survivor (a migrant written into
  pop[N-2], ga.cpp:514-540, survives only when C = 1): the device-checked
  fallback sort.

    python tools/time_replace.py [--pop 65536] [--children 8192] [--reps 20] [--lib path]
"""
import argparse
import json
import pathlib
import sys

REPO = pathlib.Path(__file__).resolve().parent.parent
sys.path.insert(0, str(REPO / "timetabling-ga-mpi-openmp_amd"))
import numpy as np  # noqa: E402
import torch  # noqa: E402

from ttga import native  # noqa: E402
import ttga  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--pop", type=int, default=65536)
ap.add_argument("--children", type=int, default=8192)
ap.add_argument("--reps", type=int, default=20)
ap.add_argument("--lib", default=None)
a = ap.parse_args()
if a.lib:
    native._lib = native.load(pathlib.Path(a.lib).resolve())
inst = ttga.config_instance("comp01")
dp = native.DeviceProblem(inst)
N, C, E = a.pop, a.children, inst.E
rng = np.random.default_rng(1)


def population(n, sort):
    pen = rng.integers(0, 2_000_000, n).astype(np.int32)
    if sort:
        pen = np.sort(pen)
    d = dict(slot=rng.integers(0, 45, (n, E), dtype=np.uint8), room=rng.integers(0, inst.R, (n, E), dtype=np.uint8),
             hcv=np.zeros(n, np.int32), scv=np.zeros(n, np.int32), feasible=np.zeros(n, np.uint8), penalty=pen)
    return {k: torch.from_numpy(v).cuda() for k, v in d.items()}


work = dp.ga_work(N)
st = torch.cuda.current_stream()


def timed(make, child_n):
    ms = []
    for _ in range(a.reps):
        pop = make()
        child = population(child_n, False) if child_n else None
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(st)
        dp.ga_replace(pop, child, work)
        e1.record(st)
        torch.cuda.synchronize()
        assert np.all(np.diff(pop["penalty"].cpu().numpy().astype(np.int64)) >= 0)
        ms.append(e0.elapsed_time(e1))
    return float(np.median(ms))


def migrant():
    pop = population(N, True)
    pop["penalty"][N - 2] = 0                   # pop[N-2] survives C = 1 out of key order
    return pop


out = {"N": N, "E": E,
       f"sorted_C{C}_ms": timed(lambda: population(N, True), C),
       "init_C0_ms": timed(lambda: population(N, False), 0),
       "migrant_C1_ms": timed(migrant, 1)}
print(json.dumps(out))
