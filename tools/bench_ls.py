"""Batched localSearch throughput (BASELINE configs[1]: medium01-size instance,
pop 4096, batched fitness + localSearch on one MI355X) vs the reference's own
Solution::localSearch on the host cores (OpenMP over individuals), same inputs,
results compared bit-for-bit on the CPU sample.

--pre-steps N first runs an untimed localSearch(N) from RandomInitialSolution
(on the GPU; the CPU sample starts from the same output), so the timed calls
start mostly feasible, in phase 2 (Solution.cpp:619-768)."""
import argparse
import ctypes
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

sys.path.insert(0, str(REPO))
from bench import host_cores  # noqa: E402  (every core this job may use + the CPU model)

ap = argparse.ArgumentParser()
ap.add_argument("--config", default="med")
ap.add_argument("--pop", type=int, default=4096)
ap.add_argument("--steps", type=int, default=200, help="maxSteps (-p 1: 200, -p 2: 1000, else 2000)")
ap.add_argument("--reps", type=int, default=3)
ap.add_argument("--cpu-sample", type=int, default=512)
ap.add_argument("--pre-steps", type=int, default=0, help="untimed localSearch steps first (phase 2 start)")
a = ap.parse_args()

inst = ttga.config_instance(a.config)
dp = native.DeviceProblem(inst)
P, E = a.pop, inst.E
seeds0 = torch.from_numpy(ttga.population_seeds(1000, P)).cuda()
s0 = torch.empty((P, E), dtype=torch.uint8, device="cuda")
r0 = torch.empty_like(s0)
dp.random_init(seeds0, s0, r0)
if a.pre_steps:
    dp.local_search(s0, r0, torch.from_numpy(ttga.population_seeds(5000, P)).cuda(), a.pre_steps)
feas_before = int(dp.eval(s0, r0)[2].sum())
lseeds = torch.from_numpy(ttga.population_seeds(9000, P)).cuda()
times = []
for rep in range(a.reps + 1):
    s, r, g = s0.clone(), r0.clone(), lseeds.clone()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    dp.local_search(s, r, g, a.steps)
    hcv, scv, feas, pen = dp.eval(s, r)
    torch.cuda.synchronize()
    if rep:
        times.append(time.perf_counter() - t0)
gpu_s = float(np.median(times))
out = {"config": a.config, "pop": P, "max_steps": a.steps, "pre_steps": a.pre_steps, "gpu_seconds": gpu_s,
       "gpu_ls_per_s": P / gpu_s, "feasible_before": feas_before, "feasible_after": int(feas.sum()),
       "mean_penalty": float(pen.double().mean())}
from oracle_lib import ref  # noqa: E402
R = ref()
if R is not None and a.cpu_sample > 0:
    n = min(a.cpu_sample, P)
    ss, rr, gg = s0[:n].cpu().numpy().copy(), r0[:n].cpu().numpy().copy(), lseeds[:n].cpu().numpy().copy()
    threads, total, model = host_cores()
    fn = R.lib.ref_local_search_timed
    fn.restype = ctypes.c_double
    fn.argtypes = [ctypes.c_void_p] * 4 + [ctypes.c_int] * 3
    h = R.problem(inst)
    P_ = lambda x: x.ctypes.data_as(ctypes.c_void_p)  # noqa: E731
    secs = fn(h.h, P_(ss), P_(rr), P_(gg), n, a.steps, threads)
    same = bool(np.array_equal(ss, s[:n].cpu().numpy()) and np.array_equal(rr, r[:n].cpu().numpy())
                and np.array_equal(gg, g[:n].cpu().numpy()))
    out["cpu_baseline"] = {"kind": "reference", "cores": threads, "cpu_model": model, "host_cores_total": total,
                           "sample": n, "seconds": secs, "ls_per_s": n / secs, "matches_gpu": same}
    out["speedup_vs_cpu"] = out["gpu_ls_per_s"] / out["cpu_baseline"]["ls_per_s"]
print(json.dumps(out))
