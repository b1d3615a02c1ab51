"""Same-box A/B timing of localSearch builds (profiling only; tools/ab_build.sh
makes the libraries): every library must give the same (slot, room, rng) as
the first; then interleaved timing, median over rounds. Both regimes: phase 1
from RandomInitialSolution (maxSteps 200) and phase 2 after an untimed
localSearch(3000) (maxSteps 1000).

    python tools/ab_ls.py comp01 8192 head wpe4
"""
import json
import pathlib
import sys
import time

REPO = pathlib.Path(__file__).resolve().parent.parent
sys.path.insert(0, str(REPO / "timetabling-ga-mpi-openmp_amd"))
import numpy as np  # noqa: E402
import torch  # noqa: E402

import ttga  # noqa: E402
from ttga import native  # noqa: E402

cfg, P = sys.argv[1], int(sys.argv[2])
names = sys.argv[3:]
inst = ttga.config_instance(cfg)
probs = {}
for name in names:
    lib = native.load(REPO / "ab_libs" / f"libttga_{name}.so")
    saved, native._lib = native._lib, lib
    probs[name] = native.DeviceProblem(inst)
    native._lib = saved
first = probs[names[0]]
s0 = torch.empty((P, inst.E), dtype=torch.uint8, device="cuda")
r0 = torch.empty_like(s0)
first.random_init(torch.from_numpy(ttga.population_seeds(1000, P)).cuda(), s0, r0)
s2, r2 = s0.clone(), r0.clone()
first.local_search(s2, r2, torch.from_numpy(ttga.population_seeds(5000, P)).cuda(), 3000)
lseeds = torch.from_numpy(ttga.population_seeds(9000, P)).cuda()
res = {"config": cfg, "P": P}
for regime, (sa, ra, steps) in {"phase1_ls200": (s0, r0, 200), "phase2_ls1000": (s2, r2, 1000)}.items():
    ref, agree, times = None, {}, {n: [] for n in names}
    for rnd in range(6):
        for n in names:
            s, r, g = sa.clone(), ra.clone(), lseeds.clone()
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            probs[n].local_search(s, r, g, steps)
            torch.cuda.synchronize()
            if rnd:
                times[n].append(time.perf_counter() - t0)
            if ref is None:
                ref = (s, r, g)
            if rnd == 0:
                agree[n] = all(bool(torch.equal(a, b)) for a, b in zip((s, r, g), ref))
    res[regime] = {"agree": agree, "ms_median": {n: round(1e3 * float(np.median(t)), 4) for n, t in times.items()}}
print(json.dumps(res))
