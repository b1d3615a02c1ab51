"""Same-box A/B timing of the room-assignment and mutation kernels (profiling
only; tools/ab_build.sh makes the libraries, "tree" is the in-tree one):
tt_assign_rooms and tt_mutation
on P rows of random slots of an instance, every library's output compared with
the first, HIP-event medians over rounds.

    python tools/ab_rooms.py comp01 8192 head abl1
"""
import json
import pathlib
import sys

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
    lib = native.load(REPO / "timetabling-ga-mpi-openmp_amd" / "libttga.so" if name == "tree"
                      else REPO / "ab_libs" / f"libttga_{name}.so")
    saved, native._lib = native._lib, lib
    probs[name] = native.DeviceProblem(inst)
    native._lib = saved
first = probs[names[0]]
seeds = torch.from_numpy(ttga.population_seeds(777, P)).cuda()
slot = torch.empty((P, inst.E), dtype=torch.uint8, device="cuda")
room = torch.empty_like(slot)
first.random_init(seeds, slot, room)
res = {"config": cfg, "P": P, "assign": {}, "mutation": {}, "agree": {}}
outs = {}
st = torch.cuda.current_stream()
times = {n: {"assign": [], "mutation": []} for n in names}
for rnd in range(11):
    for n in names:
        dp = probs[n]
        r = torch.empty_like(room)
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record(st)
        dp.assign_rooms(slot, r)
        b.record(st)
        s2, r2, g2 = slot.clone(), room.clone(), seeds.clone()
        c, d = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        c.record(st)
        dp.mutation(s2, r2, g2)
        d.record(st)
        torch.cuda.synchronize()
        if rnd:
            times[n]["assign"].append(a.elapsed_time(b))
            times[n]["mutation"].append(c.elapsed_time(d))
        else:
            outs[n] = (r, s2, r2, g2)
for n in names:
    res["assign"][n] = round(float(np.median(times[n]["assign"])), 4)
    res["mutation"][n] = round(float(np.median(times[n]["mutation"])), 4)
    res["agree"][n] = all(bool(torch.equal(x, y)) for x, y in zip(outs[n], outs[names[0]]))
print(json.dumps(res))
