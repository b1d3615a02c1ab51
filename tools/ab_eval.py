"""Same-box A/B timing of tt_eval builds (profiling only; tools/ab_build.sh
makes the libraries): every spec `lib:variant` must agree bit for bit with the
first; then interleaved timing with HIP events on the launch stream, median
over rounds.

    python tools/ab_eval.py med 65536 head:8 w1:8 w1:1032
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
specs = sys.argv[3:]
inst = ttga.config_instance(cfg)
probs = {}
for sp in specs:
    name = sp.split(":")[0]
    if name not in probs:
        lib = native.load(REPO / "ab_libs" / f"libttga_{name}.so")
        saved, native._lib = native._lib, lib
        probs[name] = native.DeviceProblem(inst)
        native._lib = saved
first = probs[specs[0].split(":")[0]]
seeds = torch.from_numpy(ttga.population_seeds(12345, P)).cuda()
slot = torch.empty((P, inst.E), dtype=torch.uint8, device="cuda")
room = torch.empty_like(slot)
first.random_init(seeds, slot, room)
ref = [t.clone() for t in first.eval(slot, room, variant=int(specs[0].split(":")[1]))]
res = {"config": cfg, "P": P, "agree": {}, "ms_median": {}}
for sp in specs:
    name, v = sp.split(":")
    got = probs[name].eval(slot, room, variant=int(v))
    res["agree"][sp] = all(bool(torch.equal(a, b)) for a, b in zip(got, ref))
st = torch.cuda.current_stream()
times = {sp: [] for sp in specs}
for rnd in range(21):
    for sp in specs:
        name, v = sp.split(":")
        dp, v = probs[name], int(v)
        out = dp.eval(slot, room, variant=v)
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record(st)
        for _ in range(10):
            dp.eval(slot, room, variant=v, out=out)
        b.record(st)
        torch.cuda.synchronize()
        times[sp].append(a.elapsed_time(b) / 10)
res["ms_median"] = {sp: round(float(np.median(t)), 5) for sp, t in times.items()}
print(json.dumps(res))
