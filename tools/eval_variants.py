"""Eval-kernel variants side by side (profiling only): every variant must agree
bit for bit with the workgroup-per-individual kernel; then interleaved timing
with HIP events on the launch stream, median over rounds."""
import json
import pathlib
import sys

REPO = pathlib.Path(__file__).resolve().parent.parent
sys.path.insert(0, str(REPO / "timetabling-ga-mpi-openmp_amd"))
import numpy as np  # noqa: E402
import torch  # noqa: E402

import ttga  # noqa: E402
from ttga import native  # noqa: E402

cfg = sys.argv[1] if len(sys.argv) > 1 else "med"
P = int(sys.argv[2]) if len(sys.argv) > 2 else 65536
variants = [int(v) for v in sys.argv[3].split(",")] if len(sys.argv) > 3 else [8, 7, 13]
inst = ttga.config_instance(cfg)
dp = native.DeviceProblem(inst)
seeds = torch.from_numpy(ttga.population_seeds(12345, P)).cuda()
slot = torch.empty((P, inst.E), dtype=torch.uint8, device="cuda")
room = torch.empty_like(slot)
dp.random_init(seeds, slot, room)
ref = [t.clone() for t in dp.eval(slot, room, variant=2)]
res = {"config": cfg, "P": P, "agree": {}, "ms_median": {}}
for v in variants:
    # ablated (profiling-only) launches give invalid results
    if v >> 4:
        continue
    got = dp.eval(slot, room, variant=v)
    res["agree"][v] = all(bool(torch.equal(a, b)) for a, b in zip(got, ref))
st = torch.cuda.current_stream()
times = {v: [] for v in variants}
for rnd in range(15):
    for v in variants:
        out = dp.eval(slot, room, variant=v)
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record(st)
        for _ in range(10):
            dp.eval(slot, room, variant=v, out=out)
        b.record(st)
        torch.cuda.synchronize()
        times[v].append(a.elapsed_time(b) / 10)
res["ms_median"] = {v: float(np.median(t)) for v, t in times.items()}
res["evals_per_s"] = {v: P / (t * 1e-3) for v, t in res["ms_median"].items()}
print(json.dumps(res))
