"""Per-phase timing of the tile eval kernel (profiling only): interleaved
rounds in one process, HIP-event timing on the launch stream, median of N."""
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
inst = ttga.config_instance(cfg)
dp = native.DeviceProblem(inst)
seeds = torch.from_numpy(ttga.population_seeds(12345, P)).cuda()
slot = torch.empty((P, inst.E), dtype=torch.uint8, device="cuda")
room = torch.empty_like(slot)
dp.random_init(seeds, slot, room)
out = dp.eval(slot, room)
variants = {"full": 1, "no_lane": 1 | 16, "no_wave": 1 | 32, "no_corr": 1 | 64, "stage_only": 1 | 48,
            "block": 2}
times = {k: [] for k in variants}
st = torch.cuda.current_stream()
for rnd in range(15):
    for k, v in variants.items():
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record(st)
        for _ in range(10):
            dp.eval(slot, room, variant=v, out=out)
        b.record(st)
        torch.cuda.synchronize()
        times[k].append(a.elapsed_time(b) / 10)
res = {k: float(np.median(v)) for k, v in times.items()}
print(json.dumps({"config": cfg, "P": P, "ms_median": res}))
