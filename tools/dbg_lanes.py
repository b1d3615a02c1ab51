import pathlib, sys, json
REPO = pathlib.Path("/root/repo") if pathlib.Path("/root/repo").exists() else pathlib.Path(".")
sys.path.insert(0, str(REPO / "timetabling-ga-mpi-openmp_amd"))
import numpy as np, torch, ttga
from ttga import native
names = sys.argv[1:]
for cfg in ("med", "syn"):
    inst = ttga.config_instance(cfg)
    P = 256
    outs = {}
    for name in names:
        lib = native.load(REPO / "ab_libs" / f"libttga_{name}.so")
        saved, native._lib = native._lib, lib
        dp = native.DeviceProblem(inst)
        native._lib = saved
        seeds = torch.from_numpy(ttga.population_seeds(12345, P)).cuda()
        slot = torch.empty((P, inst.E), dtype=torch.uint8, device="cuda"); room = torch.empty_like(slot)
        dp.random_init(seeds, slot, room)
        outs[name] = [t.cpu().numpy() for t in dp.eval(slot, room, variant=13)] + [t.cpu().numpy() for t in dp.eval(slot, room, variant=2)]
    a, b = outs[names[0]], outs[names[1]]
    for k, what in enumerate(("hcv13", "scv13", "feas13", "pen13", "hcv2", "scv2", "feas2", "pen2")):
        d = a[k].astype(np.int64) - b[k].astype(np.int64)
        print(cfg, what, "mismatch", int((d != 0).sum()), "diff sample", d[:16].tolist())
    print(cfg, "scv13 new vs block", (b[1].astype(np.int64) - b[5]).tolist()[:32])
