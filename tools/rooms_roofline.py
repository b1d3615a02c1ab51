"""Roofline / issue line of the room assignment (tt_assign_rooms:
assign_rooms_kernel, Solution::assignRooms on every slot, Solution.cpp:772-891)
at the syn instance (BASELINE configs[4]: E 2000, R 40) and a comp instance.

The kernel moves E slot bytes in and E room bytes out per individual (4 KB at
syn) and does a long, lane-uniform search per slot, so HBM does not bound it:
the line reports, per launch, the HIP-event time, the algorithmic bytes and
their rate against 8 TB/s, and from hardware counters (rocprofv3 --pmc, one
process per pass, tools/ab_rooms.py as the workload, medians over its timed
launches) the issue rate per SIMD-cycle against 1, VALU / SALU busy, the
waves' wait share, instructions per individual and per slot, and the
HBM traffic (FETCH_SIZE / WRITE_SIZE) against the algorithmic bytes; beside
it assignRooms on the host cores (cpu_baseline: the reference's own objects,
or at syn the oracle's restatement).

    python tools/rooms_roofline.py [--config syn:65536 --config comp01:65536] [--lib tree] [--out x.jsonl]
"""
import argparse
import json
import os
import pathlib
import shutil
import subprocess
import sys
import tempfile

REPO = pathlib.Path(__file__).resolve().parent.parent
sys.path.insert(0, str(REPO / "tools"))
from ls_roofline import CUS, SIMDS, XCDS, last_medians  # noqa: E402

PASSES = {
    "insts": "SQ_INSTS SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_SMEM SQ_INSTS_VMEM SQ_WAVES GRBM_GUI_ACTIVE",
    "waits": "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_BUSY_CYCLES SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE "
             "SQ_ACTIVE_INST_VALU GRBM_GUI_ACTIVE",
    "fetch": "FETCH_SIZE GRBM_GUI_ACTIVE",
    "write": "WRITE_SIZE GRBM_GUI_ACTIVE",
}
KERNEL = "assign_rooms_kernel"
HBM_PEAK = 8.0e12


def collect(cfg: str, P: int, lib: str, timeout: int) -> dict:
    prof = shutil.which("rocprofv3")
    if prof is None:
        raise SystemExit("rocprofv3 not found")
    env = {k: v for k, v in os.environ.items() if not k.startswith("ROCPROF")}
    env["TMPDIR"] = "/tmp"
    out = {}
    with tempfile.TemporaryDirectory(prefix="ttga_roomroof_", dir="/tmp") as tmp:
        for name, counters in PASSES.items():
            d = os.path.join(tmp, name)
            cmd = ["timeout", "-s", "KILL", str(timeout), prof, "--pmc", *counters.split(), "--output-format", "csv",
                   "-d", d, "-o", "pmc", "--", sys.executable, str(REPO / "tools" / "ab_rooms.py"), cfg, str(P), lib]
            print(f"[rooms_roofline] {cfg} pass {name}", file=sys.stderr, flush=True)
            r = subprocess.run(cmd, capture_output=True, text=True, env=env, timeout=timeout + 30)
            if r.returncode != 0:
                raise SystemExit(f"pass {name} failed (rc {r.returncode}): {r.stderr[-800:]}")
            med, meta, n = last_medians(d, KERNEL, 10)
            if name == "insts":
                out["dispatches"], out["meta"] = n, meta
            out.update({k: v for k, v in med.items() if k != "GRBM_GUI_ACTIVE" or name == "insts"})
            out[f"cycles_{name}"] = med.get("GRBM_GUI_ACTIVE", 0.0) / XCDS
    return out


def timed(cfg: str, P: int, lib: str) -> dict:
    r = subprocess.run([sys.executable, str(REPO / "tools" / "ab_rooms.py"), cfg, str(P), lib],
                       capture_output=True, text=True, timeout=600)
    if r.returncode != 0:
        raise SystemExit(r.stderr[-800:])
    return json.loads(r.stdout[r.stdout.index("{"):])


def cpu_leg(inst, rows: int) -> dict | None:
    """assignRooms on `rows` random rows on the host cores: the reference's own
    objects (oracle/_ref) where building its Problem is quick, else the
    oracle's restatement (the reference parses syn's Problem for ~108 s)."""
    import time

    import numpy as np
    sys.path.insert(0, str(REPO / "tests"))
    from oracle_lib import host_threads, oracle, ref, split_rows
    kind, lib = ("reference", ref()) if inst.E <= 1000 else ("port", None)
    if lib is None:
        kind, lib = "port", oracle()
    if lib is None:
        return None
    h = lib.problem(inst)
    s = np.random.default_rng(5).integers(0, 45, size=(rows, inst.E), dtype=np.uint8)
    T = host_threads()
    t0 = time.perf_counter()
    split_rows(lambda x: (h.assign_rooms(x),), (s,), threads=T)
    dt = time.perf_counter() - t0
    return {"kind": kind, "cores": T, "rows": rows, "seconds": dt, "individuals_per_s": rows / dt}


def derive(c: dict, E: int, P: int, ms: float) -> dict:
    cyc = c["cycles_insts"]
    alg = 2.0 * E * P                                   # slot row in, room row out
    return {
        "kernel_ms": ms, "individuals_per_s": P / (ms * 1e-3),
        "algorithmic_bytes": alg, "achieved_GBps": alg / (ms * 1e-3) / 1e9,
        "hbm_frac": alg / (ms * 1e-3) / HBM_PEAK,
        "hbm_fetch_bytes": c.get("FETCH_SIZE", 0.0) * 1024.0, "hbm_write_bytes": c.get("WRITE_SIZE", 0.0) * 1024.0,
        "issue_per_simd_cycle": c["SQ_INSTS"] / (SIMDS * cyc), "issue_ceiling": 1.0,
        "valu_busy": 4.0 * c["SQ_INSTS_VALU"] / (4 * CUS * cyc),
        "salu_busy": c["SQ_INSTS_SALU"] / (CUS * cyc),
        "wait_share": c.get("SQ_WAIT_ANY", 0.0) / max(c.get("SQ_WAVE_CYCLES", 1.0), 1.0),
        "active_share": c.get("SQ_ACTIVE_INST_ANY", 0.0) / max(c.get("SQ_WAVE_CYCLES", 1.0), 1.0),
        "lds_conflict_share": c.get("SQ_LDS_BANK_CONFLICT", 0.0) / max(c.get("SQ_LDS_IDX_ACTIVE", 1.0), 1.0),
        "insts_per_individual": {k: c[k] / P for k in ("SQ_INSTS", "SQ_INSTS_VALU", "SQ_INSTS_SALU", "SQ_INSTS_LDS",
                                                       "SQ_INSTS_SMEM", "SQ_INSTS_VMEM") if k in c},
        "insts_per_slot": c["SQ_INSTS"] / (45.0 * P),
        "waves": c.get("SQ_WAVES"), "cycles_per_launch": cyc,
    }


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", action="append", default=None, help="instance:P")
    ap.add_argument("--lib", default="tree", help="tree (the in-tree library) or ab_libs/libttga_<lib>.so")
    ap.add_argument("--timeout", type=int, default=180)
    ap.add_argument("--cpu-rows", type=int, default=0, help="rows of the CPU leg (0: 512 at syn, else 4096)")
    ap.add_argument("--out", default=None)
    a = ap.parse_args()
    sys.path.insert(0, str(REPO / "timetabling-ga-mpi-openmp_amd"))
    import ttga
    recs = []
    for spec in a.config or ["syn:65536", "comp01:65536"]:
        cfg, P = spec.split(":")[0], int(spec.split(":")[1])
        inst = ttga.config_instance(cfg)
        t = timed(cfg, P, a.lib)
        c = collect(cfg, P, a.lib, a.timeout)
        rec = {"config": cfg, "E": inst.E, "R": inst.R, "P": P, "lib": a.lib, "kernel": KERNEL,
               "mutation_ms": t["mutation"][a.lib], "line": derive(c, inst.E, P, t["assign"][a.lib]),
               "cpu_baseline": cpu_leg(inst, a.cpu_rows or (512 if inst.E > 1000 else 4096)),
               "meta": c.pop("meta", {}), "raw": c}
        recs.append(rec)
        print(json.dumps(rec), flush=True)
    if a.out:
        pathlib.Path(a.out).write_text("".join(json.dumps(r) + "\n" for r in recs))


if __name__ == "__main__":
    main()
