"""Roofline / issue line of the GA children's local search (the kernel that
takes 80-94 % of a GA generation): hardware counters of the steady window's
`local_search_kernel` launches plus the wave-slot occupancy from per-wave
stamps, as one JSON record per instance.

The same GA workload as tools/bench_ga.py (one island, 65,536 members, 8,192
children per generation, maxSteps 1000, warm-up to 60 % feasible) runs under
`rocprofv3 --pmc` once per counter pass (each pass a process of its own, as
MI355X_MICROARCH.md prescribes: at most 8 SQ counters, FETCH_SIZE and
WRITE_SIZE in passes of their own); the medians over the last 10 launches of
the kernel give, per launch:

* issue: all instructions issued (SQ_INSTS) per SIMD-cycle, against the
  ceiling of 1 (one instruction per SIMD per cycle);
* VALU busy (4 cycles per wave64 VALU instruction per SIMD, tools/valu_rate)
  and SALU busy (one scalar unit per CU, one instruction per cycle), the LDS
  array's busy share and its bank-conflict share, the waves' wait share;
* scratch: bytes per lane of the kernel's private segment (the code
  object's, from the counter CSV), and the HBM writes of the launch
  (WRITE_SIZE) against the algorithmic writes (slot and room rows, RNG
  states: 2E + 8 B per child), whose excess bounds the scratch traffic that
  left the caches;
* slot_busy: tools/ls_tail.py's stamps (profiling build): the busy share of
  the launch's wave slots over its span.

    python tools/ls_roofline.py --config comp15 [--config comp01 ...] [--out profiles/x.json]
"""
import argparse
import collections
import csv
import glob
import json
import os
import pathlib
import shutil
import statistics
import subprocess
import sys
import tempfile

REPO = pathlib.Path(__file__).resolve().parent.parent
CUS, SIMDS, XCDS = 256, 1024, 8
PASSES = {
    "insts": "SQ_INSTS SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_SMEM SQ_INSTS_FLAT SQ_INSTS_VMEM SQ_WAVES "
             "GRBM_GUI_ACTIVE",
    "waits": "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_BUSY_CYCLES SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE "
             "SQ_INSTS_BRANCH SQ_ACTIVE_INST_VALU GRBM_GUI_ACTIVE",
    "write": "WRITE_SIZE GRBM_GUI_ACTIVE",
    "fetch": "FETCH_SIZE GRBM_GUI_ACTIVE",
}
KERNEL = "local_search_kernel"


def ga_child(cfg: str, children: int, gens: int) -> list:
    return [str(REPO / "tools" / "bench_ga.py"), "--config", cfg, "--pop", "65536", "--children", str(children),
            "--steps", "1000", "--warm-gens", "96", "--warm-feasible", "0.6", "--gens", str(gens), "--cpu-sample", "0"]


def last_medians(root: str, kernel: str, last: int):
    """Per counter: the median over the last `last` dispatches of `kernel` (each
    dispatch's value summed over its XCD / SE instances); plus the kernel
    metadata of those dispatches."""
    per = collections.defaultdict(lambda: collections.defaultdict(float))
    meta = {}
    for f in glob.glob(f"{root}/**/*counter_collection.csv", recursive=True):
        with open(f) as fh:
            for r in csv.DictReader(fh):
                if kernel not in r["Kernel_Name"] or "redo" in r["Kernel_Name"]:
                    continue
                per[int(r["Dispatch_Id"])][r["Counter_Name"]] += float(r["Counter_Value"])
                meta[int(r["Dispatch_Id"])] = {k: r.get(k) for k in ("Kernel_Name", "Grid_Size", "Workgroup_Size",
                                                                     "LDS_Block_Size", "VGPR_Count", "SGPR_Count",
                                                                     "Scratch_Size")}
    ids = sorted(per)[-last:]
    vals = collections.defaultdict(list)
    for i in ids:
        for c, v in per[i].items():
            vals[c].append(v)
    return {c: statistics.median(v) for c, v in vals.items()}, (meta[ids[-1]] if ids else {}), len(ids)


def collect(cfg: str, children: int, gens: int, last: int, timeout: int) -> dict:
    prof = shutil.which("rocprofv3")
    if prof is None:
        raise SystemExit("rocprofv3 not found")
    env = {k: v for k, v in os.environ.items() if not k.startswith("ROCPROF")}
    env["TMPDIR"] = "/tmp"
    out, meta = {}, {}
    with tempfile.TemporaryDirectory(prefix="ttga_lsroof_", dir="/tmp") as tmp:
        for name, counters in PASSES.items():
            d = os.path.join(tmp, name)
            cmd = ["timeout", "-s", "KILL", str(timeout), prof, "--pmc", *counters.split(), "--output-format", "csv",
                   "-d", d, "-o", "pmc", "--", sys.executable, *ga_child(cfg, children, gens)]
            print(f"[ls_roofline] {cfg} pass {name}", file=sys.stderr, flush=True)
            r = subprocess.run(cmd, capture_output=True, text=True, env=env, timeout=timeout + 30)
            if r.returncode != 0:
                raise SystemExit(f"pass {name} failed (rc {r.returncode}): {r.stderr[-800:]}")
            med, m, n = last_medians(d, KERNEL, last)
            if name == "insts":
                meta, out["dispatches"] = m, n
            out.update({k: v for k, v in med.items() if k != "GRBM_GUI_ACTIVE" or name == "insts"})
            out[f"cycles_{name}"] = med.get("GRBM_GUI_ACTIVE", 0.0) / XCDS
    return out, meta


def derive(c: dict, meta: dict, E: int, children: int) -> dict:
    cyc = c["cycles_insts"]                          # shader cycles of one launch (per XCD)
    alg_write = children * (2 * E + 8)
    wr = c.get("WRITE_SIZE", 0.0) * 1024.0
    res = {
        "issue_per_simd_cycle": c["SQ_INSTS"] / (SIMDS * cyc), "issue_ceiling": 1.0,
        "valu_busy": 4.0 * c["SQ_INSTS_VALU"] / (4 * CUS * cyc),
        "salu_busy": c["SQ_INSTS_SALU"] / (CUS * cyc),
        "lds_busy": c.get("SQ_LDS_IDX_ACTIVE", 0.0) / (CUS * c["cycles_waits"]) if c.get("cycles_waits") else None,
        "lds_conflict_share": c.get("SQ_LDS_BANK_CONFLICT", 0.0) / max(c.get("SQ_LDS_IDX_ACTIVE", 1.0), 1.0),
        "wait_share": c.get("SQ_WAIT_ANY", 0.0) / max(c.get("SQ_WAVE_CYCLES", 1.0), 1.0),
        "active_share": c.get("SQ_ACTIVE_INST_ANY", 0.0) / max(c.get("SQ_WAVE_CYCLES", 1.0), 1.0),
        "per_wave": {k: c[k] / max(c.get("SQ_WAVES", 1.0), 1.0) for k in
                     ("SQ_INSTS", "SQ_INSTS_VALU", "SQ_INSTS_SALU", "SQ_INSTS_LDS", "SQ_INSTS_SMEM", "SQ_INSTS_FLAT",
                      "SQ_INSTS_VMEM") if k in c},
        "scratch_bytes_per_lane": int(meta.get("Scratch_Size") or 0),
        "vgprs": meta.get("VGPR_Count"), "sgprs": meta.get("SGPR_Count"), "lds_bytes": meta.get("LDS_Block_Size"),
        "hbm_write_bytes": wr, "algorithmic_write_bytes": alg_write,
        "hbm_write_excess_bytes": wr - alg_write,
        "hbm_fetch_bytes_raw": c.get("FETCH_SIZE", 0.0) * 1024.0,
        "cycles_per_launch": cyc, "waves": c.get("SQ_WAVES"),
    }
    return res


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", action="append", default=None)
    ap.add_argument("--children", type=int, default=8192)
    ap.add_argument("--gens", type=int, default=12)
    ap.add_argument("--last", type=int, default=10)
    ap.add_argument("--timeout", type=int, default=240)
    ap.add_argument("--no-stamps", action="store_true")
    ap.add_argument("--out", default=None)
    a = ap.parse_args()
    sys.path.insert(0, str(REPO / "timetabling-ga-mpi-openmp_amd"))
    import ttga
    recs = []
    for cfg in a.config or ["comp01", "comp10", "comp15"]:
        E = ttga.config_instance(cfg).E
        c, meta = collect(cfg, a.children, a.gens, a.last, a.timeout)
        rec = {"config": cfg, "children": a.children, "kernel": meta.get("Kernel_Name", "")[:80],
               "dispatches_used": c.get("dispatches"), "line": derive(c, meta, E, a.children), "raw": c}
        if not a.no_stamps:
            lib = REPO / "timetabling-ga-mpi-openmp_amd" / "libttga_prof.so"
            if lib.exists():
                print(f"[ls_roofline] {cfg} stamps", file=sys.stderr, flush=True)
                r = subprocess.run(["timeout", "-k", "10", str(a.timeout), sys.executable,
                                    str(REPO / "tools" / "ls_tail.py"), "--config", cfg, "--children",
                                    str(a.children)], capture_output=True, text=True)
                if r.returncode == 0:
                    t = json.loads(r.stdout[r.stdout.index("{"):])
                    rec["line"]["slot_busy"] = t.get("slot_busy")
                    rec["stamps"] = {k: t.get(k) for k in ("span_us", "slot_busy", "peak_waves", "max_wave_us",
                                                            "mean_wave_us") if k in t}
                else:
                    rec["stamps_error"] = r.stderr[-400:]
        recs.append(rec)
        print(json.dumps(rec), flush=True)
    if a.out:
        pathlib.Path(a.out).write_text("".join(json.dumps(r) + "\n" for r in recs))


if __name__ == "__main__":
    main()
