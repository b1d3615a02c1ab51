"""Hardware counters for bench.py, collected live by child processes under
rocprofv3 (one --pmc pass per counter group, as MI355X_MICROARCH.md's
HBM/rocprofv3 section prescribes: FETCH_SIZE and WRITE_SIZE cannot share a
pass). Called BEFORE the parent touches the GPU; every pass runs under its own
hard time limit, and any failure leaves the counters unmeasured (None).

Per launch of the dominant kernel (median over its dispatches):
  traffic   = FETCH_SIZE * 2 (gfx950 reports half the bytes of a wide
              streaming read) + WRITE_SIZE, both in KiB -> bytes;
  lds_busy  = SQ_LDS_IDX_ACTIVE / (CUs * GRBM_GUI_ACTIVE / XCDs)  (LDS-array cycles)
  lds_conflict = SQ_LDS_BANK_CONFLICT / SQ_LDS_IDX_ACTIVE
  valu_busy = 2 * SQ_INSTS_VALU / (4 * CUs * GRBM_GUI_ACTIVE / XCDs)  (wave64 VALU = 2 cycles on a SIMD32)
  salu_busy = SQ_INSTS_SALU / (CUs * GRBM_GUI_ACTIVE / XCDs)      (one scalar unit per CU)
  wait_any  = SQ_WAIT_ANY / SQ_WAVE_CYCLES
"""
from __future__ import annotations

import collections
import csv
import glob
import os
import shutil
import statistics
import subprocess
import sys
import tempfile

PASSES = {
    "fetch": "FETCH_SIZE",
    "write": "WRITE_SIZE",
    "sq": "SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_LDS_IDX_ACTIVE SQ_LDS_BANK_CONFLICT SQ_WAVE_CYCLES "
          "SQ_WAIT_ANY SQ_BUSY_CYCLES GRBM_GUI_ACTIVE",
}
CUS, XCDS = 256, 8


def _median_counters(root: str, kernel: str) -> dict:
    """Median over dispatches of each counter (summed over its per-XCD/SE
    instances) per kernel whose name contains `kernel`, summed over those
    kernels (a step of the wide path launches two)."""
    per = collections.defaultdict(lambda: collections.defaultdict(float))
    for f in glob.glob(f"{root}/**/*counter_collection.csv", recursive=True):
        with open(f) as fh:
            for r in csv.DictReader(fh):
                if kernel not in r["Kernel_Name"]:
                    continue
                per[(r["Kernel_Name"], f, r["Dispatch_Id"])][r["Counter_Name"]] += float(r["Counter_Value"])
    vals = collections.defaultdict(lambda: collections.defaultdict(list))
    for (name, _, _), d in per.items():
        for c, v in d.items():
            vals[name][c].append(v)
    out = collections.defaultdict(float)
    for name, cs in vals.items():
        for c, v in cs.items():
            out[c] += statistics.median(v)
    return dict(out)


def collect(child_argv: list[str], kernel: str, timeout: int = 90) -> dict | None:
    """Runs `python <child_argv>` once per pass under rocprofv3 --pmc and
    returns the medians per launch of `kernel`, or None."""
    prof = shutil.which("rocprofv3")
    if prof is None:
        return None
    out: dict = {}
    env = dict(os.environ, TMPDIR="/tmp")
    with tempfile.TemporaryDirectory(prefix="ttga_pmc_", dir="/tmp") as tmp:
        for name, counters in PASSES.items():
            d = os.path.join(tmp, name)
            cmd = ["timeout", "-s", "KILL", str(timeout), prof, "--pmc", *counters.split(), "--output-format", "csv",
                   "-d", d, "-o", "pmc", "--", sys.executable, *child_argv]
            try:
                r = subprocess.run(cmd, capture_output=True, text=True, env=env, timeout=timeout + 30)
            except subprocess.TimeoutExpired:
                return None
            if r.returncode != 0:
                sys.stderr.write(f"pmc pass {name} failed (rc {r.returncode}): {r.stderr[-500:]}\n")
                return None
            out.update(_median_counters(d, kernel))
    return out


def derive(c: dict | None) -> dict | None:
    if not c or "FETCH_SIZE" not in c or "WRITE_SIZE" not in c:
        return None
    res = {"traffic_bytes": (2 * c["FETCH_SIZE"] + c["WRITE_SIZE"]) * 1024.0,
           "fetch_kib": c["FETCH_SIZE"], "write_kib": c["WRITE_SIZE"]}
    g = c.get("GRBM_GUI_ACTIVE")
    if g:
        cyc = g / XCDS                                     # shader cycles of the launch (per XCD)
        res["cycles"] = cyc
        if "SQ_LDS_IDX_ACTIVE" in c:
            res["lds_busy"] = c["SQ_LDS_IDX_ACTIVE"] / (CUS * cyc)
            res["lds_conflict"] = c.get("SQ_LDS_BANK_CONFLICT", 0.0) / max(c["SQ_LDS_IDX_ACTIVE"], 1.0)
        if "SQ_INSTS_VALU" in c:
            res["valu_busy"] = 2.0 * c["SQ_INSTS_VALU"] / (4 * CUS * cyc)
        if "SQ_INSTS_SALU" in c:
            res["salu_busy"] = c["SQ_INSTS_SALU"] / (CUS * cyc)
        if "SQ_WAIT_ANY" in c and c.get("SQ_WAVE_CYCLES"):
            res["wait_any"] = c["SQ_WAIT_ANY"] / c["SQ_WAVE_CYCLES"]
    res["raw"] = c
    return res
