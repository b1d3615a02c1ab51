"""Hardware counters for bench.py, collected live by child processes under
rocprofv3 (one --pmc pass per counter group, as MI355X_MICROARCH.md's
HBM/rocprofv3 section prescribes: FETCH_SIZE and WRITE_SIZE cannot share a
pass). Called BEFORE the parent touches the GPU; every pass runs under its own
hard time limit, and any failure leaves the counters unmeasured (None).

Per launch of the dominant kernel (median over its dispatches):
  traffic   = FETCH_SIZE * k + WRITE_SIZE, both in KiB -> bytes, where the
              read factor k is CALIBRATED in the same run: a fourth pass runs
              the same kernel with its evaluation phases switched off
              (tt_eval_variant profiling bits: only the population rows are
              staged, exactly P*E bytes by the kernel's own load
              instructions), k = P*E / FETCH_SIZE of that pass. The raw
              FETCH_SIZE / WRITE_SIZE and k are reported next to the traffic
              (MI355X_MICROARCH.md: FETCH_SIZE reads half the bytes of a wide
              streaming read on gfx950; other widths are uncalibrated);
  lds_busy  = SQ_LDS_IDX_ACTIVE / (CUs * GRBM_GUI_ACTIVE / XCDs)  (LDS-array cycles)
  lds_conflict = SQ_LDS_BANK_CONFLICT / SQ_LDS_IDX_ACTIVE
  valu_busy = 4 * SQ_INSTS_VALU / (4 * CUs * GRBM_GUI_ACTIVE / XCDs)  (a wave64 VALU instruction
              occupies its SIMD 4 cycles: tools/valu_rate measured 0.88-0.95
              wave-instructions per CU-cycle for 32- and 64-bit opcodes; until
              round 4 this used 2 cycles and reported half the busy fraction)
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


def under_profiler() -> bool:
    """True inside a rocprofv3 run (it exports ROCPROF* variables): the live
    passes would start a profiler from a profiled, GPU-initialised process,
    so the caller skips them."""
    return any(k.startswith("ROCPROF") for k in os.environ)


def _pass(prof, counters, child_argv, kernel, tmp, name, timeout):
    d = os.path.join(tmp, name)
    # the child gets this environment minus any profiler settings of our own
    env = {k: v for k, v in os.environ.items() if not k.startswith("ROCPROF")}
    env["TMPDIR"] = "/tmp"
    cmd = ["timeout", "-s", "KILL", str(timeout), prof, "--pmc", *counters.split(), "--output-format", "csv",
           "-d", d, "-o", "pmc", "--", sys.executable, *child_argv]
    try:
        r = subprocess.run(cmd, capture_output=True, text=True, env=env, timeout=timeout + 30)
    except subprocess.TimeoutExpired:
        return None
    if r.returncode != 0:
        sys.stderr.write(f"pmc pass {name} failed (rc {r.returncode}): {r.stderr[-500:]}\n")
        return None
    return _median_counters(d, kernel)


def collect(child_argv: list[str], kernel: str, calib_argv: list[str] | None = None,
            timeout: int = 90) -> dict | None:
    """Runs `python <child_argv>` once per pass under rocprofv3 --pmc and
    returns the medians per launch of `kernel`, or None. calib_argv: the
    calibration child (FETCH_SIZE only), whose values come back prefixed
    CAL_."""
    prof = shutil.which("rocprofv3")
    if prof is None or under_profiler():
        return None
    out: dict = {}
    with tempfile.TemporaryDirectory(prefix="ttga_pmc_", dir="/tmp") as tmp:
        for name, counters in PASSES.items():
            got = _pass(prof, counters, child_argv, kernel, tmp, name, timeout)
            if got is None:
                return None
            out.update(got)
        if calib_argv:
            got = _pass(prof, PASSES["fetch"], calib_argv, kernel, tmp, "calib", timeout)
            if got:
                out.update({"CAL_" + k: v for k, v in got.items()})
    return out


def derive(c: dict | None, calib_bytes: float | None = None) -> dict | None:
    """calib_bytes: the bytes the calibration launch reads (P*E)."""
    if not c or "FETCH_SIZE" not in c or "WRITE_SIZE" not in c:
        return None
    k, how = 2.0, "factor 2 from MI355X_MICROARCH.md (calibration pass missing)"
    cal = c.get("CAL_FETCH_SIZE")
    if calib_bytes and cal:
        k, how = calib_bytes / (cal * 1024.0), "calibrated: population rows only, P*E bytes / FETCH_SIZE"
    res = {"traffic_bytes": (k * c["FETCH_SIZE"] + c["WRITE_SIZE"]) * 1024.0,
           "fetch_kib": c["FETCH_SIZE"], "write_kib": c["WRITE_SIZE"], "fetch_factor": k, "fetch_factor_how": how,
           "calib_fetch_kib": cal, "calib_bytes": calib_bytes}
    g = c.get("GRBM_GUI_ACTIVE")
    if g:
        cyc = g / XCDS                                     # shader cycles of the launch (per XCD)
        res["cycles"] = cyc
        if "SQ_LDS_IDX_ACTIVE" in c:
            res["lds_busy"] = c["SQ_LDS_IDX_ACTIVE"] / (CUS * cyc)
            res["lds_conflict"] = c.get("SQ_LDS_BANK_CONFLICT", 0.0) / max(c["SQ_LDS_IDX_ACTIVE"], 1.0)
        if "SQ_INSTS_VALU" in c:
            res["valu_busy"] = 4.0 * c["SQ_INSTS_VALU"] / (4 * CUS * cyc)
        if "SQ_INSTS_SALU" in c:
            res["salu_busy"] = c["SQ_INSTS_SALU"] / (CUS * cyc)
        if "SQ_WAIT_ANY" in c and c.get("SQ_WAVE_CYCLES"):
            res["wait_any"] = c["SQ_WAIT_ANY"] / c["SQ_WAVE_CYCLES"]
    res["raw"] = c
    return res
