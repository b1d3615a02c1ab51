"""Start-up cost of the Problem image (Problem.cpp:3-96).

Times, per configuration: the .tim parse (ttga.instance.read_tim), the whole
tt_problem_create (host CSR views + upload, and the device derivation of
studentNumber / eventCorrelations / possibleRooms: csrc/tt_derive.hip, the int8
MFMA contraction; its kernel times come from a kernel trace of this script),
the CPU oracle's student-major restatement of the derivation (O(sum of deg^2),
the form the library used on the host before round 4), and, where oracle/_ref
is present, the reference's own Problem(istream&) (its eventCorrelations
triple loop is O(E^2 S): 108 s at syn in the survey).

    python tools/time_problem.py [out.json] [repeats] [configs, comma-separated]
"""
from __future__ import annotations

import ctypes
import json
import pathlib
import sys
import tempfile
import time

REPO = pathlib.Path(__file__).resolve().parent.parent
sys.path[:0] = [str(REPO / "timetabling-ga-mpi-openmp_amd"), str(REPO / "tests")]

import ttga  # noqa: E402
from ttga import native  # noqa: E402


def main():
    out = {}
    reps = int(sys.argv[2]) if len(sys.argv) > 2 else 1
    native.DeviceProblem(ttga.config_instance("sm"))           # HIP initialisation, not timed
    from oracle_lib import oracle, ref
    O = oracle()
    R = ref()
    names = sys.argv[3].split(",") if len(sys.argv) > 3 else ["med", "lg", "comp01", "syn"]
    for name in names:
        inst = ttga.config_instance(name)
        with tempfile.TemporaryDirectory() as d:
            path = pathlib.Path(d) / f"{name}.tim"
            ttga.write_tim(inst, path)
            t = time.perf_counter()
            inst2 = ttga.read_tim(path)
            parse = time.perf_counter() - t
            times = []
            for _ in range(reps):
                t = time.perf_counter()
                dp = native.DeviceProblem(inst2)
                times.append(time.perf_counter() - t)
                if len(times) < reps:
                    dp.close()
            t = time.perf_counter()
            oh = O.problem(inst)
            odr = time.perf_counter() - t
            del oh
            row = {"E": inst.E, "R": inst.R, "F": inst.F, "S": inst.S, "parse_s": parse,
                   "tt_problem_create_s": min(times), "tt_problem_create_runs": len(times),
                   "oracle_host_derive_s": odr}
            if R is not None and inst.E * inst.E * inst.S <= 4e9:   # the reference's O(E^2 S) build (syn: ~2 min)
                t = time.perf_counter()
                h = R.problem(inst)
                row["reference_problem_s"] = time.perf_counter() - t
                del h
            del dp
        out[name] = row
        print(name, json.dumps(row), flush=True)
    if len(sys.argv) > 1:
        pathlib.Path(sys.argv[1]).write_text(json.dumps(out, indent=1) + "\n")


if __name__ == "__main__":
    main()
