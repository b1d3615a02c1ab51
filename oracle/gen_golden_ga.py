"""Generate tests/golden/ga_ref.json — TEST INFRASTRUCTURE ONLY.

Expected outputs come from the reference's OWN ga.cpp and vendored jsoncpp
(oracle/_ref/libttref_ga.so, see oracle/Makefile `ref-ga`):

* `doubles`: jsoncpp's rendering of {"x": v} (writeString, indentation "");
* `logs`: the JSON lines of setCurrentCost / setGlobalCost / endTry and main's
  final runEntry (ga.cpp:169-257,603-609) for a given sequence of pop[0]
  members on the sm golden instance (times are wall-clock: the tests compare
  everything else byte for byte);
* `selection5`: ga.cpp:129-145 winners and the final Random state for seeded
  tournaments over penalties with ties;
* `sort`: std::sort(pop, pop + N, compareSolution) (ga.cpp:150-153,583).

    make -C oracle ref-ga && python oracle/gen_golden_ga.py
"""
from __future__ import annotations

import ctypes
import json
import pathlib
import sys

import numpy as np

REPO = pathlib.Path(__file__).resolve().parent.parent
sys.path.insert(0, str(REPO / "timetabling-ga-mpi-openmp_amd"))
sys.path.insert(0, str(REPO / "tests"))

import ttga  # noqa: E402

LIB = REPO / "oracle" / "_ref" / "libttref_ga.so"
OUT = REPO / "tests" / "golden" / "ga_ref.json"
DOUBLES = [0.0, 0.1, 0.5, 1.25, 3.0, 1e-7, 2.5e-5, 0.30000000000000004, 123456.789, 1234567890.123456, 1e21,
           1.7976931348623157e308, 5e-324, 42.000000000000007, 0.000123456789012345678, 7.77e-10, 86400.5]


def lib():
    L = ctypes.CDLL(str(LIB))
    vp, i32, lng = ctypes.c_void_p, ctypes.c_int, ctypes.c_long
    L.ref_problem_create.restype = vp
    L.ref_problem_create.argtypes = [i32, i32, i32, i32, vp, vp, vp, vp]
    L.refga_json_double.argtypes = [ctypes.c_double, ctypes.c_char_p, i32]
    L.refga_log_lines.argtypes = [vp, vp, vp, i32, vp, i32, i32, ctypes.c_char_p, i32]
    L.refga_selection5.argtypes = [vp, vp, i32, lng, i32, vp, ctypes.POINTER(lng)]
    L.refga_sort_penalties.argtypes = [vp, vp, i32]
    return L


def p(a):
    return a.ctypes.data_as(ctypes.c_void_p)


def main():
    L = lib()
    z = np.load(REPO / "tests" / "golden" / "sm.npz")
    E, R, F, S = (int(x) for x in z["dims"])
    inst = ttga.Instance(E, R, F, S, z["room_size"], z["student_events"], z["room_features"], z["event_features"])
    h = L.ref_problem_create(E, R, F, S, p(inst.room_size), p(inst.student_events), p(inst.room_features),
                             p(inst.event_features))
    out = {"instance": "sm", "doubles": []}
    buf = ctypes.create_string_buffer(1 << 20)
    for v in DOUBLES:
        L.refga_json_double(v, buf, len(buf))
        out["doubles"].append({"value": v.hex(), "line": buf.value.decode()})

    # pop[0] sequences: infeasible members (canonical rooms), then feasible ones
    # (the 2000-step local-search goldens); repeats and equal values included
    feas = [int(i) for i in np.nonzero(z["eval_ls3_feasible"])[0]]
    infe = [int(i) for i in np.nonzero(z["eval_canon_feasible"] == 0)[0]]
    assert len(feas) >= 3 and len(infe) >= 4
    order_inf = sorted(infe, key=lambda i: -int(z["eval_canon_hcv"][i]) * 1000000 - int(z["eval_canon_scv"][i]))
    feas_sorted = sorted(feas, key=lambda i: -int(z["eval_ls3_scv"][i]))
    runs = []
    seq_a = [("canon", order_inf[0], 0), ("canon", order_inf[0], 1), ("canon", order_inf[1], 2),
             ("canon", order_inf[-1], 0), ("ls3", feas_sorted[0], 3), ("ls3", feas_sorted[0], 1),
             ("ls3", feas_sorted[1], 2), ("ls3", feas_sorted[-1], 0)]
    seq_b = [("canon", order_inf[0], 0), ("canon", order_inf[2], 1), ("canon", order_inf[2], 1),
             ("canon", order_inf[-1], 4)]
    for seq, proc, threads in ((seq_a, 0, 4), (seq_b, 3, 5)):
        sl = np.stack([z[("slots" if t == "canon" else "ls3_slots")][i] for t, i, _ in seq]).astype(np.uint8)
        rm = np.stack([z[("rooms" if t == "canon" else "ls3_rooms")][i] for t, i, _ in seq]).astype(np.uint8)
        tids = np.array([t for _, _, t in seq], np.int32)
        n = L.refga_log_lines(h, p(sl), p(rm), len(seq), p(tids), proc, threads, buf, len(buf))
        assert n < len(buf)
        runs.append({"slots": sl.tolist(), "rooms": rm.tolist(), "tids": tids.tolist(), "proc": proc,
                     "threads": threads, "lines": buf.value.decode().splitlines()})
    out["logs"] = runs

    sel = []
    for N, seed, pen in ((10, 42, [5, 3, 3, 9, 1000004, 3, 7, 1, 1, 1000001]),
                         (37, 12345, [(i * 7919) % 13 for i in range(37)]),
                         (3, 2147483646, [2, 2, 1]), (64, 987654321, [1000000 + (i * 31) % 17 for i in range(64)])):
        pen = np.array(pen, np.int32)
        w = np.zeros(200, np.int32)
        st = ctypes.c_long(0)
        L.refga_selection5(h, p(pen), N, seed, 200, p(w), ctypes.byref(st))
        sel.append({"N": N, "seed": seed, "penalty": pen.tolist(), "winners": w.tolist(), "state": st.value})
    out["selection5"] = sel

    srt = []
    rng = np.random.default_rng(5)
    for N in (10, 33, 200):
        pen = rng.integers(0, 9, N).astype(np.int32)
        pen[::7] += 1000000
        got = pen.copy()
        L.refga_sort_penalties(h, p(got), N)
        srt.append({"penalty": pen.tolist(), "sorted": got.tolist()})
    out["sort"] = srt
    OUT.write_text(json.dumps(out, indent=1) + "\n")
    print(f"wrote {OUT}")


if __name__ == "__main__":
    main()
