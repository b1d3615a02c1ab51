"""ctypes access to the CPU checkers — TEST INFRASTRUCTURE ONLY.

* `Oracle`  -> oracle/libttoracle.so, the clean-room CPU restatement
* `Ref`     -> oracle/_ref/libttref.so, the reference's own Problem/Solution
              objects compiled unmodified (present only where /root/reference
              was available at build time; it travels with the snapshot)

Both expose the same batched API over numpy arrays so tests can run either.
"""
from __future__ import annotations

import ctypes
import os
import pathlib
from concurrent.futures import ThreadPoolExecutor

import numpy as np

REPO = pathlib.Path(__file__).resolve().parent.parent
ORACLE_PATH = REPO / "oracle" / "libttoracle.so"
REF_PATH = REPO / "oracle" / "_ref" / "libttref.so"

_vp = ctypes.c_void_p


def _p(a):
    return a.ctypes.data_as(_vp)


class _Checker:
    prefix = ""

    def __init__(self, path):
        self.lib = ctypes.CDLL(str(path))
        pre = self.prefix
        L = self.lib
        i32, dbl, lng = ctypes.c_int, ctypes.c_double, ctypes.c_long
        getattr(L, pre + "problem_create").restype = _vp
        getattr(L, pre + "problem_create").argtypes = [i32, i32, i32, i32, _vp, _vp, _vp, _vp]
        getattr(L, pre + "problem_destroy").argtypes = [_vp]
        getattr(L, pre + "problem_derived").argtypes = [_vp, _vp, _vp, _vp]
        getattr(L, pre + "rand").argtypes = [lng, i32, _vp, _vp]
        getattr(L, pre + "eval").argtypes = [_vp, _vp, _vp, i32, _vp, _vp, _vp, _vp]
        getattr(L, pre + "assign_rooms").argtypes = [_vp, _vp, _vp, i32]
        getattr(L, pre + "random_init").argtypes = [_vp, _vp, _vp, _vp, i32]
        getattr(L, pre + "local_search").argtypes = [_vp, _vp, _vp, _vp, i32, i32, dbl, dbl, dbl]
        getattr(L, pre + "crossover").argtypes = [_vp, _vp, _vp, _vp, _vp, _vp, i32]
        getattr(L, pre + "mutation").argtypes = [_vp, _vp, _vp, _vp, i32]
        if hasattr(L, pre + "ga_breed"):
            getattr(L, pre + "ga_breed").argtypes = [_vp, _vp, _vp, _vp, i32, _vp, i32, dbl, dbl, i32, _vp, _vp, _vp]
            getattr(L, pre + "ga_replace").argtypes = [_vp] + [_vp] * 6 + [i32] + [_vp] * 6 + [i32]

    def _f(self, name):
        return getattr(self.lib, self.prefix + name)

    def problem(self, inst):
        h = self._f("problem_create")(inst.E, inst.R, inst.F, inst.S, _p(inst.room_size), _p(inst.student_events),
                                      _p(inst.room_features), _p(inst.event_features))
        return _Handle(self, h, inst)

    def rand(self, seed: int, n: int):
        out = np.zeros(n, np.float64)
        st = ctypes.c_long(0)
        self._f("rand")(int(seed), n, _p(out), ctypes.byref(st))
        return out, int(st.value)


class _Handle:
    def __init__(self, checker, h, inst):
        self.c, self.h, self.inst = checker, h, inst
        self.E, self.R = inst.E, inst.R

    def __del__(self):
        try:
            self.c._f("problem_destroy")(self.h)
        except Exception:
            pass

    def derived(self):
        E, R = self.E, self.R
        sn = np.zeros(E, np.int32)
        corr = np.zeros((E, E), np.int32)
        poss = np.zeros((E, R), np.int32)
        self.c._f("problem_derived")(self.h, _p(sn), _p(corr), _p(poss))
        return sn, corr, poss

    def eval(self, slot, room):
        slot = np.ascontiguousarray(slot, np.uint8)
        room = np.ascontiguousarray(room, np.uint8)
        P = slot.shape[0]
        hcv = np.zeros(P, np.int32); scv = np.zeros(P, np.int32)
        feas = np.zeros(P, np.uint8); pen = np.zeros(P, np.int32)
        self.c._f("eval")(self.h, _p(slot), _p(room), P, _p(hcv), _p(scv), _p(feas), _p(pen))
        return hcv, scv, feas, pen

    def assign_rooms(self, slot):
        slot = np.ascontiguousarray(slot, np.uint8)
        room = np.zeros_like(slot)
        self.c._f("assign_rooms")(self.h, _p(slot), _p(room), slot.shape[0])
        return room

    def random_init(self, seeds):
        rng = np.ascontiguousarray(seeds, np.int64).copy()
        P = rng.size
        slot = np.zeros((P, self.E), np.uint8); room = np.zeros((P, self.E), np.uint8)
        self.c._f("random_init")(self.h, _p(rng), _p(slot), _p(room), P)
        return slot, room, rng

    def local_search(self, slot, room, seeds, max_steps, p1=1.0, p2=1.0, p3=0.0):
        slot = np.ascontiguousarray(slot, np.uint8).copy()
        room = np.ascontiguousarray(room, np.uint8).copy()
        rng = np.ascontiguousarray(seeds, np.int64).copy()
        self.c._f("local_search")(self.h, _p(slot), _p(room), _p(rng), slot.shape[0], int(max_steps),
                                  float(p1), float(p2), float(p3))
        return slot, room, rng

    def crossover(self, s1, s2, seeds):
        s1 = np.ascontiguousarray(s1, np.uint8); s2 = np.ascontiguousarray(s2, np.uint8)
        rng = np.ascontiguousarray(seeds, np.int64).copy()
        slot = np.zeros_like(s1); room = np.zeros_like(s1)
        self.c._f("crossover")(self.h, _p(s1), _p(s2), _p(rng), _p(slot), _p(room), s1.shape[0])
        return slot, room, rng

    def mutation(self, slot, room, seeds):
        slot = np.ascontiguousarray(slot, np.uint8).copy()
        room = np.ascontiguousarray(room, np.uint8).copy()
        rng = np.ascontiguousarray(seeds, np.int64).copy()
        self.c._f("mutation")(self.h, _p(slot), _p(room), _p(rng), slot.shape[0])
        return slot, room, rng


def _ga_breed(self, pop_slot, pop_room, pen, seeds, C, p_cross=0.8, p_mut=0.5, skip_init=1):
    pop_slot = np.ascontiguousarray(pop_slot, np.uint8); pop_room = np.ascontiguousarray(pop_room, np.uint8)
    pen = np.ascontiguousarray(pen, np.int32)
    rng = np.ascontiguousarray(seeds, np.int64).copy()
    cs = np.zeros((C, self.E), np.uint8); cr = np.zeros((C, self.E), np.uint8); fl = np.zeros(C, np.uint8)
    self.c._f("ga_breed")(self.h, _p(pop_slot), _p(pop_room), _p(pen), pop_slot.shape[0], _p(rng), C,
                          float(p_cross), float(p_mut), int(skip_init), _p(cs), _p(cr), _p(fl))
    return cs, cr, fl, rng


def _ga_replace(self, pop, child):
    """pop/child: dicts with slot, room, hcv, scv, feasible, penalty (numpy); returns the new pop."""
    out = {k: np.ascontiguousarray(v).copy() for k, v in pop.items()}
    ch = {k: np.ascontiguousarray(v) for k, v in child.items()}
    N, C = out["slot"].shape[0], ch["slot"].shape[0]
    self.c._f("ga_replace")(self.h, _p(out["slot"]), _p(out["room"]), _p(out["hcv"]), _p(out["scv"]),
                            _p(out["feasible"]), _p(out["penalty"]), N, _p(ch["slot"]), _p(ch["room"]),
                            _p(ch["hcv"]), _p(ch["scv"]), _p(ch["feasible"]), _p(ch["penalty"]), C)
    return out


_Handle.ga_breed = _ga_breed
_Handle.ga_replace = _ga_replace


class Oracle(_Checker):
    prefix = "tto_"


class Ref(_Checker):
    prefix = "ref_"


def oracle():
    if not ORACLE_PATH.exists():
        raise FileNotFoundError(f"{ORACLE_PATH} missing: run `make -C oracle oracle`")
    return Oracle(ORACLE_PATH)


def ref():
    """The reference build, or None where it was never built (no /root/reference)."""
    return Ref(REF_PATH) if REF_PATH.exists() else None


def _ga_run(self, seeds, pop_size=10, gens=2001, max_steps=200, as_is=1, threads=1):
    """ref_ga_run: whole single-island reference GA runs, one per seed (Ref only).
    Returns (hcv, scv, feasible, penalty, trace[runs, gens+1], seconds)."""
    seeds = np.ascontiguousarray(seeds, np.int64)
    n = seeds.size
    hcv = np.zeros(n, np.int32); scv = np.zeros(n, np.int32)
    feas = np.zeros(n, np.uint8); pen = np.zeros(n, np.int32)
    trace = np.zeros((n, gens + 1), np.int64)
    fn = self.c._f("ga_run")
    fn.restype = ctypes.c_double
    fn.argtypes = [_vp, _vp] + [ctypes.c_int] * 6 + [_vp] * 5
    secs = fn(self.h, _p(seeds), n, int(pop_size), int(gens), int(max_steps), int(as_is), int(threads),
              _p(hcv), _p(scv), _p(feas), _p(pen), _p(trace))
    return hcv, scv, feas, pen, trace, secs


_Handle.ga_run = _ga_run


def _ga_children(self, pop_slot, pop_room, pop_penalty, seeds, max_steps, threads=1, as_is=0):
    """ref_ga_children: the reference's per-child path of ga.cpp:543-577 (Ref
    only), child c on Random(seeds[c]). Returns (dict of the children's slot,
    room, hcv, scv, feasible, penalty; final streams; seconds)."""
    pop_slot = np.ascontiguousarray(pop_slot, np.uint8); pop_room = np.ascontiguousarray(pop_room, np.uint8)
    pen = np.ascontiguousarray(pop_penalty, np.int32)
    rng = np.ascontiguousarray(seeds, np.int64).copy()
    C, N = rng.size, pop_slot.shape[0]
    out = dict(slot=np.zeros((C, self.E), np.uint8), room=np.zeros((C, self.E), np.uint8),
               hcv=np.zeros(C, np.int32), scv=np.zeros(C, np.int32), feasible=np.zeros(C, np.uint8),
               penalty=np.zeros(C, np.int32))
    fn = self.c._f("ga_children")
    fn.restype = ctypes.c_double
    fn.argtypes = [_vp] * 4 + [ctypes.c_int, _vp] + [ctypes.c_int] * 4 + [_vp] * 6
    secs = fn(self.h, _p(pop_slot), _p(pop_room), _p(pen), N, _p(rng), C, int(max_steps), int(threads), int(as_is),
              _p(out["slot"]), _p(out["room"]), _p(out["hcv"]), _p(out["scv"]), _p(out["feasible"]),
              _p(out["penalty"]))
    return out, rng, secs


_Handle.ga_children = _ga_children


def host_threads(cap: int = 16) -> int:
    """Threads for the checkers: the cores this job may use, at most `cap`
    (the GPU box grants 16; os.cpu_count() there shows the whole machine)."""
    try:
        n = len(os.sched_getaffinity(0))
    except AttributeError:
        n = os.cpu_count() or 1
    return max(1, min(cap, n))


def split_rows(fn, arrays, *args, threads: int | None = None):
    """fn(*row_slices, *args) over contiguous row blocks of `arrays` on host
    threads (ctypes releases the GIL; the checkers keep no shared mutable
    state), the per-block result tuples concatenated row-wise. Results equal
    one serial call: every individual carries its own stream."""
    n = arrays[0].shape[0]
    T = threads or host_threads()
    blocks = [b for b in np.array_split(np.arange(n), min(T, max(n, 1))) if b.size]
    with ThreadPoolExecutor(len(blocks)) as ex:
        parts = list(ex.map(lambda b: fn(*(np.ascontiguousarray(a[b]) for a in arrays), *args), blocks))
    return tuple(np.concatenate(x) for x in zip(*parts))
