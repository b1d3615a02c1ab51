"""ctypes binding of libttga.so (include/ttga.h) for device-resident populations.

There is no CPU fallback anywhere in this module: if the HIP library is missing
or the device calls fail, every entry point raises. Tensors are torch CUDA
(=HIP) tensors; calls are enqueued on torch's current stream of the tensor's
device.
"""
from __future__ import annotations

import ctypes
import os
import pathlib

import numpy as np

PKG_DIR = pathlib.Path(__file__).resolve().parent.parent
LIB_PATH = PKG_DIR / "libttga.so"

TT_OK, TT_ERR_INVALID, TT_ERR_DEVICE, TT_ERR_LIMIT = 0, 1, 2, 3
NUM_SLOTS = 45

EXPORTS = (
    "tt_problem_create", "tt_problem_destroy", "tt_problem_dims", "tt_problem_derived", "tt_eval",
    "tt_eval_variant", "tt_assign_rooms", "tt_random_init", "tt_crossover", "tt_mutation", "tt_local_search",
    "tt_device_status", "tt_last_error", "tt_version", "tt_ga_breed", "tt_ga_work_bytes", "tt_ga_replace",
    "tt_eval_auto_variant", "tt_local_search_ordered", "tt_lpt_order", "tt_ga_work_source_offset",
    "tt_local_search_stats", "tt_local_search_masks", "tt_local_search_eval",
)

_lib = None


class TTError(RuntimeError):
    def __init__(self, code: int, msg: str):
        super().__init__(f"ttga error {code}: {msg}")
        self.code = code


def load(path: os.PathLike | str | None = None) -> ctypes.CDLL:
    """Load libttga.so (built in-tree by `make -C timetabling-ga-mpi-openmp_amd`)."""
    global _lib
    if _lib is not None and path is None:
        return _lib
    p = pathlib.Path(path) if path else LIB_PATH
    if not p.exists():
        raise FileNotFoundError(f"{p} not built: run `make -C {PKG_DIR}` (hipcc --offload-arch=gfx950)")
    lib = ctypes.CDLL(str(p))
    vp, i32, dbl = ctypes.c_void_p, ctypes.c_int, ctypes.c_double
    P = ctypes.POINTER
    lib.tt_problem_create.argtypes = [i32, i32, i32, i32, vp, vp, vp, vp, i32, P(vp)]
    lib.tt_problem_destroy.argtypes = [vp]
    lib.tt_problem_dims.argtypes = [vp, vp]
    lib.tt_problem_derived.argtypes = [vp, vp, vp, vp]
    lib.tt_eval.argtypes = [vp, vp, vp, i32, vp, vp, vp, vp, vp]
    lib.tt_eval_variant.argtypes = [vp, vp, vp, i32, vp, vp, vp, vp, i32, vp]
    lib.tt_assign_rooms.argtypes = [vp, vp, vp, i32, vp]
    lib.tt_random_init.argtypes = [vp, vp, vp, vp, i32, vp]
    lib.tt_crossover.argtypes = [vp, vp, vp, vp, vp, vp, i32, vp]
    lib.tt_mutation.argtypes = [vp, vp, vp, vp, i32, vp]
    lib.tt_local_search.argtypes = [vp, vp, vp, vp, i32, i32, dbl, dbl, dbl, vp]
    lib.tt_local_search_ordered.argtypes = [vp, vp, vp, vp, i32, i32, dbl, dbl, dbl, vp, vp]
    lib.tt_lpt_order.argtypes = [vp, vp, i32, vp, vp, vp]
    lib.tt_local_search_stats.argtypes = [vp, vp, vp]
    lib.tt_local_search_masks.argtypes = [vp, vp, vp]
    lib.tt_local_search_eval.argtypes = [vp, vp, vp, vp, i32, i32, dbl, dbl, dbl, vp, vp, vp, vp, vp, vp]
    lib.tt_device_status.argtypes = [vp, vp]
    lib.tt_eval_auto_variant.argtypes = [vp]
    lib.tt_ga_breed.argtypes = [vp, vp, vp, vp, i32, vp, i32, dbl, dbl, i32, vp, vp, vp, vp]
    lib.tt_ga_work_bytes.argtypes = [i32, i32]
    lib.tt_ga_work_bytes.restype = ctypes.c_size_t
    lib.tt_ga_work_source_offset.argtypes = [i32, i32]
    lib.tt_ga_work_source_offset.restype = ctypes.c_size_t
    lib.tt_ga_replace.argtypes = [vp] * 7 + [i32] + [vp] * 6 + [i32, vp, vp]
    lib.tt_last_error.restype = ctypes.c_char_p
    lib.tt_last_error.argtypes = []
    lib.tt_version.argtypes = []
    for name in EXPORTS:
        if name not in ("tt_last_error", "tt_ga_work_bytes", "tt_ga_work_source_offset"):
            getattr(lib, name).restype = ctypes.c_int
    if path is None:
        _lib = lib
    return lib


def _check(lib, rc: int):
    if rc != TT_OK:
        raise TTError(rc, lib.tt_last_error().decode(errors="replace"))


def _np_ptr(a: np.ndarray):
    return a.ctypes.data_as(ctypes.c_void_p)


class DeviceProblem:
    """A tt_problem handle: the Problem image resident on one GPU."""

    def __init__(self, inst, device: int = 0):
        self.lib = load()
        self.inst = inst
        self.device = device
        self.E, self.R, self.F, self.S = inst.E, inst.R, inst.F, inst.S
        h = ctypes.c_void_p()
        rs, A = inst.room_size, inst.student_events
        rf, ef = inst.room_features, inst.event_features
        _check(self.lib, self.lib.tt_problem_create(self.E, self.R, self.F, self.S, _np_ptr(rs), _np_ptr(A),
                                                    _np_ptr(rf), _np_ptr(ef), device, ctypes.byref(h)))
        self.handle = h

    def close(self):
        if getattr(self, "handle", None):
            self.lib.tt_problem_destroy(self.handle)
            self.handle = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def derived(self):
        sn = np.zeros(self.E, np.int32)
        corr = np.zeros((self.E, self.E), np.int32)
        poss = np.zeros((self.E, self.R), np.int32)
        _check(self.lib, self.lib.tt_problem_derived(self.handle, _np_ptr(sn), _np_ptr(corr), _np_ptr(poss)))
        return sn, corr, poss

    def eval_variant(self) -> int:
        """The kernel tt_eval runs for this instance (tt_eval_variant numbering)."""
        return int(self.lib.tt_eval_auto_variant(self.handle))

    def status(self) -> int:
        v = ctypes.c_int32(0)
        _check(self.lib, self.lib.tt_device_status(self.handle, ctypes.byref(v)))
        return int(v.value)

    # -- population operations (torch tensors on this device) -------------------
    @staticmethod
    def _stream(t):
        # note: every library call makes the handle's device current (hipSetDevice)
        # and leaves it so; tensors of another device are rejected by _pop/_rng
        import torch
        return ctypes.c_void_p(torch.cuda.current_stream(t.device).cuda_stream)

    def _pop(self, slot, room=None):
        import torch
        for t in (slot, room):
            if t is None:
                continue
            if not (t.is_cuda and t.dtype == torch.uint8 and t.is_contiguous() and t.dim() == 2 and t.shape[1] == self.E):
                raise ValueError("population tensors must be contiguous uint8 CUDA tensors of shape [P, E]")
            if t.device.index != self.device:
                raise ValueError(f"tensor on cuda:{t.device.index}, problem handle on cuda:{self.device}")
        return slot.shape[0]

    def eval(self, slot, room, variant: int = 0, out=None):
        import torch
        P = self._pop(slot, room)
        if out is None:
            dev = slot.device
            out = (torch.empty(P, dtype=torch.int32, device=dev), torch.empty(P, dtype=torch.int32, device=dev),
                   torch.empty(P, dtype=torch.uint8, device=dev), torch.empty(P, dtype=torch.int32, device=dev))
        hcv, scv, feas, pen = out
        _check(self.lib, self.lib.tt_eval_variant(self.handle, slot.data_ptr(), room.data_ptr(), P, hcv.data_ptr(),
                                                  scv.data_ptr(), feas.data_ptr(), pen.data_ptr(), variant,
                                                  self._stream(slot)))
        return out

    def assign_rooms(self, slot, room=None):
        import torch
        P = self._pop(slot, room)
        if room is None:
            room = torch.empty_like(slot)
        _check(self.lib, self.lib.tt_assign_rooms(self.handle, slot.data_ptr(), room.data_ptr(), P, self._stream(slot)))
        return room

    def random_init(self, rng, slot, room):
        P = self._pop(slot, room)
        self._rng(rng, P)
        _check(self.lib, self.lib.tt_random_init(self.handle, rng.data_ptr(), slot.data_ptr(), room.data_ptr(), P,
                                                 self._stream(slot)))

    def crossover(self, slot1, slot2, rng, slot, room):
        P = self._pop(slot, room)
        self._pop(slot1, slot2)
        self._rng(rng, P)
        _check(self.lib, self.lib.tt_crossover(self.handle, slot1.data_ptr(), slot2.data_ptr(), rng.data_ptr(),
                                               slot.data_ptr(), room.data_ptr(), P, self._stream(slot)))

    def mutation(self, slot, room, rng):
        P = self._pop(slot, room)
        self._rng(rng, P)
        _check(self.lib, self.lib.tt_mutation(self.handle, slot.data_ptr(), room.data_ptr(), rng.data_ptr(), P,
                                              self._stream(slot)))

    def local_search(self, slot, room, rng, max_steps: int, p1=1.0, p2=1.0, p3=0.0, order=None, out=None):
        """order: optional int32 device permutation, the dispatch order (results unchanged).
        out: optional (hcv, scv, feasible, penalty) device tensors of P entries, filled with
        the searched individuals' evaluation in the same launch (tt_local_search_eval)."""
        import torch
        P = self._pop(slot, room)
        self._rng(rng, P)
        if out is not None:
            if order is not None and not (order.is_cuda and order.dtype == torch.int32 and order.is_contiguous()
                                          and order.numel() == P):
                raise ValueError("order must be a contiguous int32 CUDA tensor of P entries")
            hcv, scv, feas, pen = out
            for t, dt in ((hcv, torch.int32), (scv, torch.int32), (feas, torch.uint8), (pen, torch.int32)):
                if not (t.is_cuda and t.dtype == dt and t.is_contiguous() and t.numel() == P):
                    raise ValueError("out must be contiguous CUDA tensors (int32, int32, uint8, int32) of P entries")
            _check(self.lib, self.lib.tt_local_search_eval(
                self.handle, slot.data_ptr(), room.data_ptr(), rng.data_ptr(), P, int(max_steps), float(p1),
                float(p2), float(p3), ctypes.c_void_p(order.data_ptr() if order is not None else None),
                hcv.data_ptr(), scv.data_ptr(), feas.data_ptr(), pen.data_ptr(), self._stream(slot)))
            return
        if order is None:
            _check(self.lib, self.lib.tt_local_search(self.handle, slot.data_ptr(), room.data_ptr(), rng.data_ptr(),
                                                      P, int(max_steps), float(p1), float(p2), float(p3),
                                                      self._stream(slot)))
            return
        if not (order.is_cuda and order.dtype == torch.int32 and order.is_contiguous() and order.numel() == P):
            raise ValueError("order must be a contiguous int32 CUDA tensor of P entries")
        _check(self.lib, self.lib.tt_local_search_ordered(self.handle, slot.data_ptr(), room.data_ptr(),
                                                          rng.data_ptr(), P, int(max_steps), float(p1), float(p2),
                                                          float(p3), ctypes.c_void_p(order.data_ptr()),
                                                          self._stream(slot)))

    def local_search_stats(self, stream=None):
        """(phase-2 steps, all steps) of the last tt_local_search call on the
        stream (torch's current stream by default); waits for that call's
        counts (diagnostics)."""
        import torch
        st = torch.cuda.current_stream(self.device) if stream is None else stream
        out = (ctypes.c_ulonglong * 2)()
        _check(self.lib, self.lib.tt_local_search_stats(self.handle, ctypes.c_void_p(st.cuda_stream), out))
        return int(out[0]), int(out[1])

    def local_search_masks(self, stream=None) -> int:
        """Students with phase-2 masks in the last tt_local_search call's first
        launch on the stream (0: none, -1: no call yet; diagnostics)."""
        import torch
        st = torch.cuda.current_stream(self.device) if stream is None else stream
        out = ctypes.c_int32(0)
        _check(self.lib, self.lib.tt_local_search_masks(self.handle, ctypes.c_void_p(st.cuda_stream),
                                                        ctypes.byref(out)))
        return int(out.value)

    def lpt_order(self, key, work):
        """tt_lpt_order: indices of key (int32 CUDA) by key descending, ties by
        index, negative keys last, as an int32 CUDA tensor."""
        import torch
        n = key.numel()
        if not (key.is_cuda and key.dtype == torch.int32 and key.is_contiguous()):
            raise ValueError("key must be a contiguous int32 CUDA tensor")
        order = torch.empty(n, dtype=torch.int32, device=key.device)
        _check(self.lib, self.lib.tt_lpt_order(self.handle, ctypes.c_void_p(key.data_ptr()), n,
                                               ctypes.c_void_p(order.data_ptr()), ctypes.c_void_p(work.data_ptr()),
                                               self._stream(key)))
        return order

    # -- GA generation primitives ---------------------------------------------------
    def ga_breed(self, pop_slot, pop_room, pop_penalty, rng, child_slot, child_room, child_flags,
                 p_cross=0.8, p_mut=0.5, skip_init_draws=True):
        N = self._pop(pop_slot, pop_room)
        C = self._pop(child_slot, child_room)
        self._rng(rng, C)
        _check(self.lib, self.lib.tt_ga_breed(self.handle, pop_slot.data_ptr(), pop_room.data_ptr(),
                                              pop_penalty.data_ptr(), N, rng.data_ptr(), C, float(p_cross),
                                              float(p_mut), int(bool(skip_init_draws)), child_slot.data_ptr(),
                                              child_room.data_ptr(), child_flags.data_ptr(), self._stream(pop_slot)))

    def ga_work(self, N):
        import torch
        return torch.empty(int(self.lib.tt_ga_work_bytes(N, self.E)), dtype=torch.uint8,
                           device=torch.device("cuda", self.device))

    def ga_work_source(self, work, N) -> int:
        """The merged position tt_ga_replace's new pop[0] came from (synchronises)."""
        import torch
        off = int(self.lib.tt_ga_work_source_offset(N, self.E))
        return int(work[off:off + 4].view(torch.int32)[0].item())

    def ga_replace(self, pop, child, work):
        """pop/child: dicts of device tensors slot, room, hcv, scv, feasible, penalty."""
        N = self._pop(pop["slot"], pop["room"])
        C = self._pop(child["slot"], child["room"]) if child is not None else 0
        c = child or {k: pop[k] for k in pop}
        _check(self.lib, self.lib.tt_ga_replace(
            self.handle, pop["slot"].data_ptr(), pop["room"].data_ptr(), pop["hcv"].data_ptr(),
            pop["scv"].data_ptr(), pop["feasible"].data_ptr(), pop["penalty"].data_ptr(), N,
            c["slot"].data_ptr(), c["room"].data_ptr(), c["hcv"].data_ptr(), c["scv"].data_ptr(),
            c["feasible"].data_ptr(), c["penalty"].data_ptr(), C, work.data_ptr(), self._stream(pop["slot"])))

    @staticmethod
    def _rng(rng, P):
        import torch
        if not (rng.is_cuda and rng.dtype == torch.int64 and rng.is_contiguous() and rng.numel() == P):
            raise ValueError("rng must be a contiguous int64 CUDA tensor with one state per individual")
