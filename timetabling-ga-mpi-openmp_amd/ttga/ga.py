"""The GA of ga.cpp on the device: one island per GPU, batched generations.

Mirrors ga.cpp:370-613 with the per-child operators running as batched
kernels (include/ttga.h):

* initial population: RandomInitialSolution + localSearch(maxSteps) +
  computePenalty per member (ga.cpp:429-434), then sorted;
* a generation breeds C children from the current population
  (tt_ga_breed: selection5 x2, crossover p=0.8 / copy, mutation p=0.5),
  runs localSearch + evaluation on all of them, and replaces the C worst
  members, re-sorting by penalty (tt_ga_replace). C = 1 is the reference's
  single-thread steady state; C > 1 is the batched counterpart of its
  OpenMP threads (every thread breeding against the shared population);
* migration (ga.cpp:514-540) and the final MIN reduction (ga.cpp:234-257) are
  in ttga.islands.

Each population member and each child slot owns a Park-Miller stream
(the reference shares one unlocked stream between threads).
Stream k of an island with seed s starts at Random(|s| + 1 + k).
"""
from __future__ import annotations

import json
import math
import time

import numpy as np

# ga.cpp:389-397: -p 1 -> 200, -p 2 -> 1000, otherwise 2000
MAX_STEPS = {1: 200, 2: 1000}


def max_steps_for(problem_type: int) -> int:
    return MAX_STEPS.get(int(problem_type), 2000)


def _fmt(v):
    if isinstance(v, bool):
        return "true" if v else "false"
    if isinstance(v, (int, np.integer)):
        return str(int(v))
    if isinstance(v, float):
        if math.isnan(v):
            return "null"
        if math.isinf(v):
            return "1e+9999" if v > 0 else "-1e+9999"
        return "%.17g" % v
    if isinstance(v, dict):
        return "{" + ",".join(json.dumps(k) + ":" + _fmt(v[k]) for k in sorted(v)) + "}"
    if isinstance(v, (list, tuple, np.ndarray)):
        return "[" + ",".join(_fmt(x) for x in v) + "]"
    return json.dumps(v)


def json_line(obj) -> str:
    """jsoncpp StreamWriterBuilder with indentation "" (ga.cpp:171): compact,
    keys sorted (std::map, json/json.h:584), doubles as %.17g (jsoncpp.cpp:4049)."""
    return _fmt(obj)


def stream_seeds(seed: int, first: int, n: int) -> np.ndarray:
    return (np.arange(first, first + n, dtype=np.int64) + np.int64(abs(int(seed)) + 1)).astype(np.int64)


def pack_member(pop: dict, k: int):
    """serializeSolutions(k, 1, ...) (ga.cpp:318-335): one migrant as a flat
    uint8 tensor on the population's device: slot[E], room[E], then int32
    hcv, scv, feasible, penalty."""
    import torch
    meta = torch.stack([pop["hcv"][k], pop["scv"][k], pop["feasible"][k].to(torch.int32), pop["penalty"][k]])
    return torch.cat([pop["slot"][k], pop["room"][k], meta.view(torch.uint8)])


def unpack_member(pop: dict, pos: int, buf) -> None:
    """deserializeSolution(offset, 1, ...) into position `pos` (ga.cpp:344-368).
    `buf` may live on another device (a host-staged payload)."""
    import torch
    E = pop["slot"].shape[1]
    buf = buf.to(pop["slot"].device)
    pop["slot"][pos].copy_(buf[:E])
    pop["room"][pos].copy_(buf[E:2 * E])
    meta = buf[2 * E:2 * E + 16].clone().view(torch.int32)
    pop["hcv"][pos] = meta[0]
    pop["scv"][pos] = meta[1]
    pop["feasible"][pos] = meta[2].to(torch.uint8)
    pop["penalty"][pos] = meta[3]


def new_population(n: int, E: int, device):
    import torch
    return {"slot": torch.zeros((n, E), dtype=torch.uint8, device=device),
            "room": torch.zeros((n, E), dtype=torch.uint8, device=device),
            "hcv": torch.zeros(n, dtype=torch.int32, device=device),
            "scv": torch.zeros(n, dtype=torch.int32, device=device),
            "feasible": torch.zeros(n, dtype=torch.uint8, device=device),
            "penalty": torch.zeros(n, dtype=torch.int32, device=device)}


class Members:
    """A population [N] of (slot, room, hcv, scv, feasible, penalty) tensors
    and the migration interface of ga.cpp (pack / unpack_into). Island adds
    the device GA on top; the class itself works on any torch device, which
    is what the CPU (gloo) tests of the ring use."""

    min_pop = 3     # ring migration writes pop[N-1] and pop[N-2] and reads pop[0], pop[1]

    def __init__(self, pop: dict):
        self.pop = pop
        self.N = int(pop["slot"].shape[0])

    def pack(self, k: int):
        return pack_member(self.pop, k)

    def unpack_into(self, pos: int, buf) -> None:
        unpack_member(self.pop, pos, buf)

    def copy_from(self, other: "Members") -> None:
        for k, t in self.pop.items():
            t.copy_(other.pop[k].to(t.device))

    def member(self, k: int) -> dict:
        """deserialised Solution fields of member k (ga.cpp:318-335 payload)."""
        p = self.pop
        return {"slot": p["slot"][k].cpu().numpy(), "room": p["room"][k].cpu().numpy(),
                "feasible": bool(p["feasible"][k].item()), "scv": int(p["scv"][k].item()),
                "hcv": int(p["hcv"][k].item()), "penalty": int(p["penalty"][k].item())}

    def member_meta(self, k: int):
        p = self.pop
        return (bool(p["feasible"][k].item()), int(p["scv"][k].item()), int(p["hcv"][k].item()),
                int(p["penalty"][k].item()))

    def best_value(self) -> tuple[bool, int]:
        """(feasible, scv) if feasible else (False, hcv*1e6 + scv) (ga.cpp:191,218,247)."""
        b = self.member_meta(0)
        return (True, b[1]) if b[0] else (False, b[2] * 1000000 + b[1])


_SIDE_STREAMS: dict = {}


def _side_streams(dev, base, n: int) -> list:
    """n streams for a staggered island's parts 1..n, cached per (device, base
    stream): islands built one after another on the same base stream reuse the
    same side streams. (A process gets a few hardware queues, GPU_MAX_HW_QUEUES,
    and HIP maps streams onto them as they are created: fresh streams per
    island can land on the queue of the base stream and serialise the parts.)"""
    import torch
    key = (dev.index, None if base is None else base.cuda_stream)
    pool = _SIDE_STREAMS.setdefault(key, [])
    while len(pool) < n:
        pool.append(torch.cuda.Stream(dev))
    return pool[:n]


class Island(Members):
    """One island: population [N] + C child slots, all device-resident.

    schedule "batch": a generation breeds all C children from the population,
    searches them in one launch and replaces the C worst (the next generation
    waits for the slowest child). schedule "staggered": the child slots are
    split into `parts` sub-batches (part j: child slots [j*C/parts, ...) rounded
    as numpy.array_split) on as many streams, and sub-batch h is bred from the
    population after the replacement of sub-batch h - parts, so sub-batch h's
    local search runs while the searches of h - parts + 1 .. h - 1 finish. The
    population operations are totally ordered -- breed(h) after replace(h -
    parts), replace(h - parts + 1) after breed(h) -- so results are
    deterministic, and C children are in flight at every breed, as in the batch
    schedule and as with ga.cpp:488-588's C threads breeding from the shared
    population while the other threads' children are still searched. step()
    advances `parts` sub-batches and leaves parts - 1 of them pending; flush()
    replaces them (every host read of the population flushes first; the
    snapshots the drivers log from do not). The parts run on streams of their
    own even when the island's stream is None; initialize(), step() and
    flush() order their population operations after the caller's work on its
    stream (the island's, else torch's current stream) and make that stream
    wait for the last of them, so the caller's next reads and writes of the
    population are ordered as on a batch island.
    """

    def __init__(self, dp, pop_size: int = 10, children: int = 1, max_steps: int = 200, seed: int = 1,
                 p_cross: float = 0.8, p_mut: float = 0.5, skip_init_draws: bool = True, device=None,
                 p1: float = 1.0, p2: float = 1.0, p3: float = 0.0, lpt: bool | None = None, stream=None,
                 schedule: str = "batch", parts: int = 2):
        """stream: a torch.cuda.Stream of the island's own, or None (torch's current
        stream). Islands multiplexed on one GPU (ttga.islands --islands K) each take
        one, so one island's launches fill the SIMD slots another's local-search tail
        leaves idle; every host read of the island (member, member_meta, best_thread)
        synchronises its stream first, and a caller that moves data between islands
        (migration) synchronises the device around it."""
        import torch
        if not (1 <= children <= pop_size):
            raise ValueError("need 1 <= children <= pop_size")
        if schedule not in ("batch", "staggered"):
            raise ValueError("schedule must be 'batch' or 'staggered'")
        if schedule == "staggered" and not (2 <= parts <= children):
            raise ValueError("the staggered schedule needs 2 <= parts <= children")
        dev = torch.device("cuda", dp.device if device is None else device)
        super().__init__(new_population(int(pop_size), dp.E, dev))
        self.dp, self.C = dp, int(children)
        self.max_steps, self.seed = int(max_steps), int(seed)
        self.p_cross, self.p_mut, self.skip = float(p_cross), float(p_mut), bool(skip_init_draws)
        self.p1, self.p2, self.p3 = float(p1), float(p2), float(p3)   # LS move probabilities (Solution.h:61)
        # longest-expected-first dispatch of the children's local search (only the
        # launch order changes); by default for generations of >= 4096 children
        self.lpt = (int(children) >= 4096) if lpt is None else bool(lpt)
        self.child = new_population(self.C, dp.E, dev)
        self.flags = torch.zeros(self.C, dtype=torch.uint8, device=dev)
        self.rng_init = torch.from_numpy(stream_seeds(seed, 0, self.N)).to(dev)
        self.rng_child = torch.from_numpy(stream_seeds(seed, self.N, self.C)).to(dev)
        self.work = dp.ga_work(self.N)
        self.generation = 0
        self._user_stream = stream                    # None: torch's current stream at each call
        if schedule == "staggered" and stream is None:
            # every part on a stream of its own, the first included: work on the legacy
            # null stream orders itself against the other streams' work, which would
            # serialise the parts (profiles/r06_n_trace_overlap_comp20_staggered.json)
            stream = _side_streams(dev, None, 1)[0]
        self.stream = stream
        self.schedule = schedule
        self.parts = int(parts) if schedule == "staggered" else 1
        self._snap = None
        self._streams = [stream]
        if schedule == "staggered":
            bounds = np.cumsum([0] + [len(x) for x in np.array_split(np.arange(self.C), self.parts)])
            # sub-batch j: its child rows, child streams, flags and work buffer; part 0 runs
            # on the island's stream, the others on streams of their own
            self._part = [{"off": int(bounds[j]), "rows": slice(int(bounds[j]), int(bounds[j + 1])),
                           "work": self.work if j == 0 else dp.ga_work(self.N)} for j in range(self.parts)]
            for d in self._part:
                r = d["rows"]
                d.update(child={k: v[r] for k, v in self.child.items()}, rng=self.rng_child[r], flags=self.flags[r])
            self._streams = [stream] + _side_streams(dev, stream, self.parts - 1)
            self._ev_op = torch.cuda.Event()          # the last population operation (breed or replace)
            self._pending = []                        # parts searched but not yet replaced, in breed order
            self._last_replace = 0                    # part whose work buffer holds the last replace's source
        if stream is not None:
            stream.wait_stream(torch.cuda.current_stream(dev))     # the zero-filled buffers above
        for st in self._streams[1:]:
            st.wait_stream(torch.cuda.current_stream(dev) if stream is None else stream)
        # the buffers were allocated on the creating stream and are used on the island's
        # own stream(s): tell the caching allocator, so a dropped island's blocks are not
        # handed out again while its kernels may still write them
        self._side_streams = [st for st in self._streams if st is not None]
        self._record_streams(self._owned())

    def _owned(self):
        ts = list(self.pop.values()) + list(self.child.values()) + [self.flags, self.rng_init, self.rng_child,
                                                                    self.work]
        if self.schedule == "staggered":
            ts += [d["work"] for d in self._part[1:]]
        return ts

    def _record_streams(self, tensors):
        for st in self._side_streams:
            for t in tensors:
                t.record_stream(st)

    def close(self):
        """Wait for everything the island has enqueued (its buffers can then be
        freed safely whatever the allocator knows)."""
        import torch
        self.flush()
        for st in self._side_streams:
            st.synchronize()
        torch.cuda.current_stream(self.pop["slot"].device).synchronize()

    def _base(self):
        """The stream the caller orders its own work on: the island's stream as
        given, else torch's current stream."""
        import torch
        return (self._user_stream if self._user_stream is not None
                else torch.cuda.current_stream(self.pop["slot"].device))

    def _fork(self):
        """Staggered: the population operations enqueued next come after the
        caller's work enqueued so far on _base() (the chain's event takes it in)."""
        s0 = self._streams[0]
        b = self._base()
        if b != s0:
            s0.wait_stream(b)
        s0.wait_event(self._ev_op)
        self._ev_op.record(s0)

    def _join(self):
        """Staggered: the caller's stream (_base()) waits for the population's
        last operation, so what it enqueues next sees the population as a batch
        schedule on that stream would leave it (pending sub-batches aside)."""
        self._base().wait_event(self._ev_op)

    def _on_stream(self, stream=None):
        import contextlib

        import torch
        st = self.stream if stream is None else stream
        return torch.cuda.stream(st) if st is not None else contextlib.nullcontext()

    def sync(self):
        """Wait for the island's work: pending sub-batches are replaced first
        (staggered schedule), then the island's stream is waited for."""
        import torch
        self.flush()
        if self.stream is not None:
            self.stream.synchronize()
        elif self.schedule == "staggered":
            torch.cuda.current_stream(self.pop["slot"].device).synchronize()

    def member(self, k: int) -> dict:
        self.sync()
        return super().member(k)

    def member_meta(self, k: int):
        self.sync()
        return super().member_meta(k)

    def _evaluate(self, p):
        self.dp.eval(p["slot"], p["room"], out=(p["hcv"], p["scv"], p["feasible"], p["penalty"]))

    def initialize(self):
        """ga.cpp:429-434 for every member, then the population is sorted."""
        if self.schedule == "staggered":
            self._fork()
        with self._on_stream():
            p = self.pop
            self.dp.random_init(self.rng_init, p["slot"], p["room"])
            self.dp.local_search(p["slot"], p["room"], self.rng_init, self.max_steps, self.p1, self.p2, self.p3,
                                 out=(p["hcv"], p["scv"], p["feasible"], p["penalty"]))
            self.dp.ga_replace(p, None, self.work)
            if self.schedule == "staggered":
                self._ev_op.record()
        if self.schedule == "staggered":
            self._join()

    def step(self):
        """One generation of C children (ga.cpp:543-585), enqueued on the island's
        stream(s): the whole batch, or (staggered) each sub-batch in turn."""
        if self.schedule == "staggered":
            self._fork()
            for j in range(self.parts):
                self._part_step(j)
            self._join()
            self.generation += 1
            return
        with self._on_stream():
            self._step()

    def _search(self, c, rng, work):
        """LPT order (optional), localSearch and evaluation of children c (one
        launch: tt_local_search_eval, ga.cpp:574-575)."""
        order = None
        if self.lpt:
            # dispatch the children longest-expected first (hcv before the search,
            # descending): the launch's tail is its slowest waves; results unchanged
            self._evaluate(c)
            order = self.dp.lpt_order(c["hcv"], work)
        self.dp.local_search(c["slot"], c["room"], rng, self.max_steps, self.p1, self.p2, self.p3, order=order,
                             out=(c["hcv"], c["scv"], c["feasible"], c["penalty"]))

    def _step(self):
        c = self.child
        self.dp.ga_breed(self.pop["slot"], self.pop["room"], self.pop["penalty"], self.rng_child, c["slot"], c["room"],
                         self.flags, self.p_cross, self.p_mut, self.skip)
        self._search(c, self.rng_child, self.work)
        self.dp.ga_replace(self.pop, c, self.work)
        self.generation += 1

    def _part_step(self, j: int):
        """Sub-batch j: bred from the population behind the last population
        operation; then, with parts - 1 sub-batches pending, the oldest of them
        is replaced behind that breed; then sub-batch j is searched."""
        import torch
        d, st = self._part[j], self._streams[j]
        with self._on_stream(st):
            torch.cuda.current_stream().wait_event(self._ev_op)           # breed(h) after replace(h - parts)
            self.dp.ga_breed(self.pop["slot"], self.pop["room"], self.pop["penalty"], d["rng"], d["child"]["slot"],
                             d["child"]["room"], d["flags"], self.p_cross, self.p_mut, self.skip)
            self._ev_op.record()
        if len(self._pending) >= self.parts - 1:
            self._replace_oldest()                                          # replace(h - parts + 1) after breed(h)
        with self._on_stream(st):
            self._search(d["child"], d["rng"], d["work"])
        self._pending.append(j)

    def _replace_oldest(self):
        import torch
        j = self._pending.pop(0)
        d = self._part[j]
        with self._on_stream(self._streams[j]):
            torch.cuda.current_stream().wait_event(self._ev_op)
            self.dp.ga_replace(self.pop, d["child"], d["work"])
            self._ev_op.record()
        self._last_replace = j

    def flush(self):
        """Staggered schedule: replace the pending sub-batches in order, and make
        the island's stream wait for the population's last operation (no-op for
        the batch schedule)."""
        import torch
        if self.schedule != "staggered":
            return
        self._fork()
        while self._pending:
            self._replace_oldest()
        self._join()
        with self._on_stream():
            torch.cuda.current_stream().wait_event(self._ev_op)

    def _work_of_last_replace(self):
        return self._part[self._last_replace]["work"] if self.schedule == "staggered" else self.work

    def snapshot(self) -> "Snapshot":
        """pop[0]'s (feasible, scv, hcv) and best_thread()'s source position,
        copied into pinned host memory behind the last replacement enqueued
        (staggered: pending sub-batches stay pending, so the snapshot is the
        population as the last replacement left it); Snapshot.values() waits for
        that copy only, so the host can log generation g while generation g + 1
        runs. Two pinned buffers and events are reused in turn (generation g's
        snapshot is read after g + 1 has been enqueued)."""
        import torch
        if self._snap is None:
            self._snap = [(torch.empty(4, dtype=torch.int32, pin_memory=True), torch.cuda.Event()) for _ in range(2)]
            self._snap_meta = torch.empty(4, dtype=torch.int32, device=self.pop["slot"].device)
            self._record_streams([self._snap_meta])
            self._snap_i = 0
            self._snap_owner = [None, None]
        i = self._snap_i
        host, ev = self._snap[i]
        if self._snap_owner[i] is not None:
            self._snap_owner[i].values()     # the buffer's previous snapshot, read before the reuse
        self._snap_i ^= 1
        st = self._streams[self._last_replace] if self.schedule == "staggered" else None
        with self._on_stream(st):
            off = int(self.dp.lib.tt_ga_work_source_offset(self.N, self.dp.E))
            p, w = self.pop, self._work_of_last_replace()
            m = self._snap_meta
            m[0] = p["feasible"][0]
            m[1] = p["scv"][0]
            m[2] = p["hcv"][0]
            m[3] = w[off:off + 4].view(torch.int32)[0]
            host.copy_(m, non_blocking=True)
            ev.record()
        snap = Snapshot(host, ev, self.generation, self.N - self._last_batch(), self.N, self._thread_base())
        self._snap_owner[i] = snap
        return snap

    def _last_batch(self) -> int:
        """Children merged by the last replacement (best_thread's offset)."""
        if self.schedule != "staggered":
            return self.C
        return self._part[self._last_replace]["child"]["slot"].shape[0]

    def _thread_base(self) -> int:
        """Child slot of the last replacement's first child (staggered: its part's offset)."""
        return self._part[self._last_replace]["off"] if self.schedule == "staggered" else 0

    def best_thread(self) -> int:
        """The reference thread (ga.cpp:498, one per child slot) whose
        replacement put the current pop[0] in place: child c of the last
        tt_ga_replace (the source position it leaves in its own slot of the
        work buffer, tt_ga_work_source_offset), else thread 0. Staggered: the
        child slot index over all sub-batches, after the pending ones are
        replaced."""
        self.sync()
        src = self.dp.ga_work_source(self._work_of_last_replace(), self.N)
        k = self.N - self._last_batch()
        return self._thread_base() + src - k if self.generation > 0 and k <= src < self.N else 0


class Snapshot:
    """Island.snapshot(): pop[0]'s fields after a generation, landing in
    pinned host memory behind an event."""

    def __init__(self, host, event, generation: int, k: int, n: int, base: int = 0):
        self.host, self.event, self.generation, self.k, self.n, self.base = host, event, generation, k, n, base
        self._vals = None

    def values(self):
        """(feasible, scv, hcv, best thread) once the copy has landed (read once:
        the pinned buffer is reused two snapshots later)."""
        if self._vals is None:
            self.event.synchronize()
            f, scv, hcv, src = (int(v) for v in self.host.tolist())
            thread = self.base + src - self.k if self.generation > 0 and self.k <= src < self.n else 0
            self._vals = (bool(f), scv, hcv, thread)
        return self._vals


class CostLog:
    """setCurrentCost (ga.cpp:203-228): a logEntry line whenever pop[0] changes
    the island's best (feasible: scv differs; infeasible: hcv*1e6+scv lower)."""

    def __init__(self, proc_id: int, out, t0: float):
        self.proc_id, self.out, self.t0 = proc_id, out, t0
        self.best_scv = 2 ** 31 - 1          # beginTry (ga.cpp:163-167)
        self.best_eval = 2 ** 31 - 1

    def offer(self, feasible: bool, scv: int, hcv: int, thread_id: int = 0, t: float | None = None):
        """pop[0] now has these fields; returns the logged line or None."""
        entry = None
        if feasible:
            if scv != self.best_scv:
                self.best_scv = scv
                self.best_eval = scv
                entry = scv
        else:
            ev = hcv * 1000000 + scv
            if ev < self.best_eval:
                self.best_eval = ev
                entry = ev
        if entry is None:
            return None
        if t is None:
            t = max(0.0, time.perf_counter() - self.t0)
        line = json_line({"logEntry": {"best": entry, "procID": self.proc_id, "threadID": thread_id, "time": t}})
        if self.out is not None:
            self.out.write(line + "\n")
        return line

    def update(self, island, thread_id: int = 0):
        feas, scv, hcv, _ = island.member_meta(0)
        return self.offer(feas, scv, hcv, thread_id)

    def update_from(self, snap: "Snapshot"):
        """update() from a Snapshot taken right after the generation."""
        feas, scv, hcv, thread = snap.values()
        return self.offer(feas, scv, hcv, thread)


def run_best_line(feasible: bool, total_best: int) -> str:
    """setGlobalCost's line (ga.cpp:234-257), printed by rank 0."""
    return json_line({"runEntry": {"feasible": bool(feasible), "totalBest": int(total_best)}})


def solution_line(best: dict, proc_id: int, total_time: float) -> str:
    """endTry (ga.cpp:169-197) for pop[0] = `best` (Members.member fields);
    threadID is the global tid, 0 outside the parallel region."""
    sol = {"feasible": bool(best["feasible"]), "procID": int(proc_id), "threadID": 0, "totalTime": float(total_time)}
    if best["feasible"]:
        sol["totalBest"] = int(best["scv"])
        sol["timeslots"] = [int(x) for x in best["slot"]]
        sol["rooms"] = [int(x) for x in best["room"]]
    else:
        sol["totalBest"] = int(best["hcv"]) * 1000000 + int(best["scv"])
    return json_line({"solution": sol})


def run_final_line(procs: int, threads: int, total_time: float) -> str:
    """main's closing runEntry (ga.cpp:603-609)."""
    return json_line({"runEntry": {"procsNum": int(procs), "threadsNum": int(threads), "totalTime": float(total_time)}})
