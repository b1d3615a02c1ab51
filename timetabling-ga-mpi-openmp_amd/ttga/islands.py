"""ga.cpp's driver on MI355X: one island per GPU, torch.distributed (RCCL over
xGMI) for the island model; optionally K islands multiplexed on each GPU.

    python -m ttga.islands -i instance.tim -s 42 -p 1 [-c C] [--pop N] [--islands K]
    python -m torch.distributed.run --nproc-per-node 8 --master-addr 127.0.0.1 \
        -m ttga.islands -i instance.tim -s 42 -p 1

Reference correspondence:
* CLI: `-key value` pairs as Control.cpp:3-137; honoured: -i -p -s -c
  (as ga.cpp) plus -p1 -p2 -p3 (LS move probabilities, a documented superset);
  -o -n -t -m -l are parsed and echoed like Control.cpp, then ignored like
  ga.cpp (every JSON line goes to stdout, ga.cpp:60). `-c` (threads) sets the
  children bred per generation. Extensions: `--pop N` (ga.cpp:64 has 10,
  N >= 3), `--islands K` (islands per process, default 1), `--generations G`,
  `--stagger` / `--stagger-parts P` (the children of a generation as 2 / P
  sub-batches on as many streams, each bred P - 1 sub-batches behind:
  ttga.ga.Island's staggered schedule),
  `--backend nccl|gloo` (gloo stages migrants through host memory; with it
  several ranks may share one GPU), `--force-dist` (initialise the process
  group and route the broadcast, the ring send/recv pairs and the MIN through
  torch.distributed even at world 1: a one-rank RCCL communicator whose ring
  neighbours are the rank itself, so the RCCL calls run on a one-GPU box).
* islands: island g = rank*K + k of W = world*K; seed abs(seed + g*(seed/10))
  (ga.cpp:410-415), the base seed chosen by rank 0 (time(NULL) when -s is
  missing, ga.cpp:401) and broadcast; procID = g.
* every island starts from island 0's initial population (ga.cpp:429-444,463-464).
* 2001 children per island (generations 0..2000 of ga.cpp:510), migration
  before generations g with (g+1) % 100 == 50 (ga.cpp:514): best -> island
  (g+1) % W's pop[N-1], 2nd best -> island (g-1) % W's pop[N-2]
  (ga.cpp:479-540); within a process the ring is local copies, across ranks
  one batched send/recv pair per direction.
* setCurrentCost per island with threadID = the child slot (thread) whose
  replacement produced the new best (ga.cpp:203-228,584); setGlobalCost MIN
  all-reduce (ga.cpp:234-257), endTry per island (ga.cpp:169-197), final
  runEntry (ga.cpp:602-609). logEntry/solution times run from beginTry
  (ga.cpp:476, after the initial population is shared), the final totalTime
  from process start (ga.cpp:381). JSON lines in the reference's format.
"""
from __future__ import annotations

import math
import os
import sys
import time

USAGE = "-i InputFile [-o OutputFile] [-n NumberOfTries] [-s RandomSeed] [-t TimeLimit] [-p ProblemType]"
TOTAL_CHILDREN = 2001          # generations 0..2000 per rank, ga.cpp:510


def parse_control(argv, out=sys.stdout, err=sys.stderr) -> dict:
    """Control::Control (Control.cpp:3-137): `-key value` pairs."""
    args = list(argv)
    extra = {}
    if "--stagger" in args:               # the staggered schedule (ttga.ga.Island), 2 sub-batches
        args.remove("--stagger")
        extra["stagger"] = 2
    for k in ("--pop", "--children", "--generations", "--islands", "--stagger-parts"):
        if k in args:
            i = args.index(k)
            extra[k[2:].replace("-", "_")] = int(args[i + 1])
            del args[i:i + 2]
    if len(args) % 2 != 0:
        err.write("Parse error: Number of command line parameters incorrect\nUsage:\n" + USAGE + "\n")
        raise SystemExit(1)
    kv = {args[i]: args[i + 1] for i in range(0, len(args), 2)}
    c = {"threads": 1, "tries": 10, "time_limit": 90.0, "problem_type": 1, "max_steps": 100, "ls_limit": 99999.0,
         "p1": 1.0, "p2": 1.0, "p3": 0.0}
    if "-c" in kv:
        c["threads"] = int(kv["-c"]); out.write(f"Max number of threads {c['threads']}\n")
    else:
        err.write("Warning: Number of threads is set to default (1)\n")
    if "-i" not in kv:
        err.write("Error: No input file given, exiting\nUsage:\n" + USAGE + "\n")
        raise SystemExit(1)
    c["input"] = kv["-i"]
    c["output"] = kv.get("-o")
    if c["output"] is None:
        err.write("Warning: No output file given, writing to stdout\n")
    if "-n" in kv:
        c["tries"] = int(kv["-n"]); out.write(f"Max number of tries {c['tries']}\n")
    else:
        err.write("Warning: Number of tries is set to default (10)\n")
    if "-t" in kv:
        c["time_limit"] = float(kv["-t"]); out.write(f"Time limit {kv['-t']}\n")
    else:
        err.write("Warning: Time limit is set to default (90 sec)\n")
    if "-p" in kv:
        c["problem_type"] = int(kv["-p"]); out.write(f"Problem instance type {c['problem_type']}\n")
    if "-m" in kv:
        c["max_steps"] = int(kv["-m"]); out.write(f"Max number of steps in the local search {c['max_steps']}\n")
    if "-l" in kv:
        c["ls_limit"] = float(kv["-l"]); out.write(f"Local search time limit {kv['-l']}\n")
    else:
        err.write("Warning: The local search time limit is set to default (99999 sec)\n")
    for k, name in (("-p1", "p1"), ("-p2", "p2"), ("-p3", "p3")):
        if k in kv:
            c[name] = float(kv[k]); out.write(f"LS move {k[2]} probability {kv[k]}\n")
        else:
            d = {"p1": "1.0", "p2": "1.0", "p3": "0.0"}[name]
            err.write(f"Warning: The local search move {k[2]} probability is set to default {d}\n")
    if "-s" in kv:
        c["seed"] = int(kv["-s"])
    else:
        c["seed"] = int(time.time())
        err.write(f"Warning: {c['seed']} used as default random seed\n")
    c.update(extra)
    return c


def _free_port() -> int:
    import socket
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def rank_seed(seed: int, rank: int) -> int:
    """ga.cpp:412 with C int division."""
    q = abs(seed) // 10
    q = q if seed >= 0 else -q
    return abs(seed + rank * q)


def _wire(t, backend: str):
    """Payload as the process group can move it: gloo moves host tensors."""
    return t.cpu() if backend == "gloo" else t


def _exchange(send, dst: int, src: int, backend: str):
    import torch
    import torch.distributed as dist
    buf = _wire(send.contiguous(), backend)
    got = torch.empty_like(buf)
    for r in dist.batch_isend_irecv([dist.P2POp(dist.isend, buf, dst), dist.P2POp(dist.irecv, got, src)]):
        r.wait()
    return got


def ring_migrate(islands, rank: int, world: int, backend: str = "nccl", use_dist: bool | None = None):
    """ga.cpp:514-540 with one migrant each way over the ring of all W =
    world * K islands (island g = rank * K + k): g's best replaces pop[N-1] of
    island (g+1) % W, g's 2nd best replaces pop[N-2] of island (g-1) % W. All
    payloads are packed before any is written (MPI_Sendrecv semantics; with
    N >= 3 the rows read and written are disjoint, as in the reference)."""
    if not isinstance(islands, (list, tuple)):
        islands = [islands]
    K, N = len(islands), islands[0].N
    if N < 3:
        raise ValueError("ring migration needs a population of at least 3")
    best = [isl.pack(0) for isl in islands]
    second = [isl.pack(1) for isl in islands]
    if not (world > 1 if use_dist is None else use_dist):
        from_left, from_right = best[-1], second[0]
    else:
        right, left = (rank + 1) % world, (rank - 1 + world) % world
        from_left = _exchange(best[-1], right, left, backend)
        from_right = _exchange(second[0], left, right, backend)
    for k, isl in enumerate(islands):
        isl.unpack_into(N - 1, best[k - 1] if k > 0 else from_left)
        isl.unpack_into(N - 2, second[k + 1] if k < K - 1 else from_right)


def global_min(value: int, device, world: int, backend: str = "nccl", use_dist: bool | None = None) -> int:
    import torch
    import torch.distributed as dist
    if not (world > 1 if use_dist is None else use_dist):
        return int(value)
    t = torch.tensor([int(value)], dtype=torch.int64, device=device if backend != "gloo" else "cpu")
    dist.all_reduce(t, op=dist.ReduceOp.MIN)
    return int(t.item())


def share_seed(seed, world: int, use_dist: bool | None = None) -> int:
    """Rank 0's base seed on every rank (ga.cpp:401,410-415)."""
    import torch.distributed as dist
    if not (world > 1 if use_dist is None else use_dist):
        return int(seed)
    lst = [int(seed)]
    dist.broadcast_object_list(lst, src=0)
    return int(lst[0])


def broadcast_population(islands, world: int, backend: str = "nccl", use_dist: bool | None = None):
    """Island 0 of rank 0 to every island (ga.cpp:436-444,461-464)."""
    import torch.distributed as dist
    if world > 1 if use_dist is None else use_dist:
        for t in islands[0].pop.values():
            if backend == "gloo" and t.is_cuda:
                h = t.cpu()
                dist.broadcast(h, src=0)
                t.copy_(h)
            else:
                dist.broadcast(t, src=0)
    for isl in islands[1:]:
        isl.copy_from(islands[0])


def main(argv=None):
    import torch
    import torch.distributed as dist

    from . import instance as tim
    from .ga import CostLog, Island, max_steps_for, run_best_line, run_final_line, solution_line

    from .native import DeviceProblem

    t_start = time.perf_counter()
    argv = sys.argv[1:] if argv is None else argv
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    backend = "nccl"
    if "--backend" in argv:
        i = argv.index("--backend")
        backend = argv[i + 1]
        argv = argv[:i] + argv[i + 2:]
    use_dist = world > 1
    if "--force-dist" in argv:
        use_dist = True
        argv = [a for a in argv if a != "--force-dist"]
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        os.environ.setdefault("MASTER_PORT", str(_free_port()))
        os.environ.setdefault("WORLD_SIZE", str(world))
        os.environ.setdefault("RANK", str(rank))
    device = local % max(1, torch.cuda.device_count())
    torch.cuda.set_device(device)
    if use_dist:
        if backend == "nccl":
            dist.init_process_group("nccl", device_id=torch.device("cuda", device))
        else:
            dist.init_process_group(backend)
    ctl = parse_control(argv, out=sys.stdout if rank == 0 else open(os.devnull, "w"),
                        err=sys.stderr if rank == 0 else open(os.devnull, "w"))
    out = sys.stdout                 # ga.cpp:60: -o is parsed, output always goes to cout
    seed = share_seed(ctl["seed"], world, use_dist)
    inst = tim.read_tim(ctl["input"])
    dp = DeviceProblem(inst, device=device)
    C = ctl.get("children", ctl["threads"])
    N = ctl.get("pop", 10)
    if N < 3:
        sys.stderr.write("Error: --pop must be at least 3 (ring migration writes pop[N-1] and pop[N-2])\n")
        raise SystemExit(1)
    C = max(1, min(C, N))
    K = max(1, ctl.get("islands", 1))
    W = world * K
    # K > 1: a stream per island, so one island's launches fill the SIMD slots
    # another's local-search tail leaves idle (the islands are independent
    # between migrations)
    streams = [torch.cuda.Stream(device=device) for _ in range(K)] if K > 1 else [None]
    # the staggered schedule: --stagger (2 sub-batches) or --stagger-parts P, at most C
    parts = min(C, ctl.get("stagger_parts", ctl.get("stagger", 0)))
    islands = [Island(dp, pop_size=N, children=C, max_steps=max_steps_for(ctl["problem_type"]),
                      seed=rank_seed(seed, rank * K + k), p1=ctl["p1"], p2=ctl["p2"], p3=ctl["p3"],
                      stream=streams[k], schedule="staggered" if parts >= 2 else "batch", parts=max(parts, 2))
               for k in range(K)]
    if rank == 0:
        islands[0].initialize()
    torch.cuda.synchronize()
    broadcast_population(islands, world, backend, use_dist)
    torch.cuda.synchronize()
    t_begin = time.perf_counter()    # beginTry (ga.cpp:476)
    logs = [CostLog(rank * K + k, out, t_begin) for k in range(K)]
    for log, isl in zip(logs, islands):
        log.update(isl, 0)           # ga.cpp:503
    gens = ctl.get("generations", math.ceil(TOTAL_CHILDREN / C))
    # a generation's log lines are written once the next generation is enqueued:
    # the host waits for generation g's pop[0] snapshot while g + 1 runs
    # (same lines, same order; each line's time is taken when its snapshot lands)
    pending = []

    def flush():
        for log, snap in pending:
            log.update_from(snap)
        pending.clear()
    for g in range(gens):
        if (g + 1) % 100 == 50:
            flush()
            for isl in islands:                  # staggered: the pending half-batch replaced first
                isl.flush()
            torch.cuda.synchronize()             # every island's stream, before the copies
            if use_dist:
                dist.barrier()
            ring_migrate(islands, rank, world, backend, use_dist)
            torch.cuda.synchronize()             # the migrants in place before the islands go on
        snaps = []
        for isl in islands:                      # enqueued back to back: the islands' streams overlap
            isl.step()
            snaps.append(isl.snapshot())
        flush()
        pending.extend(zip(logs, snaps))
    flush()
    torch.cuda.synchronize()
    vals = [isl.best_value() for isl in islands]
    gmin = global_min(min(v for _, v in vals), torch.device("cuda", device), world, backend, use_dist)
    if rank == 0:
        # setGlobalCost: "feasible" is rank 0's own pop[0] (ga.cpp:236-256)
        out.write(run_best_line(vals[0][0], gmin) + "\n")
    for k, isl in enumerate(islands):
        out.write(solution_line(isl.member(0), rank * K + k, time.perf_counter() - t_begin) + "\n")
    out.flush()
    if use_dist:
        dist.barrier()
    if rank == 0:
        out.write(run_final_line(W, C, time.perf_counter() - t_start) + "\n")
    out.flush()
    if use_dist:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
