"""ga.cpp's driver on MI355X: one island per GPU, torch.distributed (RCCL over
xGMI) for the island model.

    python -m ttga.islands -i instance.tim -s 42 -p 1 [-c C] [--pop N]
    python -m torch.distributed.run --nproc-per-node 8 --master-addr 127.0.0.1 \
        -m ttga.islands -i instance.tim -s 42 -p 1

Reference correspondence:
* CLI: `-key value` pairs as Control.cpp:3-137; honoured: -i -o -p -s -c
  (as ga.cpp) plus -p1 -p2 -p3 (LS move probabilities, a documented superset);
  -n -t -m -l are parsed and echoed like Control.cpp, then ignored like ga.cpp.
  `-c` (threads) sets the children bred per generation. `--pop` sets the
  population size (ga.cpp:64 has 10).
* seeds: rank i uses abs(seed + i*(seed/10)) (ga.cpp:410-415).
* every island starts from rank 0's initial population (ga.cpp:429-444,463-464).
* 2001 children per island (generations 0..2000 of ga.cpp:510), migration
  before generations g with (g+1) % 100 == 50 (ga.cpp:514): best -> right
  neighbour's pop[N-1], 2nd best -> left neighbour's pop[N-2] (ga.cpp:479-540).
* setGlobalCost MIN all-reduce (ga.cpp:234-257), endTry per rank (ga.cpp:169-197),
  final runEntry (ga.cpp:602-609). JSON lines in the reference's format.
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
    for k in ("--pop", "--children", "--generations"):
        if k in args:
            i = args.index(k)
            extra[k[2:]] = int(args[i + 1])
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


def rank_seed(seed: int, rank: int) -> int:
    """ga.cpp:412 with C int division."""
    q = abs(seed) // 10
    q = q if seed >= 0 else -q
    return abs(seed + rank * q)


def ring_migrate(island, rank: int, world: int):
    """ga.cpp:514-540 with one migrant each way: best -> (rank+1) replaces its
    pop[N-1]; 2nd best -> (rank-1) replaces its pop[N-2]."""
    import torch
    import torch.distributed as dist
    N = island.N
    snd, rcv = (rank + 1) % world, (rank - 1 + world) % world
    for k, dst, src, pos in ((0, snd, rcv, N - 1), (1, rcv, snd, N - 2)):
        if pos < 0:
            continue
        buf = island.pack(min(k, N - 1)).contiguous()
        if world == 1:
            island.unpack_into(pos, buf.clone())
            continue
        got = torch.empty_like(buf)
        ops = [dist.P2POp(dist.isend, buf, dst), dist.P2POp(dist.irecv, got, src)]
        for r in dist.batch_isend_irecv(ops):
            r.wait()
        island.unpack_into(pos, got)


def global_min(value: int, device, world: int) -> int:
    import torch
    import torch.distributed as dist
    if world == 1:
        return int(value)
    t = torch.tensor([int(value)], dtype=torch.int64, device=device)
    dist.all_reduce(t, op=dist.ReduceOp.MIN)
    return int(t.item())


def broadcast_population(island, world: int):
    import torch.distributed as dist
    if world == 1:
        return
    for t in island.pop.values():
        dist.broadcast(t, src=0)


def main(argv=None):
    import torch
    import torch.distributed as dist

    from . import instance as tim
    from .ga import CostLog, Island, json_line, max_steps_for
    from .native import DeviceProblem

    argv = sys.argv[1:] if argv is None else argv
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world > 1:
        torch.cuda.set_device(local)
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))
    t0 = time.perf_counter()
    ctl = parse_control(argv, out=sys.stdout if rank == 0 else open(os.devnull, "w"))
    out = open(ctl["output"], "w") if ctl.get("output") else sys.stdout
    inst = tim.read_tim(ctl["input"])
    dp = DeviceProblem(inst, device=local)
    C = ctl.get("children", ctl["threads"])
    N = ctl.get("pop", 10)
    C = max(1, min(C, N))
    island = Island(dp, pop_size=N, children=C, max_steps=max_steps_for(ctl["problem_type"]),
                    seed=rank_seed(ctl["seed"], rank), p1=ctl["p1"], p2=ctl["p2"], p3=ctl["p3"])
    if rank == 0:
        island.initialize()
    broadcast_population(island, world)
    log = CostLog(rank, out, t0)
    log.update(island)
    gens = ctl.get("generations", math.ceil(TOTAL_CHILDREN / C))
    for g in range(gens):
        if (g + 1) % 100 == 50:
            if world > 1:
                dist.barrier()
            ring_migrate(island, rank, world)
        island.step()
        log.update(island)
    torch.cuda.synchronize()
    feasible, value = island.best_value()
    gmin = global_min(value, torch.device("cuda", local), world)
    if rank == 0:
        out.write(json_line({"runEntry": {"feasible": feasible, "totalBest": gmin}}) + "\n")
    best = island.member(0)
    sol = {"feasible": best["feasible"], "procID": rank, "threadID": 0,
           "totalTime": time.perf_counter() - t0}
    if best["feasible"]:
        sol["totalBest"] = best["scv"]
        sol["timeslots"] = [int(x) for x in best["slot"]]
        sol["rooms"] = [int(x) for x in best["room"]]
    else:
        sol["totalBest"] = best["hcv"] * 1000000 + best["scv"]
    out.write(json_line({"solution": sol}) + "\n")
    if world > 1:
        dist.barrier()
    if rank == 0:
        out.write(json_line({"runEntry": {"procsNum": world, "threadsNum": C,
                                          "totalTime": time.perf_counter() - t0}}) + "\n")
    out.flush()
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
