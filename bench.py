"""Headline benchmark: fitness evaluations per second (hcv + scv + feasibility +
penalty, Solution.cpp:63-170) of a device-resident population of 65,536
individuals on the 400-event medium01-size instance, per GPU (weak scaling:
one independent population shard per rank, no data-path collective).

    python bench.py [--gpus N] [--steps K] [--warmup W] [--config med|lg|syn|sm]
    python bench.py --gpus N --config syn --global-pop 262144      (strong scaling)
    python -m torch.distributed.run --nproc-per-node N ... bench.py --gpus N

`--gpus N > 1` without a launcher (no WORLD_SIZE in the environment) starts its
own N ranks: the parent, before it makes any GPU call, runs
`python -m torch.distributed.run --nproc-per-node N ... bench.py` as a child
process (the `mpiexec -n k` fan-out of ga.cpp:370-381), relays rank 0's JSON
line and exits with the children's return code. N above the visible GPUs fails
(rc 2) unless TTGA_BENCH_BACKEND=gloo asks for a rehearsal on fewer GPUs.
`--global-pop G` splits G individuals across the ranks (strong scaling, BASELINE
configs[4]); by default every rank evaluates --pop individuals (weak scaling).

TTGA_BENCH_FORCE_DIST=1 initialises the process group (RCCL) at world 1 too, so
the timing barrier and the MAX all-reduce run through RCCL on a one-GPU box
(tests/test_gpu_bench.py); the numbers are the same workload.

A step is one tt_eval over the rank's whole population. Rank 0 prints one JSON
line (BASELINE.json metric) with the dominant kernel's roofline and, at N=1, a
CPU baseline: the reference's own computeFeasibility/Hcv/Scv (oracle/_ref,
OpenMP over individuals on every core this job may use) timed on a bounded
sample of the same population. At N=1 the roofline's `traffic` and the LDS /
VALU / SALU busy fractions are measured live: before this process touches the
GPU, three short child runs of the same workload under `rocprofv3 --pmc`
(tools/pmc_live.py) read FETCH_SIZE, WRITE_SIZE and the SQ counters.
"""
from __future__ import annotations

import argparse
import ctypes
import json
import os
import pathlib
import sys
import time

import numpy as np

REPO = pathlib.Path(__file__).resolve().parent
sys.path.insert(0, str(REPO / "timetabling-ga-mpi-openmp_amd"))
sys.path.insert(0, str(REPO / "tests"))

METRIC = json.loads((REPO / "BASELINE.json").read_text())["metric"]
HBM_PEAK_GBS = 8000.0        # MI355X HBM3E spec (MI355X_MICROARCH.md)
POP_PER_GPU = 65536
SIZE_NAMES = {"sm": "small01-size", "med": "medium01-size", "lg": "large01-size",
              "syn": "synthetic 2000/40/10/5000 scaling instance"}
KERNELS = {2: "eval_block", 7: "eval_tile5", 8: "eval_tile5_w8", 13: "eval_lanes_w16+eval_corr"}


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=1000)
    ap.add_argument("--warmup", type=int, default=10)
    ap.add_argument("--warm-seconds", type=float, default=0.25,
                    help="keep warming up until this much wall time of launches has run")
    ap.add_argument("--pop", type=int, default=POP_PER_GPU, help="individuals per GPU (weak scaling)")
    ap.add_argument("--global-pop", type=int, default=0,
                    help="individuals over all ranks, split across them (strong scaling); overrides --pop")
    ap.add_argument("--config", default="med", choices=["sm", "med", "lg", "syn"])
    ap.add_argument("--variant", type=int, default=0, help="tt_eval kernel: 0 auto, 2 block, 7/8 tile5, 13 wide path")
    ap.add_argument("--cpu-sample", type=int, default=0,
                    help="individuals in the CPU-baseline sample (0: sized to about --cpu-seconds of CPU work)")
    ap.add_argument("--cpu-seconds", type=float, default=15.0)
    ap.add_argument("--no-cpu", action="store_true")
    ap.add_argument("--no-pmc", action="store_true", help="skip the live rocprofv3 counter passes")
    ap.add_argument("--pmc-child", action="store_true", help=argparse.SUPPRESS)
    args = ap.parse_args()
    if args.global_pop and args.global_pop < max(1, args.gpus):
        ap.error("--global-pop must be at least --gpus")
    return args


def _free_port() -> int:
    import socket
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def host_cores():
    """Cores this job may use (affinity, cgroup CPU quota), the machine's
    total and the CPU model (/proc/cpuinfo)."""
    total = os.cpu_count() or 1
    try:
        avail = len(os.sched_getaffinity(0))
    except AttributeError:
        avail = total
    try:
        q, per = open("/sys/fs/cgroup/cpu.max").read().split()[:2]
        if q != "max":
            avail = min(avail, max(1, -(-int(q) // int(per))))
    except (OSError, ValueError):
        pass
    model = "unknown"
    try:
        for ln in open("/proc/cpuinfo"):
            if ln.startswith("model name"):
                model = ln.split(":", 1)[1].strip()
                break
    except OSError:
        pass
    return avail, total, model


def cpu_baseline(inst, slot_np, room_np, gpu_out):
    """The reference's evaluation (oracle/_ref) or, without it, the oracle port."""
    threads, total, model = host_cores()
    from oracle_lib import oracle, ref
    n = slot_np.shape[0]
    hcv = np.zeros(n, np.int32); scv = np.zeros(n, np.int32)
    feas = np.zeros(n, np.uint8); pen = np.zeros(n, np.int32)
    R = ref()
    if R is not None:
        h = R.problem(inst)
        fn = R.lib.ref_eval_timed
        fn.restype = ctypes.c_double
        fn.argtypes = [ctypes.c_void_p] * 3 + [ctypes.c_int] * 2 + [ctypes.c_void_p] * 4
        P_ = lambda a: a.ctypes.data_as(ctypes.c_void_p)  # noqa: E731
        secs = fn(h.h, P_(slot_np), P_(room_np), n, threads, P_(hcv), P_(scv), P_(feas), P_(pen))
        kind, cores = "reference", threads
    else:
        o = oracle().problem(inst)
        t0 = time.perf_counter()
        hcv, scv, feas, pen = o.eval(slot_np, room_np)
        secs = time.perf_counter() - t0
        kind, cores = "port", 1
    agree = all(np.array_equal(a, b[:n]) for a, b in zip((hcv, scv, feas, pen), gpu_out))
    return {"value": n / secs, "unit": "evals/s", "cores": cores, "kind": kind,
            "sample": f"{n} individuals of the same population, computeFeasibility+computeHcv+computeScv+penalty, "
                      f"OpenMP dynamic over individuals, {secs:.2f} s", "matches_gpu": bool(agree),
            "cpu_model": model, "host_cores_total": total,
            "cores_note": "every core this job may use (affinity and cgroup quota); the GPU box grants one GPU's share"}


DOMINANT = {7: "eval_tile5_kernel", 8: "eval_tile5_kernel", 13: "eval_", 2: "eval_block_kernel"}   # kernel name substrings


def visible_gpus() -> int:
    """GPUs the ranks may use, counted in a short child process: importing
    torch maps the HIP runtime into a process, and the launcher parent must
    stay free of it (it only starts and relays the ranks)."""
    import subprocess
    r = subprocess.run([sys.executable, "-c", "import torch; print(torch.cuda.device_count())"],
                       capture_output=True, text=True, timeout=600)
    try:
        return int(r.stdout.strip().splitlines()[-1])
    except (ValueError, IndexError):
        return 0


def hip_mapped() -> bool:
    """Whether the HIP runtime library is mapped into this process."""
    try:
        with open("/proc/self/maps") as f:
            return any("libamdhip64" in ln for ln in f)
    except OSError:
        return False


def launch_ranks(args) -> int:
    """--gpus N > 1 with no launcher around us: run N ranks as child processes
    of torch.distributed.run (one rank per GPU, 127.0.0.1 rendezvous) and relay
    rank 0's JSON line. This process never touches the GPU."""
    n = args.gpus
    gpus = visible_gpus()
    rehearsal = os.environ.get("TTGA_BENCH_BACKEND", "nccl") == "gloo"
    if n > gpus and not rehearsal:
        print(f"bench.py: --gpus {n} but {gpus} GPU(s) visible; set TTGA_BENCH_BACKEND=gloo to rehearse "
              f"{n} ranks on fewer GPUs", file=sys.stderr, flush=True)
        return 2
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", str(n),
           "--master-addr", "127.0.0.1", "--master-port", str(_free_port()), str(REPO / "bench.py"), *sys.argv[1:]]
    import subprocess
    env = dict(os.environ)
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    launcher = {"pid": os.getpid(), "hip_mapped_before_launch": hip_mapped(), "visible_gpus": gpus}
    proc = subprocess.Popen(cmd, cwd=str(REPO), env=env, stdout=subprocess.PIPE, text=True)
    for ln in proc.stdout:                   # rank 0's line on stdout; anything else to stderr
        if ln.startswith("{"):
            try:
                d = json.loads(ln)
                d["launcher"] = launcher     # the parent's own record: it never loaded HIP
                ln = json.dumps(d) + "\n"
            except json.JSONDecodeError:
                pass
        (sys.stdout if ln.startswith("{") else sys.stderr).write(ln)
        sys.stdout.flush()
    return proc.wait()


def rank_share(args, rank: int, world: int):
    """(individuals of this rank, index of its first individual in the global
    population, global population)."""
    if args.global_pop > 0:
        base, extra = divmod(args.global_pop, world)
        p = base + (1 if rank < extra else 0)
        start = rank * base + min(rank, extra)
        return p, start, args.global_pop
    return args.pop, rank * args.pop, args.pop * world


def verify_shard(inst, slot, room, out, rows: int = 256) -> dict:
    """Checker, after the timed region: `rows` individuals of this rank's shard,
    evenly strided over it, re-evaluated by the CPU oracle (oracle/, test
    infrastructure) and compared field by field with the GPU's outputs."""
    from oracle_lib import host_threads, oracle, split_rows
    P = int(slot.shape[0])
    idx = np.unique(np.linspace(0, max(P - 1, 0), min(P, rows)).round().astype(np.int64))
    if idx.size == 0:
        return {"rows_checked": 0, "matches_oracle": True}
    import torch
    ti = torch.from_numpy(idx).to(slot.device)
    s_np, r_np = slot[ti].cpu().numpy(), room[ti].cpu().numpy()
    got = [o[ti].cpu().numpy() for o in out]
    exp = split_rows(oracle().problem(inst).eval, (s_np, r_np), threads=max(1, host_threads() // 2))
    names = ("hcv", "scv", "feasible", "penalty")
    bad = {n: int((g != e).sum()) for n, g, e in zip(names, got, exp) if not np.array_equal(g, e)}
    rec = {"rows_checked": int(idx.size), "matches_oracle": not bad}
    if bad:                                   # enough to tell a wrong kernel from a wrong read
        rows = np.nonzero(np.any([g != e for g, e in zip(got, exp)], axis=0))[0]
        k = int(rows[0])
        rec["mismatch"] = {"fields": bad, "rows": int(rows.size), "first_row": int(idx[k]),
                           "gpu": [int(g[k]) for g in got], "oracle": [int(e[k]) for e in exp]}
    return rec


def rank_record(rank: int, dev, kernel_ms: float, wall: float, P: int, first: int, check: dict) -> dict:
    """What one rank reports to rank 0: the device it bound (index and PCI
    location, so distinct ranks can be seen to use distinct GPUs), its kernel
    time, its shard and the oracle check of that shard."""
    import torch
    pr = torch.cuda.get_device_properties(dev)
    return {"rank": rank, "device": int(dev.index), "pci": f"{pr.pci_domain_id:04x}:{pr.pci_bus_id:02x}:{pr.pci_device_id:02x}",
            "uuid": str(getattr(pr, "uuid", "")), "host": os.uname().nodename, "kernel_ms": kernel_ms, "wall_s": wall,
            "pop": P, "first": first, **check}


def merge_ranks(records: list, backend: str, world: int) -> dict:
    """Rank 0's summary of every rank's record (all_gather_object)."""
    records = sorted(records, key=lambda r: r["rank"])
    locs = {(r["host"], r["pci"]) for r in records}
    return {"world": world, "backend": backend, "ranks_verified": sum(1 for r in records if r["matches_oracle"]),
            "rows_checked": sum(r["rows_checked"] for r in records), "distinct_devices": len(locs),
            "devices": [{k: r[k] for k in ("rank", "device", "pci", "uuid", "kernel_ms", "rows_checked",
                                           "matches_oracle", "mismatch") if k in r} for r in records]}


def main():
    args = parse()
    if args.gpus > 1 and "WORLD_SIZE" not in os.environ and not args.pmc_child:
        sys.exit(launch_ranks(args))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    P, first, global_pop = rank_share(args, rank, world)
    pmc = None
    if world == 1 and not args.no_pmc and not args.pmc_child:
        # live counters of the same workload, before this process initialises the GPU
        sys.path.insert(0, str(REPO / "tools"))
        import pmc_live
        v = args.variant or (8 if args.config != "syn" else 13)
        child = [str(REPO / "bench.py"), "--pmc-child", "--config", args.config, "--pop", str(P),
                 "--steps", "20", "--warmup", "2", "--variant", str(v)]
        # FETCH_SIZE read-factor calibration: the same kernel with its evaluation phases
        # off (tile5: lane and wave phase; wide path: eval_lanes only), which reads
        # exactly the P*E bytes of the slot rows with the kernel's own loads
        calib = list(child)
        calib[-1] = str(v | (0x30 if v in (7, 8) else 0x40 if v == 13 else 0))
        E = {"sm": 100, "syn": 2000}.get(args.config, 400)
        pmc = pmc_live.derive(pmc_live.collect(child, DOMINANT.get(v, "eval_"), calib if v in (7, 8, 13) else None),
                              calib_bytes=float(P) * E)
    import torch
    import torch.distributed as dist

    import ttga
    from ttga import native

    # one rank per GPU; LOCAL_RANK modulo the visible GPUs and TTGA_BENCH_BACKEND=gloo
    # let a one-GPU box rehearse the N > 1 path (RCCL needs distinct GPUs)
    local = int(os.environ.get("LOCAL_RANK", "0")) % max(1, torch.cuda.device_count())
    backend = os.environ.get("TTGA_BENCH_BACKEND", "nccl")
    if backend == "nccl" and world > max(1, torch.cuda.device_count()):
        # more ranks than GPUs: RCCL refuses two ranks on one device ("Duplicate GPU
        # detected"), so the rehearsal takes gloo (the line says so in config.rehearsal)
        backend = "gloo"
    use_dist = world > 1 or os.environ.get("TTGA_BENCH_FORCE_DIST", "") not in ("", "0")
    if use_dist and world == 1:
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        os.environ.setdefault("MASTER_PORT", str(_free_port()))
        os.environ.setdefault("RANK", "0")
        os.environ.setdefault("WORLD_SIZE", "1")
    if use_dist:
        torch.cuda.set_device(local)
        if backend == "nccl":
            dist.init_process_group("nccl", device_id=torch.device("cuda", local))
        else:
            dist.init_process_group(backend)
        if dist.get_world_size() != world:            # n_gpus is what the process group holds
            raise SystemExit(f"bench.py: WORLD_SIZE {world} but the process group has {dist.get_world_size()} ranks")
    dev = torch.device("cuda", local)
    torch.cuda.set_device(dev)

    inst = ttga.config_instance(args.config)
    dp = native.DeviceProblem(inst, device=local)
    E = inst.E
    # synthetic population: RandomInitialSolution per individual (seed base 12345 + global index),
    # canonical rooms from the matcher; setup, not timed
    seeds = torch.from_numpy(ttga.population_seeds(12345 + first, P)).to(dev)
    slot = torch.empty((P, E), dtype=torch.uint8, device=dev)
    room = torch.empty_like(slot)
    dp.random_init(seeds, slot, room)
    out = (torch.empty(P, dtype=torch.int32, device=dev), torch.empty(P, dtype=torch.int32, device=dev),
           torch.empty(P, dtype=torch.uint8, device=dev), torch.empty(P, dtype=torch.int32, device=dev))
    torch.cuda.synchronize(dev)

    # warm-up: W launches, then more until >= WARM_S of launches have run, so the
    # timed steps see settled clocks (outside the timed region)
    t_w = time.perf_counter()
    launched = 0
    while launched < args.warmup or time.perf_counter() - t_w < args.warm_seconds:
        for _ in range(max(1, min(args.warmup, 50)) if launched < args.warmup else 50):
            dp.eval(slot, room, variant=args.variant, out=out)
            launched += 1
        torch.cuda.synchronize(dev)

    stream = torch.cuda.current_stream(dev)      # tt_eval launches its one kernel on this stream
    ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    if use_dist:
        dist.barrier()
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    ev0.record(stream)
    for _ in range(args.steps):
        dp.eval(slot, room, variant=args.variant, out=out)
    ev1.record(stream)
    torch.cuda.synchronize(dev)
    if use_dist:
        dist.barrier()
    wall = time.perf_counter() - t0
    kernel_ms = ev0.elapsed_time(ev1) / args.steps

    t = torch.tensor([wall], dtype=torch.float64, device=dev if backend == "nccl" else "cpu")
    if use_dist:
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
    wall_max = float(t.item())

    if args.pmc_child:
        return
    ranks = None
    if use_dist:
        # every rank checks its own shard against the oracle (outside the timed region) and
        # reports its device; rank 0 puts the gathered records into the line
        rec = rank_record(rank, dev, kernel_ms, wall, P, first, verify_shard(inst, slot, room, out))
        recs = [None] * dist.get_world_size()
        dist.all_gather_object(recs, rec)
        ranks = merge_ranks(recs, dist.get_backend(), dist.get_world_size())
    if rank == 0:
        total = global_pop * args.steps
        value = total / wall_max
        strong = args.global_pop > 0
        ncu = torch.cuda.get_device_properties(dev).multi_processor_count    # CUs (256 on a whole MI355X)
        bytes_per_eval = 2 * E + 13                     # u8 slot+room in; i32 hcv,scv,penalty + u8 feasible out
        achieved = bytes_per_eval * P / (kernel_ms * 1e-3) / 1e9
        variant = args.variant or dp.eval_variant()
        line = {
            "metric": METRIC, "value": value, "unit": "evals/s", "n_gpus": world, "steps": args.steps,
            "warmup": args.warmup, "warmup_launches": launched, "ms_per_step": wall_max / args.steps * 1e3, "higher_is_better": True,
            "scaling": "strong" if strong else "weak", "vs_baseline": None, "dtype": "i32", "data": "synthetic",
            "config": {"workload": f"{args.config} instance E={E} R={inst.R} F={inst.F} S={inst.S} (seeded synthetic, "
                                   f"{SIZE_NAMES[args.config]}), "
                                   + (f"global population {global_pop} split over {world} GPU(s)" if strong
                                      else f"population {P} per GPU")
                                   + ", one tt_eval (hcv+scv+feasible+penalty) per step",
                       "pop_per_gpu": P, "global_pop": global_pop,
                       "kernel": KERNELS[variant],
                       "parallelism": f"dp{world} (independent population shards)"},
            "roofline": {"bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                         "frac": achieved / HBM_PEAK_GBS,
                         "traffic": None if pmc is None else pmc["traffic_bytes"],
                         "traffic_unit": "bytes per launch (FETCH_SIZE x calibrated read factor + WRITE_SIZE, "
                                         "live rocprofv3 passes; see traffic_detail)",
                         "algorithmic_bytes": bytes_per_eval * P,
                         "kernel_ms": kernel_ms, "bytes_per_eval": bytes_per_eval},
        }
        if world > torch.cuda.device_count():
            line["config"]["rehearsal"] = (f"{world} ranks on {torch.cuda.device_count()} GPU(s), {backend} "
                                           f"process group: checks the multi-rank path, not a scaling number")
        if pmc is not None:
            line["roofline"]["traffic_detail"] = {k: pmc.get(k) for k in ("fetch_kib", "write_kib", "fetch_factor",
                                                                          "fetch_factor_how", "calib_fetch_kib",
                                                                          "calib_bytes")}
            line["roofline"]["pipes"] = {k: pmc[k] for k in ("lds_busy", "lds_conflict", "valu_busy", "salu_busy",
                                                            "wait_any", "cycles") if k in pmc}
            raw = pmc.get("raw", {})
            if "SQ_LDS_IDX_ACTIVE" in raw and pmc.get("cycles"):
                # the units that bind these kernels are the VALU and the LDS (and the issue
                # around them), not HBM: each unit's busy cycles against its issue peak --
                # one LDS-array cycle per CU per shader cycle, and 4 SIMD cycles per wave64
                # VALU instruction (one per CU per cycle: tools/valu_rate) -- the busier one
                # is the binding unit
                clk = pmc["cycles"] / (kernel_ms * 1e-3)
                units = {"lds": {"cycles_per_individual": raw["SQ_LDS_IDX_ACTIVE"] / P,
                                 "frac": pmc.get("lds_busy"), "bank_conflict_share": pmc.get("lds_conflict"),
                                 "only_us": raw["SQ_LDS_IDX_ACTIVE"] / (ncu * clk) * 1e6,
                                 "peak": "1 LDS-array cycle per CU per shader cycle (MI355X_MICROARCH.md §LDS)"}}
                if "SQ_INSTS_VALU" in raw:
                    units["valu"] = {"instructions_per_individual": raw["SQ_INSTS_VALU"] / P,
                                     "frac": pmc.get("valu_busy"),
                                     "only_us": raw["SQ_INSTS_VALU"] / (ncu * clk) * 1e6,
                                     "peak": "1 wave64 VALU instruction per CU per shader cycle (4 SIMDs x 4 cycles; "
                                             "tools/valu_rate, profiles/r04_j_valu_rate.json)"}
                bind = max(units, key=lambda k: units[k]["frac"] or 0.0)
                line["roofline"]["binding_unit"] = {
                    "unit": bind, "frac": units[bind]["frac"], "units": units,
                    "lds_cycles_per_individual": raw["SQ_LDS_IDX_ACTIVE"] / P,
                    "valu_frac": pmc.get("valu_busy"), "salu_frac": pmc.get("salu_busy"),
                    "clock_ghz": clk / 1e9}
        if variant == 13 and not args.pmc_child:
            # the wide path's lane phase alone (eval_lanes: variant bit 6 skips eval_corr), on
            # the LDS byte-gather roofline: one ds_read_u8 per (individual, student id), 64 per
            # wave-instruction in 2 LDS cycles (32 banks) = 32 lookups per CU per shader cycle
            lookups = float(sum(n + (n & 1) for n in inst.student_events.sum(axis=1).tolist()))
            ea, eb = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            ea.record(stream)
            for _ in range(5):
                dp.eval(slot, room, variant=13 | (4 << 4), out=out)
            eb.record(stream)
            torch.cuda.synchronize(dev)
            lanes_ms = ea.elapsed_time(eb) / 5
            dp.eval(slot, room, variant=args.variant, out=out)        # restore the full outputs
            torch.cuda.synchronize(dev)
            clk = pmc["cycles"] / (kernel_ms * 1e-3) if pmc and pmc.get("cycles") else 2.4e9
            rate = P * lookups / (lanes_ms * 1e-3)
            line["roofline"]["lane_phase"] = {
                "kernel": "eval_lanes_w16", "kernel_ms": lanes_ms, "lookups_per_individual": lookups,
                "lookups_per_s": rate, "peak_lookups_per_s": 32 * ncu * clk,
                "frac": rate / (32 * ncu * clk), "clock_ghz": clk / 1e9,
                "peak_note": "ds_read_u8: 64 lanes in 2 LDS cycles (32 banks) per CU; clock from the live pass"}
        if world == 1 and not args.no_cpu:
            n = args.cpu_sample
            if n <= 0:      # calibrate on a small slice, then size the sample to ~cpu_seconds
                n0 = min(P, 256)
                c = cpu_baseline(inst, slot[:n0].cpu().numpy(), room[:n0].cpu().numpy(),
                                 [o[:n0].cpu().numpy() for o in out])
                n = int(max(n0, min(P, c["value"] * args.cpu_seconds)))
            n = min(max(n, 2048), P)              # at least 2,048 individuals
            s_np, r_np = slot[:n].cpu().numpy(), room[:n].cpu().numpy()
            gpu_out = [o[:n].cpu().numpy() for o in out]
            line["cpu_baseline"] = cpu_baseline(inst, s_np, r_np, gpu_out)
        if use_dist and world == 1:
            line["config"]["process_group"] = f"{backend} at world 1 (TTGA_BENCH_FORCE_DIST)"
        if ranks is not None:
            line["ranks"] = ranks
        print(json.dumps(line), flush=True)
    if use_dist:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
