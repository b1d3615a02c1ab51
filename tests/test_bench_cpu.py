"""bench.py's host logic without a GPU: the rank fan-out refuses more ranks
than visible GPUs (unless a gloo rehearsal is asked for) before any GPU call,
and --global-pop splits the population exactly (strong scaling)."""
import os
import pathlib
import subprocess
import sys
import types

REPO = pathlib.Path(__file__).resolve().parent.parent
sys.path.insert(0, str(REPO))

import bench  # noqa: E402


def test_rank_share_weak_and_strong():
    weak = types.SimpleNamespace(global_pop=0, pop=65536)
    assert [bench.rank_share(weak, r, 4) for r in range(4)] == [(65536, r * 65536, 4 * 65536) for r in range(4)]
    for world in (1, 2, 3, 4, 7, 8):
        strong = types.SimpleNamespace(global_pop=262144 + 5, pop=65536)
        parts = [bench.rank_share(strong, r, world) for r in range(world)]
        assert sum(p for p, _, _ in parts) == 262149
        assert all(g == 262149 for _, _, g in parts)
        # contiguous, non-overlapping shards in rank order
        assert [s for _, s, _ in parts] == [sum(p for p, _, _ in parts[:r]) for r in range(world)]
        assert max(p for p, _, _ in parts) - min(p for p, _, _ in parts) <= 1


def test_gpus_above_visible_fails_loudly():
    """No GPU here: --gpus 2 must fail with rc 2 from the parent (no rank started)."""
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "TTGA_BENCH_BACKEND")}
    r = subprocess.run([sys.executable, "bench.py", "--gpus", "2", "--no-pmc", "--no-cpu", "--steps", "1"],
                       cwd=REPO, capture_output=True, text=True, timeout=240, env=env)
    assert r.returncode == 2, (r.returncode, r.stderr[-2000:])
    assert "GPU(s) visible" in r.stderr and r.stdout.strip() == ""


def test_global_pop_below_ranks_rejected():
    r = subprocess.run([sys.executable, "bench.py", "--gpus", "4", "--global-pop", "3"],
                       cwd=REPO, capture_output=True, text=True, timeout=240)
    assert r.returncode != 0 and "--global-pop" in r.stderr


def _verify_rank(rank, world, port, q):
    """One gloo rank of the N > 1 bench path's check: its shard (CPU tensors
    standing in for device memory) verified against the oracle, the records
    all-gathered as the bench does and merged on rank 0."""
    import numpy as np
    import torch
    import torch.distributed as dist
    import ttga
    from oracle_lib import oracle
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    inst = ttga.config_instance("sm")
    o = oracle().problem(inst)
    P = 600
    s, r, _ = o.random_init(ttga.population_seeds(100 + 1000 * rank, P))
    out = [torch.from_numpy(x.copy()) for x in o.eval(s, r)]
    if rank == 1:
        out[1][599] += 1                      # the last row of rank 1's shard is wrong
    chk = bench.verify_shard(inst, torch.from_numpy(s), torch.from_numpy(r), out)
    rec = {"rank": rank, "device": 0, "pci": f"0000:{rank:02x}:00", "uuid": "", "host": "h", "kernel_ms": 1.0,
           "wall_s": 1.0, "pop": P, "first": rank * P, **chk}
    recs = [None] * world
    dist.all_gather_object(recs, rec)
    if rank == 0:
        q.put(bench.merge_ranks(recs, dist.get_backend(), dist.get_world_size()))
    dist.destroy_process_group()


def test_rank_verification_gloo_world2():
    """The N > 1 bench line's self-check on two gloo ranks: each rank checks 256
    strided rows of its shard (first and last row included) against the oracle;
    rank 0's summary counts the ranks that matched and the distinct devices."""
    import socket
    import torch.multiprocessing as mp
    with socket.socket() as sk:
        sk.bind(("127.0.0.1", 0))
        port = sk.getsockname()[1]
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_verify_rank, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    m = q.get(timeout=240)
    for p in procs:
        p.join(60)
        assert p.exitcode == 0
    assert m["world"] == 2 and m["backend"] == "gloo" and m["distinct_devices"] == 2
    assert m["ranks_verified"] == 1 and m["rows_checked"] == 512
    assert [d["matches_oracle"] for d in m["devices"]] == [True, False]
    bad = m["devices"][1]["mismatch"]
    assert bad["fields"] == {"scv": 1} and bad["rows"] == 1 and bad["first_row"] == 599
    assert bad["gpu"][1] == bad["oracle"][1] + 1 and "mismatch" not in m["devices"][0]
