"""Host logic of the GA driver (no GPU): Control-style CLI, rank seeds, the
reference's JSON line format, and the island-model communication over gloo
with world_size 2 (ring migration ga.cpp:479-540, MIN reduce ga.cpp:234-257)."""
import io
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from ttga.ga import json_line, max_steps_for, stream_seeds
from ttga.islands import global_min, parse_control, rank_seed, ring_migrate


def test_control_parsing_and_messages():
    out, err = io.StringIO(), io.StringIO()
    c = parse_control(["-i", "x.tim", "-s", "42", "-p", "2", "-c", "4", "-p3", "0.5", "--pop", "16"], out, err)
    assert c["input"] == "x.tim" and c["seed"] == 42 and c["problem_type"] == 2 and c["threads"] == 4
    assert c["p3"] == 0.5 and c["pop"] == 16
    assert "Max number of threads 4" in out.getvalue() and "Problem instance type 2" in out.getvalue()
    assert "Warning: No output file given, writing to stdout" in err.getvalue()
    with pytest.raises(SystemExit):
        parse_control(["-i"], io.StringIO(), io.StringIO())
    with pytest.raises(SystemExit):
        parse_control(["-s", "1"], io.StringIO(), io.StringIO())


def test_max_steps_and_seeds():
    assert [max_steps_for(p) for p in (1, 2, 3, 0)] == [200, 1000, 2000, 2000]
    # ga.cpp:412 abs(seed + i*(seed/10)) with C division
    assert rank_seed(42, 0) == 42 and rank_seed(42, 3) == 54 and rank_seed(-42, 1) == 46
    s = stream_seeds(7, 0, 3)
    assert list(s) == [8, 9, 10] and all(s > 0)


def test_json_line_matches_jsoncpp_format():
    # format probed from the reference's jsoncpp (indentation "", keys sorted, %.17g)
    line = json_line({"solution": {"threadID": 0, "totalTime": 1.25, "totalBest": 7, "feasible": True,
                                   "timeslots": [3, 44], "procID": 0}})
    assert line == '{"solution":{"feasible":true,"procID":0,"threadID":0,"timeslots":[3,44],"totalBest":7,"totalTime":1.25}}'
    assert json_line({"logEntry": {"procID": 0, "threadID": 1, "best": 12, "time": 0.1}}) == \
        '{"logEntry":{"best":12,"procID":0,"threadID":1,"time":0.10000000000000001}}'


def host_island(g, N=6, E=5):
    """A real ttga.ga.Members population on CPU tensors (the same pack /
    unpack_into payload code the device islands use), distinct per island g."""
    from ttga.ga import Members, new_population
    pop = new_population(N, E, torch.device("cpu"))
    for k in range(N):
        pop["slot"][k] = torch.tensor([(g * 61 + k * 11 + e) % 45 for e in range(E)], dtype=torch.uint8)
        pop["room"][k] = torch.tensor([(g * 7 + k + e) % 10 for e in range(E)], dtype=torch.uint8)
        pop["hcv"][k] = g * 100 + k
        pop["scv"][k] = 1000 + g * 10 + k
        pop["feasible"][k] = (g + k) % 2
        pop["penalty"][k] = 1000000 * ((g + k) % 2 == 0) + 7 * k + g
    return Members(pop)


def snapshot(isl):
    return [isl.pack(k).numpy().copy() for k in range(isl.N)]


def _worker(rank, world, K, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    isl = [host_island(rank * K + k) for k in range(K)]
    before = [snapshot(i) for i in isl]
    ring_migrate(isl, rank, world, backend="gloo")
    m = global_min(1000 + 7 * (world - rank), torch.device("cpu"), world, backend="gloo")
    q.put((rank, before, [snapshot(i) for i in isl], m))
    dist.barrier()
    dist.destroy_process_group()


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def test_ring_migration_local_islands():
    """K islands in one process: the ring is local copies (world 1)."""
    K = 4
    isl = [host_island(g) for g in range(K)]
    before = [snapshot(i) for i in isl]
    ring_migrate(isl, 0, 1)
    N = isl[0].N
    for g in range(K):
        after = snapshot(isl[g])
        assert np.array_equal(after[N - 1], before[(g - 1) % K][0])
        assert np.array_equal(after[N - 2], before[(g + 1) % K][1])
        assert all(np.array_equal(after[k], before[g][k]) for k in range(N - 2))
    # unpack restores every field of the payload
    m = isl[1].member(N - 1)
    assert (m["hcv"], m["scv"], m["penalty"]) == (0, 1000, 1000000)


@pytest.mark.parametrize("world,K", [(2, 1), (3, 1), (2, 3)])
def test_ring_migration_gloo(world, K):
    """world ranks x K islands each, real Members payloads over gloo."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, K, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    before, after = {}, {}
    for _ in range(world):
        r, b, a, m = q.get(timeout=120)
        assert m == 1007                                        # MIN over ranks
        for k in range(K):
            before[r * K + k], after[r * K + k] = b[k], a[k]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    W = world * K
    N = len(before[0])
    for g in range(W):
        assert np.array_equal(after[g][N - 1], before[(g - 1) % W][0])    # best of the left neighbour
        assert np.array_equal(after[g][N - 2], before[(g + 1) % W][1])    # 2nd best of the right neighbour
        assert all(np.array_equal(after[g][k], before[g][k]) for k in range(N - 2))


class _Landed:
    """An event whose copy has already landed (Snapshot.values waits on it)."""

    def synchronize(self):
        pass


def test_snapshot_log_values_and_best_thread():
    """ttga.islands logs a generation from Island.snapshot's pinned copy: the
    fields come back as (feasible, scv, hcv, thread), the thread being child c
    of the last replacement when pop[0] came from child slot N - C + c, else 0
    (also before the first generation); CostLog.update_from writes the same
    line CostLog.offer would."""
    from ttga.ga import CostLog, Snapshot
    N, C = 10, 4
    k = N - C
    s = Snapshot(torch.tensor([1, 37, 0, k + 2], dtype=torch.int32), _Landed(), 3, k, N)
    assert s.values() == (True, 37, 0, 2)
    assert Snapshot(torch.tensor([0, 5, 9, 1], dtype=torch.int32), _Landed(), 3, k, N).values() == (False, 5, 9, 0)
    assert Snapshot(torch.tensor([1, 5, 0, k], dtype=torch.int32), _Landed(), 0, k, N).values()[3] == 0
    out_a, out_b = io.StringIO(), io.StringIO()
    a, b = CostLog(3, out_a, 0.0), CostLog(3, out_b, 0.0)
    a.offer(True, 37, 0, 2, t=0.5)
    b.offer(*s.values(), t=0.5)
    assert out_a.getvalue() == out_b.getvalue() != ""
