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


class FakeIsland:
    """CPU stand-in with the Island migration interface (pack / unpack_into)."""

    def __init__(self, rank, N=6, E=5):
        self.N, self.E = N, E
        self.rows = torch.tensor([[(rank * 61 + k * 11 + e) % 256 for e in range(2 * E + 16)] for k in range(N)],
                                 dtype=torch.uint8)

    def pack(self, k):
        return self.rows[k].clone()

    def unpack_into(self, pos, buf):
        self.rows[pos].copy_(buf)


def _worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    isl = FakeIsland(rank)
    before = isl.rows.clone()
    ring_migrate(isl, rank, world)
    m = global_min(1000 + 7 * (world - rank), torch.device("cpu"), world)
    q.put((rank, before.numpy(), isl.rows.numpy(), m))
    dist.barrier()
    dist.destroy_process_group()


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


@pytest.mark.parametrize("world", [2, 3])
def test_ring_migration_gloo(world):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = {}
    for _ in range(world):
        r, before, after, m = q.get(timeout=120)
        res[r] = (before, after, m)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    N = res[0][0].shape[0]
    for r in range(world):
        before, after, m = res[r]
        left, right = (r - 1) % world, (r + 1) % world
        assert np.array_equal(after[N - 1], res[left][0][0])    # best of the left neighbour
        assert np.array_equal(after[N - 2], res[right][0][1])   # 2nd best of the right neighbour
        assert np.array_equal(after[:N - 2], before[:N - 2])
        assert m == 1007                                        # MIN over ranks
