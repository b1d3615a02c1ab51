"""The BASELINE.json configurations on the GPU against the CPU oracle:

* large01-size (lg 400/10/10/400) and the twenty ITC-2002-size instances
  comp01..comp20: derived data, RandomInitialSolution, evaluation and
  localSearch(200) bit-exact;
* the island model (ga.cpp:479-540, 234-257) with 8 lg islands multiplexed on
  one GPU through the real Island pack / unpack / ring code, through the first
  migration (before generation 49), against an oracle island model built from
  the oracle's GA primitives; the Python and native drivers with 8 islands on
  one GPU print the same JSON lines; two ranks over gloo (one GPU) equal one
  process with the same islands.
"""
import json
import os
import pathlib
import socket
import subprocess
import sys

import numpy as np
import pytest

import ttga
from oracle_lib import oracle

pytestmark = pytest.mark.gpu
torch = pytest.importorskip("torch")
from ttga import native  # noqa: E402
from ttga.ga import Island, stream_seeds  # noqa: E402
from ttga.instance import comp_dims  # noqa: E402
from ttga.islands import broadcast_population, rank_seed, ring_migrate  # noqa: E402

REPO = pathlib.Path(__file__).resolve().parent.parent
KEYS = ("slot", "room", "hcv", "scv", "feasible", "penalty")
CONFIGS = ["lg"] + [f"comp{k:02d}" for k in range(1, 21)]


def dev(a):
    return torch.from_numpy(np.ascontiguousarray(a)).cuda()


def host(t):
    torch.cuda.synchronize()
    return t.cpu().numpy()


@pytest.fixture(scope="module")
def orc():
    return oracle()


@pytest.mark.parametrize("name", CONFIGS)
def test_config_instance_vs_oracle(orc, name):
    inst = ttga.config_instance(name)
    if name.startswith("comp"):
        E, R, F, S = comp_dims(int(name[4:]))
        assert (inst.E, inst.R, inst.F, inst.S) == (E, R, F, S) and 350 <= E <= 440 and R in (10, 11)
    dp = native.DeviceProblem(inst)
    o = orc.problem(inst)
    for a, b in zip(dp.derived(), o.derived()):
        assert np.array_equal(a, b)
    P = 48
    seeds = ttga.population_seeds(5000 + inst.E, P)
    es, er, eg = o.random_init(seeds)
    g = dev(seeds)
    s = torch.empty((P, inst.E), dtype=torch.uint8, device="cuda")
    r = torch.empty_like(s)
    dp.random_init(g, s, r)
    assert np.array_equal(host(s), es) and np.array_equal(host(r), er) and np.array_equal(host(g), eg)
    for got, want in zip(dp.eval(s, r), o.eval(es, er)):
        assert np.array_equal(host(got), want)
    n = 16
    ls_seeds = ttga.population_seeds(6000 + inst.E, n)
    s2, r2, g2 = dev(es[:n]), dev(er[:n]), dev(ls_seeds)
    dp.local_search(s2, r2, g2, 200)
    xs, xr, xg = o.local_search(es[:n], er[:n], ls_seeds, 200)
    assert np.array_equal(host(s2), xs) and np.array_equal(host(r2), xr) and np.array_equal(host(g2), xg)
    for got, want in zip(dp.eval(s2, r2), o.eval(xs, xr)):
        assert np.array_equal(host(got), want)
    assert dp.status() == 0


def test_local_search_bound_never_fires(orc):
    """The defensive visit bound of local_search_kernel (status bit 2) is never
    reached: zero budgets, move probabilities 0 and phase-2 runs included."""
    inst = ttga.config_instance("sm")
    dp = native.DeviceProblem(inst)
    o = orc.problem(inst)
    P = 32
    s0, r0, _ = o.random_init(ttga.population_seeds(77, P))
    for steps, p1, p2, p3 in ((0, 1.0, 1.0, 0.0), (200, 0.0, 0.0, 0.0), (50, 0.0, 1.0, 0.0), (3000, 1.0, 1.0, 0.0),
                              (3000, 0.3, 0.0, 0.2)):
        seeds = ttga.population_seeds(88 + steps, P)
        s, r, g = dev(s0), dev(r0), dev(seeds)
        dp.local_search(s, r, g, steps, p1, p2, p3)
        es, er, eg = o.local_search(s0, r0, seeds, steps, p1, p2, p3)
        assert np.array_equal(host(s), es) and np.array_equal(host(r), er) and np.array_equal(host(g), eg)
        assert dp.status() == 0


def test_invalid_genome_ranks_last(orc):
    """tt_eval's -1 sentinel (an invalid genome, which the reference cannot
    produce) sorts after every valid member and never wins selection5."""
    inst = ttga.config_instance("sm")
    dp = native.DeviceProblem(inst)
    o = orc.problem(inst)
    N, C = 12, 4
    rng = np.random.default_rng(3)
    pop = dict(slot=rng.integers(0, 45, (N, inst.E), dtype=np.uint8),
               room=rng.integers(0, inst.R, (N, inst.E), dtype=np.uint8),
               hcv=np.arange(N, dtype=np.int32), scv=np.arange(N, dtype=np.int32),
               feasible=np.zeros(N, np.uint8), penalty=(1000000 + np.arange(N)).astype(np.int32))
    pop["penalty"][[0, 3]] = -1
    ch = {k: v[:C].copy() for k, v in pop.items()}
    ch["penalty"][:] = [5, -1, 7, 1000003]
    exp = o.ga_replace(pop, ch)
    assert list(exp["penalty"][-3:]) == [-1, -1, -1]
    gpop = {k: dev(v) for k, v in pop.items()}
    dp.ga_replace(gpop, {k: dev(v) for k, v in ch.items()}, dp.ga_work(N))
    for k in KEYS:
        assert np.array_equal(host(gpop[k]), exp[k]), k
    pen = (1000000 + np.arange(N)).astype(np.int32)
    pen[[0, 3]] = -1                 # the two best positions hold invalid genomes
    seeds = stream_seeds(9, N, 64)
    cs, cr, fl, g = o.ga_breed(pop["slot"], pop["room"], pen, seeds, 64, 0.0, 0.0, 1)
    for bad in (0, 3):               # copies only (p_cross = p_mut = 0): never of an invalid member
        assert not (cs == pop["slot"][bad][None]).all(axis=1).any()
    gs, gr = dev(np.zeros((64, inst.E), np.uint8)), dev(np.zeros((64, inst.E), np.uint8))
    gf, grng = dev(np.zeros(64, np.uint8)), dev(seeds)
    dp.ga_breed(dev(pop["slot"]), dev(pop["room"]), dev(pen), grng, gs, gr, gf, 0.0, 0.0, True)
    assert np.array_equal(host(gs), cs) and np.array_equal(host(grng), g)


# ---------------------------------------------------------------- island model
def oracle_population(o, N, seed, steps):
    s, r, g = o.random_init(stream_seeds(seed, 0, N))
    s, r, g = o.local_search(s, r, g, steps)
    h, sc, f, p = o.eval(s, r)
    pop = dict(slot=s, room=r, hcv=h, scv=sc, feasible=f, penalty=p)
    return o.ga_replace(pop, {k: v[:0] for k, v in pop.items()})


def oracle_islands(o, W, N, C, gens, seed, steps):
    """The island model restated over the oracle's primitives: island g has
    seed abs(seed + g*(seed/10)) (ga.cpp:412) and starts from island 0's
    initial population (ga.cpp:429-444); before generations with
    (gen+1) % 100 == 50 island g's best replaces pop[N-1] of island g+1 and its
    2nd best pop[N-2] of island g-1 (ga.cpp:514-540)."""
    seeds = [rank_seed(seed, g) for g in range(W)]
    pop0 = oracle_population(o, N, seeds[0], steps)
    pops = [{k: v.copy() for k, v in pop0.items()} for _ in range(W)]
    rngs = [stream_seeds(seeds[g], N, C) for g in range(W)]
    migrations = 0
    for gen in range(gens):
        if (gen + 1) % 100 == 50:
            best = [{k: v[0].copy() for k, v in p.items()} for p in pops]
            second = [{k: v[1].copy() for k, v in p.items()} for p in pops]
            for g in range(W):
                for k in KEYS:
                    pops[g][k][N - 1] = best[(g - 1) % W][k]
                    pops[g][k][N - 2] = second[(g + 1) % W][k]
            migrations += 1
        for g in range(W):
            p = pops[g]
            cs, cr, fl, rngs[g] = o.ga_breed(p["slot"], p["room"], p["penalty"], rngs[g], C, 0.8, 0.5, 1)
            cs, cr, rngs[g] = o.local_search(cs, cr, rngs[g], steps)
            h, sc, f, pe = o.eval(cs, cr)
            pops[g] = o.ga_replace(p, dict(slot=cs, room=cr, hcv=h, scv=sc, feasible=f, penalty=pe))
    return pops, rngs, migrations


def test_eight_islands_lg_vs_oracle(orc):
    """BASELINE configs[3]: 8 islands on the lg instance, multiplexed on one GPU
    (the ring is local device copies through Island.pack / unpack_into),
    through the first migration; every island's population and streams are
    bit-exact with the oracle island model, and migrants arrived."""
    inst = ttga.config_instance("lg")
    dp = native.DeviceProblem(inst)
    o = orc.problem(inst)
    W, N, C, gens, seed, steps = 8, 10, 2, 54, 42, 200
    islands = [Island(dp, pop_size=N, children=C, max_steps=steps, seed=rank_seed(seed, g)) for g in range(W)]
    islands[0].initialize()
    broadcast_population(islands, 1)
    mig = 0
    for gen in range(gens):
        if (gen + 1) % 100 == 50:
            before = [(host(i.pop["slot"][0]).copy(), host(i.pop["slot"][1]).copy()) for i in islands]
            ring_migrate(islands, 0, 1)
            for g in range(W):
                assert np.array_equal(host(islands[g].pop["slot"][N - 1]), before[(g - 1) % W][0])
                assert np.array_equal(host(islands[g].pop["slot"][N - 2]), before[(g + 1) % W][1])
            mig += 1
        for isl in islands:
            isl.step()
    pops, rngs, omig = oracle_islands(o, W, N, C, gens, seed, steps)
    assert mig == omig == 1
    for g in range(W):
        for k in KEYS:
            assert np.array_equal(host(islands[g].pop[k]), pops[g][k]), (g, k)
        assert np.array_equal(host(islands[g].rng_child), rngs[g]), g
    assert dp.status() == 0


def test_islands_on_streams_match_serial_comp01():
    """Islands multiplexed on one GPU, each on a stream of its own (ttga.islands
    --islands K, tools/bench_ga.py --islands K) with their generations enqueued
    back to back so the launches overlap, end bit-identical to the same islands
    stepped one after another on torch's current stream: 8,192-child generations
    (LPT dispatch, the small-task + redo local search) with a migration between."""
    inst = ttga.config_instance("comp01")
    dp = native.DeviceProblem(inst)
    W, N, C, gens, seed, steps = 3, 8192, 4096, 4, 42, 200
    runs = []
    for streamed in (False, True):
        isl = [Island(dp, pop_size=N, children=C, max_steps=steps, seed=rank_seed(seed, g),
                      stream=torch.cuda.Stream() if streamed else None) for g in range(W)]
        isl[0].initialize()
        torch.cuda.synchronize()
        broadcast_population(isl, 1)
        torch.cuda.synchronize()
        for gen in range(gens):
            if gen == 2:
                torch.cuda.synchronize()
                ring_migrate(isl, 0, 1)
                torch.cuda.synchronize()
            for i in isl:
                i.step()
        torch.cuda.synchronize()
        runs.append([{k: host(i.pop[k]).copy() for k in KEYS} | {"rng": host(i.rng_child).copy(),
                                                                 "best": i.best_thread()} for i in isl])
    for g in range(W):
        for k in runs[0][g]:
            assert np.array_equal(runs[0][g][k], runs[1][g][k]), (g, k)
    assert dp.status() == 0


def _lines(text):
    """JSON lines with wall-clock fields removed, grouped per procID in order."""
    per, other = {}, []
    for ln in text.splitlines():
        if not ln.startswith("{"):
            continue
        obj = json.loads(ln)
        for v in obj.values():
            v.pop("time", None)
            v.pop("totalTime", None)
        body = next(iter(obj.values()))
        if "procID" in body:
            per.setdefault(body["procID"], []).append(obj)
        else:
            other.append(obj)
    return per, other


def _env():
    return dict(os.environ, PYTHONPATH=str(REPO / "timetabling-ga-mpi-openmp_amd"))


def test_islands_drivers_multiplexed_lg(tmp_path, orc):
    """`python -m ttga.islands --islands 8` and `ttga-ga --islands 8` (eight lg
    islands on one GPU, one migration) print the same JSON lines per island;
    every feasible printed timetable re-evaluates to its totalBest."""
    inst = ttga.config_instance("lg")
    tim = tmp_path / "lg.tim"
    ttga.write_tim(inst, tim)
    args = ["-i", str(tim), "-s", "42", "-p", "1", "-c", "2", "--islands", "8", "--generations", "54"]
    py = subprocess.run([sys.executable, "-m", "ttga.islands", *args], capture_output=True, text=True, timeout=300,
                        env=_env(), cwd=str(tmp_path))
    assert py.returncode == 0, py.stderr[-2000:]
    exe = REPO / "timetabling-ga-mpi-openmp_amd" / "ttga-ga"
    cc = subprocess.run([str(exe), *args], capture_output=True, text=True, timeout=300, cwd=str(tmp_path))
    assert cc.returncode == 0, cc.stderr[-2000:]
    a, b = _lines(py.stdout), _lines(cc.stdout)
    assert sorted(a[0]) == list(range(8)) and a == b
    runs = [x["runEntry"] for x in a[1]]
    assert runs[-1]["procsNum"] == 8 and runs[-1]["threadsNum"] == 2
    sols = [v[-1]["solution"] for v in a[0].values()]
    assert runs[0]["totalBest"] == min(s["totalBest"] for s in sols)
    from test_gpu_ga import assert_validated
    assert_validated(inst, tim, py.stdout)
    assert_validated(inst, tim, cc.stdout)
    threads = {e["logEntry"]["threadID"] for v in a[0].values() for e in v if "logEntry" in e}
    assert threads <= {0, 1}


def test_rccl_one_rank_drivers_lg(tmp_path):
    """The RCCL calls of both drivers on one GPU: `ttga-ga --rccl` (a one-rank
    communicator from ncclCommInitAll: the population ncclBroadcast, the
    migration's grouped ncclSend/ncclRecv pairs -- the ring neighbours are the
    rank itself -- and the ncclAllReduce MIN) and `python -m ttga.islands
    --force-dist` (an nccl process group at world 1: dist.broadcast,
    batch_isend_irecv and all_reduce MIN) print the same JSON lines as the
    device-copy paths on the lg instance through one migration (before
    generation 49, ga.cpp:514-540); the printed timetables validate."""
    inst = ttga.config_instance("lg")
    tim = tmp_path / "lg.tim"
    ttga.write_tim(inst, tim)
    args = ["-i", str(tim), "-s", "11", "-p", "1", "-c", "4", "--pop", "16", "--generations", "54"]
    exe = str(REPO / "timetabling-ga-mpi-openmp_amd" / "ttga-ga")
    runs = {}
    for name, cmd in (("cc", [exe, *args]), ("cc_rccl", [exe, *args, "--rccl"]),
                      ("py", [sys.executable, "-m", "ttga.islands", *args]),
                      ("py_dist", [sys.executable, "-m", "ttga.islands", *args, "--force-dist"])):
        p = subprocess.run(cmd, capture_output=True, text=True, timeout=300, env=_env(), cwd=str(tmp_path))
        assert p.returncode == 0, (name, p.stderr[-2000:])
        runs[name] = p.stdout
    lines = {k: _lines(v) for k, v in runs.items()}
    assert sorted(lines["cc"][0]) == [0] and len(lines["cc"][0][0]) >= 2
    for k in ("cc_rccl", "py", "py_dist"):
        assert lines[k] == lines["cc"], k
    from test_gpu_ga import assert_validated
    for v in runs.values():
        assert_validated(inst, tim, v)


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def test_islands_two_ranks_gloo_one_gpu(tmp_path):
    """Two torch.distributed ranks (gloo, both on the one GPU) with two islands
    each: the cross-rank ring (batched send/recv, host-staged), the population
    broadcast, the shared seed and the MIN all-reduce give the same JSON lines
    as one process with the four islands."""
    inst = ttga.config_instance("sm")
    tim = tmp_path / "sm.tim"
    ttga.write_tim(inst, tim)
    common = ["-i", str(tim), "-s", "7", "-p", "1", "-c", "3", "--generations", "60"]
    one = subprocess.run([sys.executable, "-m", "ttga.islands", *common, "--islands", "4"], capture_output=True,
                         text=True, timeout=300, env=_env(), cwd=str(tmp_path))
    assert one.returncode == 0, one.stderr[-2000:]
    two = subprocess.run([sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
                          "--master-addr", "127.0.0.1", "--master-port", str(_free_port()), "-m", "ttga.islands",
                          *common, "--islands", "2", "--backend", "gloo"],
                         capture_output=True, text=True, timeout=300, env=_env(), cwd=str(tmp_path))
    assert two.returncode == 0, two.stderr[-3000:]
    a, b = _lines(one.stdout), _lines(two.stdout)
    assert sorted(a[0]) == [0, 1, 2, 3] and a == b
    from test_gpu_ga import assert_validated
    assert_validated(inst, tim, two.stdout)
