"""GA engine on the GPU vs the CPU restatement: breeding (selection5,
crossover/copy, mutation), replace-worst + sort, whole island generations, and
the ga.cpp-style driver end to end. Bit-exact."""
import json
import pathlib
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

REPO = pathlib.Path(__file__).resolve().parent.parent
KEYS = ("slot", "room", "hcv", "scv", "feasible", "penalty")


def dev(a):
    return torch.from_numpy(np.ascontiguousarray(a)).cuda()


def host(t):
    torch.cuda.synchronize()
    return t.cpu().numpy()


def oracle_population(o, N, seed, steps):
    s, r, g = o.random_init(stream_seeds(seed, 0, N))
    s, r, g = o.local_search(s, r, g, steps)
    h, sc, f, p = o.eval(s, r)
    pop = dict(slot=s, room=r, hcv=h, scv=sc, feasible=f, penalty=p)
    empty = {k: v[:0] for k, v in pop.items()}
    return o.ga_replace(pop, empty)


@pytest.fixture(scope="module")
def sm():
    inst = ttga.config_instance("sm")
    return inst, native.DeviceProblem(inst), oracle().problem(inst)


@pytest.mark.parametrize("N,C,skip", [(10, 1, 1), (10, 10, 1), (64, 37, 0), (200, 130, 1), (4096, 2048, 1)])
def test_breed_vs_oracle(sm, N, C, skip):
    inst, dp, o = sm
    pop = oracle_population(o, N, 3 + N, 50)
    seeds = stream_seeds(11 + C, N, C)
    cs, cr, fl, rng = o.ga_breed(pop["slot"], pop["room"], pop["penalty"], seeds, C, 0.8, 0.5, skip)
    gs, gr = dev(np.zeros((C, inst.E), np.uint8)), dev(np.zeros((C, inst.E), np.uint8))
    gf, grng = dev(np.zeros(C, np.uint8)), dev(seeds)
    dp.ga_breed(dev(pop["slot"]), dev(pop["room"]), dev(pop["penalty"]), grng, gs, gr, gf, 0.8, 0.5, bool(skip))
    assert np.array_equal(host(gf), fl)
    assert np.array_equal(host(gs), cs) and np.array_equal(host(gr), cr)
    assert np.array_equal(host(grng), rng)
    assert (fl & 1).any() and (fl & 2).any() if C >= 10 else True


# N up to 65,536: the tiled sort (8,192-key LDS tiles + global steps above them) for
# C > 8,192; for C <= 8,192 the merge of the survivors with the sorted children
# when the survivors are in order (presorted: as a previous tt_ga_replace leaves
# them; "migrant": one survivor out of order, as after a migration), else the
# one-workgroup fallback sort
@pytest.mark.parametrize("N,C,order", [(10, 1, "random"), (10, 4, "random"), (300, 300, "random"),
                                       (5000, 100, "random"), (20000, 3000, "random"), (65536, 8192, "random"),
                                       (20000, 9000, "random"), (10, 4, "presorted"), (300, 300, "presorted"),
                                       (5000, 100, "presorted"), (65536, 8192, "presorted"),
                                       (65536, 8192, "migrant"), (4096, 1, "migrant")])
def test_replace_vs_oracle(sm, N, C, order):
    inst, dp, o = sm
    rng = np.random.default_rng(N + C)
    def rand_pop(n):
        pen = rng.integers(0, 40, n).astype(np.int32)       # many ties: checks the stable order
        pen[rng.integers(0, n, max(1, n // 50))] = -1        # invalid genomes sort last
        return dict(slot=rng.integers(0, 45, (n, inst.E), dtype=np.uint8),
                    room=rng.integers(0, inst.R, (n, inst.E), dtype=np.uint8),
                    hcv=rng.integers(0, 9, n).astype(np.int32), scv=rng.integers(0, 99, n).astype(np.int32),
                    feasible=rng.integers(0, 2, n).astype(np.uint8), penalty=pen)
    pop, ch = rand_pop(N), rand_pop(C)
    if order != "random":
        pop["penalty"] = np.sort(pop["penalty"].astype(np.uint32)).astype(np.int32)   # key order: -1 last
        if order == "migrant":
            pop["penalty"][(N - C) // 2] = 39 + 1              # one survivor out of order
    exp = o.ga_replace(pop, ch)
    gpop = {k: dev(v) for k, v in pop.items()}
    dp.ga_replace(gpop, {k: dev(v) for k, v in ch.items()}, dp.ga_work(N))
    for k in KEYS:
        assert np.array_equal(host(gpop[k]), exp[k]), k


@pytest.mark.parametrize("N,C,gens,lpt", [(10, 1, 12, None), (16, 8, 6, None), (64, 48, 4, True)])
def test_island_generations_vs_oracle(sm, N, C, gens, lpt):
    inst, dp, o = sm
    steps, seed = 120, 29
    isl = Island(dp, pop_size=N, children=C, max_steps=steps, seed=seed, lpt=lpt)
    isl.initialize()
    for _ in range(gens):
        isl.step()
    pop = oracle_population(o, N, seed, steps)
    rng = stream_seeds(seed, N, C)
    for _ in range(gens):
        cs, cr, fl, rng = o.ga_breed(pop["slot"], pop["room"], pop["penalty"], rng, C, 0.8, 0.5, 1)
        cs, cr, rng = o.local_search(cs, cr, rng, steps)
        h, sc, f, p = o.eval(cs, cr)
        pop = o.ga_replace(pop, dict(slot=cs, room=cr, hcv=h, scv=sc, feasible=f, penalty=p))
    for k in KEYS:
        assert np.array_equal(host(isl.pop[k]), pop[k]), k
    assert np.array_equal(host(isl.rng_child), rng)
    assert np.all(np.diff(pop["penalty"]) >= 0)


def oracle_staggered(o, pop, rng_child, C, gens, steps, flush_after=(), parts=2):
    """The staggered schedule of Island(schedule="staggered", parts=K) on the
    oracle's GA primitives: the child streams split into K sub-batches as
    numpy.array_split does; sub-batch h is bred from the population after the
    replacement of sub-batch h - K, and sub-batch h - K + 1 is replaced right
    after that breed; the pending sub-batches are replaced at the end, and after
    every generation listed in flush_after (a host read of the island)."""
    sizes = [len(x) for x in np.array_split(np.arange(C), parts)]
    offs = np.cumsum([0] + sizes)
    rng = [rng_child[offs[j]:offs[j + 1]].copy() for j in range(parts)]
    pending = []
    for g in range(gens):
        for j in range(parts):
            cs, cr, fl, rng[j] = o.ga_breed(pop["slot"], pop["room"], pop["penalty"], rng[j], sizes[j], 0.8, 0.5, 1)
            if len(pending) >= parts - 1:
                pop = o.ga_replace(pop, pending.pop(0))
            cs, cr, rng[j] = o.local_search(cs, cr, rng[j], steps)
            h, sc, f, p = o.eval(cs, cr)
            pending.append(dict(slot=cs, room=cr, hcv=h, scv=sc, feasible=f, penalty=p))
        if g in flush_after:
            while pending:
                pop = o.ga_replace(pop, pending.pop(0))
    while pending:
        pop = o.ga_replace(pop, pending.pop(0))
    return pop, np.concatenate(rng)


@pytest.mark.parametrize("N,C,gens,lpt,reads,parts", [(10, 2, 12, False, (), 2), (16, 7, 6, False, (2,), 2),
                                                      (64, 48, 5, True, (1, 3), 2), (30, 11, 6, False, (3,), 3),
                                                      (64, 40, 4, True, (), 4)],
                         ids=["N10C2", "N16C7_read", "N64C48_lpt_reads", "N30C11_3parts", "N64C40_4parts_lpt"])
def test_island_staggered_vs_oracle(sm, N, C, gens, lpt, reads, parts):
    """Island(schedule="staggered"): K sub-batches on K streams, each bred from
    the population K - 1 sub-batches behind; bit-exact against the same
    dependency order on the oracle's GA primitives, with host reads of the
    island (which replace the pending sub-batches) after the generations in
    `reads`, odd C, uneven parts, and LPT dispatch."""
    inst, dp, o = sm
    steps, seed = 120, 41
    isl = Island(dp, pop_size=N, children=C, max_steps=steps, seed=seed, lpt=lpt, schedule="staggered", parts=parts)
    isl.initialize()
    for g in range(gens):
        isl.step()
        if g in reads:
            isl.member_meta(0)
    pop = oracle_population(o, N, seed, steps)
    pop, rng = oracle_staggered(o, pop, stream_seeds(seed, N, C), C, gens, steps, reads, parts)
    isl.sync()
    for k in KEYS:
        assert np.array_equal(host(isl.pop[k]), pop[k]), k
    assert np.array_equal(host(isl.rng_child), rng)
    assert np.all(np.diff(pop["penalty"].astype(np.uint32)) >= 0)


def test_island_staggered_orders_the_callers_stream():
    """Island(stream=None, schedule="staggered") runs its parts on streams of
    their own; the caller's work on torch's current stream must still see the
    population as the last step left it (what tools/ga_quality.py's per-
    generation log does): clones taken on the current stream right after each
    step, with no host sync, equal those of a twin island read after a full
    device sync; pop[0]'s penalty never rises."""
    inst = ttga.config_instance("comp01")
    dp = native.DeviceProblem(inst)
    N, C, gens, steps, seed = 256, 128, 6, 1000, 11
    logs = []
    for synced in (False, True):
        isl = Island(dp, pop_size=N, children=C, max_steps=steps, seed=seed, lpt=True, schedule="staggered")
        isl.initialize()
        got = []
        for _ in range(gens):
            isl.step()
            if synced:
                torch.cuda.synchronize()
            got.append(torch.stack([isl.pop["penalty"].clone(), isl.pop["scv"].clone()]))
        isl.flush()
        got.append(torch.stack([isl.pop["penalty"].clone(), isl.pop["scv"].clone()]))
        torch.cuda.synchronize()
        logs.append([host(t) for t in got])
        isl.close()
    for g, (a, b) in enumerate(zip(*logs)):
        assert np.array_equal(a, b), g
    best = np.array([t[0, 0] for t in logs[0]]).astype(np.uint32).astype(np.int64)    # -1 sentinel: last
    assert np.all(np.diff(best) <= 0), best


def test_island_staggered_comp01_vs_oracle():
    """The staggered schedule on a comp01-size instance (the GA bench's
    configs[2] shape): 512 members, 256 children per generation (LPT on), four
    generations against the oracle, bit-exact; and the snapshots taken after
    each generation (the islands driver's log source) equal the population as
    the oracle has it after that generation's half-batch A."""
    inst = ttga.config_instance("comp01")
    dp = native.DeviceProblem(inst)
    o = oracle().problem(inst)
    N, C, gens, steps, seed = 512, 256, 4, 300, 7
    isl = Island(dp, pop_size=N, children=C, max_steps=steps, seed=seed, lpt=True, schedule="staggered")
    isl.initialize()
    snaps = []
    for _ in range(gens):
        isl.step()
        snaps.append(isl.snapshot())
    from oracle_lib import split_rows
    s, r, g = o.random_init(stream_seeds(seed, 0, N))
    s, r, g = split_rows(o.local_search, (s, r, g), steps)
    h, sc, f, p = o.eval(s, r)
    pop = o.ga_replace(dict(slot=s, room=r, hcv=h, scv=sc, feasible=f, penalty=p),
                       {k: v[:0] for k, v in dict(slot=s, room=r, hcv=h, scv=sc, feasible=f, penalty=p).items()})
    hA = C // 2
    rng = [stream_seeds(seed, N, C)[:hA].copy(), stream_seeds(seed, N, C)[hA:].copy()]
    pending, firsts = None, []
    for gg in range(gens):
        for k in (0, 1):
            cs, cr, fl, rng[k] = o.ga_breed(pop["slot"], pop["room"], pop["penalty"], rng[k], hA, 0.8, 0.5, 1)
            if pending is not None:
                pop = o.ga_replace(pop, pending)
            cs, cr, rng[k] = split_rows(o.local_search, (cs, cr, rng[k]), steps)
            hh, sc, f, p = o.eval(cs, cr)
            pending = dict(slot=cs, room=cr, hcv=hh, scv=sc, feasible=f, penalty=p)
        firsts.append((bool(pop["feasible"][0]), int(pop["scv"][0]), int(pop["hcv"][0])))
    pop = o.ga_replace(pop, pending)
    assert [sn.values()[:3] for sn in snaps] == firsts
    isl.sync()
    for k in KEYS:
        assert np.array_equal(host(isl.pop[k]), pop[k]), k
    assert np.array_equal(host(isl.rng_child), np.concatenate(rng))
    assert dp.status() == 0


def test_islands_cli_end_to_end(tmp_path, sm):
    """python -m ttga.islands on one GPU: Control-style CLI, JSON lines in the
    reference's format, one self-migration (generation 49), and the printed
    timetable re-evaluates to the printed totalBest."""
    inst, dp, o = sm
    tim = tmp_path / "sm.tim"
    ttga.write_tim(inst, tim)
    cmd = [sys.executable, "-m", "ttga.islands", "-i", str(tim), "-s", "42", "-p", "1", "-c", "2",
           "--generations", "60"]
    env = dict(__import__("os").environ, PYTHONPATH=str(REPO / "timetabling-ga-mpi-openmp_amd"))
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=240, env=env, cwd=str(tmp_path))
    assert r.returncode == 0, r.stderr[-2000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    objs = [json.loads(ln) for ln in lines]
    assert "Max number of threads 2" in r.stdout
    assert any("logEntry" in x for x in objs)
    runs = [x["runEntry"] for x in objs if "runEntry" in x]
    assert runs[0].keys() == {"feasible", "totalBest"} and runs[-1]["procsNum"] == 1 and runs[-1]["threadsNum"] == 2
    sol = [x["solution"] for x in objs if "solution" in x][0]
    assert sol["procID"] == 0 and sol["threadID"] == 0 and sol["totalBest"] == runs[0]["totalBest"]
    assert_validated(inst, tim, r.stdout)


def assert_validated(inst, tim, stdout):
    """Every printed solution line re-derives from the instance (ttga.validate
    and the native ttga-check, Solution.cpp:63-160)."""
    from ttga.validate import check_text
    reps = check_text(inst, stdout)
    assert reps and all(r["ok"] for r in reps), reps
    chk = REPO / "timetabling-ga-mpi-openmp_amd" / "ttga-check"
    out = subprocess.run([str(chk), str(tim), "-"], input=stdout, capture_output=True, text=True, timeout=60)
    assert out.returncode == 0, out.stdout


def _json_lines(text):
    """JSON lines with the wall-clock fields removed."""
    out = []
    for ln in text.splitlines():
        if ln.startswith("{"):
            obj = json.loads(ln)
            for v in obj.values():
                v.pop("time", None)
                v.pop("totalTime", None)
            out.append(obj)
    return out


def test_native_driver_matches_python_driver(tmp_path, sm):
    """The C++ driver (ttga-ga, C-ABI + RCCL) and the Python driver
    (ttga.islands) run the same GA on one GPU: identical JSON lines apart from
    wall-clock times (log entries, run entries, the printed timetable)."""
    inst, dp, o = sm
    exe = REPO / "timetabling-ga-mpi-openmp_amd" / "ttga-ga"
    assert exe.exists(), "ttga-ga not built (make -C timetabling-ga-mpi-openmp_amd)"
    tim = tmp_path / "sm.tim"
    ttga.write_tim(inst, tim)
    args = ["-i", str(tim), "-s", "42", "-p", "1", "-c", "3", "--generations", "120", "--pop", "12"]
    env = dict(__import__("os").environ, PYTHONPATH=str(REPO / "timetabling-ga-mpi-openmp_amd"))
    py = subprocess.run([sys.executable, "-m", "ttga.islands", *args], capture_output=True, text=True, timeout=240,
                        env=env, cwd=str(tmp_path))
    cc = subprocess.run([str(exe), *args], capture_output=True, text=True, timeout=240, cwd=str(tmp_path))
    assert py.returncode == 0, py.stderr[-2000:]
    assert cc.returncode == 0, cc.stderr[-2000:]
    a, b = _json_lines(py.stdout), _json_lines(cc.stdout)
    assert len(a) > 3 and a == b
    assert "Max number of threads 3" in cc.stdout
    assert "Warning: No output file given, writing to stdout" in cc.stderr
    assert_validated(inst, tim, cc.stdout)


@pytest.mark.parametrize("args", [["-c", "3", "--generations", "120", "--pop", "12", "--stagger"],
                                  ["-c", "4096", "--generations", "5", "--pop", "4096", "--stagger"],
                                  ["-c", "7", "--generations", "60", "--pop", "16", "--stagger-parts", "3"]],
                         ids=["c3_migration", "c4096_lpt", "c7_3parts"])
def test_native_driver_matches_python_driver_staggered(tmp_path, sm, args):
    """Both drivers with --stagger (two sub-batches per generation on two
    streams, each bred one sub-batch behind) and --stagger-parts 3: identical
    JSON lines apart from wall-clock times, through a migration (generation
    49: the pending sub-batches are replaced first) and with LPT dispatch per
    sub-batch; the staggered run differs from the batch one (a different GA
    schedule)."""
    inst, dp, o = sm
    exe = REPO / "timetabling-ga-mpi-openmp_amd" / "ttga-ga"
    tim = tmp_path / "sm.tim"
    ttga.write_tim(inst, tim)
    base = ["-i", str(tim), "-s", "42", "-p", "1", *args]
    env = dict(__import__("os").environ, PYTHONPATH=str(REPO / "timetabling-ga-mpi-openmp_amd"))
    py = subprocess.run([sys.executable, "-m", "ttga.islands", *base], capture_output=True, text=True,
                        timeout=240, env=env, cwd=str(tmp_path))
    cc = subprocess.run([str(exe), *base], capture_output=True, text=True, timeout=240, cwd=str(tmp_path))
    plain = [a for a in base if a != "--stagger"]
    if "--stagger-parts" in plain:
        i = plain.index("--stagger-parts")
        del plain[i:i + 2]
    bat = subprocess.run([str(exe), *plain], capture_output=True, text=True, timeout=240, cwd=str(tmp_path))
    assert py.returncode == 0, py.stderr[-2000:]
    assert cc.returncode == 0, cc.stderr[-2000:]
    assert bat.returncode == 0, bat.stderr[-2000:]
    a, b = _json_lines(py.stdout), _json_lines(cc.stdout)
    assert len(a) >= 3 and a == b
    assert a != _json_lines(bat.stdout)
    assert_validated(inst, tim, cc.stdout)


def test_lpt_order_vs_numpy(sm):
    """tt_lpt_order: indices by key descending, ties by index, negative keys last
    (the sizes cover the small LDS sort, the register-blocked one-workgroup sort
    up to 8,192 keys -- in-thread, in-wave and cross-wave steps -- and the tiled one)."""
    inst, dp, o = sm
    rng = np.random.default_rng(8)
    for n in (1, 5, 8, 9, 100, 511, 512, 513, 4096, 5000, 8192, 20000):
        key = rng.integers(-1, 30, n).astype(np.int32)
        hi = np.where(key < 0, np.int64(2 ** 32), np.int64(2 ** 31 - 1) - key.astype(np.int64))
        exp = np.lexsort((np.arange(n), hi)).astype(np.int32)
        got = host(dp.lpt_order(dev(key), dp.ga_work(max(n, 2))))
        assert np.array_equal(got, exp), n


def test_native_driver_matches_python_driver_lpt(tmp_path, sm):
    """Both drivers with 4,096 children per generation (longest-expected-first
    dispatch in both): identical JSON lines apart from wall-clock times."""
    inst, dp, o = sm
    exe = REPO / "timetabling-ga-mpi-openmp_amd" / "ttga-ga"
    tim = tmp_path / "sm.tim"
    ttga.write_tim(inst, tim)
    args = ["-i", str(tim), "-s", "5", "-p", "1", "-c", "4096", "--generations", "6", "--pop", "4096"]
    env = dict(__import__("os").environ, PYTHONPATH=str(REPO / "timetabling-ga-mpi-openmp_amd"))
    py = subprocess.run([sys.executable, "-m", "ttga.islands", *args], capture_output=True, text=True, timeout=240,
                        env=env, cwd=str(tmp_path))
    cc = subprocess.run([str(exe), *args], capture_output=True, text=True, timeout=240, cwd=str(tmp_path))
    assert py.returncode == 0, py.stderr[-2000:]
    assert cc.returncode == 0, cc.stderr[-2000:]
    a, b = _json_lines(py.stdout), _json_lines(cc.stdout)
    assert len(a) >= 3 and a == b


def test_ga_trajectories_match_reference_statistically(sm):
    """Whole-GA outcomes over fixed seeds (the RNG streams differ):
    the device GA (pop 10, one child per generation) against the reference's
    own ga.cpp loop (oracle/_ref ref_ga_run, fresh crossover child) on the sm
    instance, 16 seeds x 1000 generations, maxSteps 200. Same feasibility rate
    (Fisher), no detectable shift of the final best (Mann-Whitney U, p > 0.01)
    and the device's median best within 20 % of the reference's (a guard
    against a quality regression that the rank test alone could miss).
    tools/ga_quality.py is the full 16-seed x 2001-generation version
    (profiles/r01_ga_quality_sm.json)."""
    from oracle_lib import ref
    R = ref()
    if R is None:
        pytest.skip("reference build oracle/_ref not present")
    stats = pytest.importorskip("scipy.stats")
    sys.path.insert(0, str(REPO / "tools"))
    from ga_quality import device_runs
    from oracle_lib import host_threads
    inst = sm[0]
    seeds, gens = list(range(1, 17)), 1000
    _, _, rfeas, _, rtrace, _ = R.problem(inst).ga_run(seeds, 10, gens, 200, 0, host_threads())
    dfinal, dfeas, dtrace, _ = device_runs(inst, seeds, 10, gens, 200)
    # the logged best never gets worse along a trajectory (ga.cpp keeps pop[0])
    assert np.all(np.diff(dtrace, axis=1) <= 0)
    _assert_same_quality(stats, seeds, dfinal, dfeas, rtrace[:, -1], rfeas)


def test_ga_staggered_trajectories_match_reference_statistically(sm):
    """The staggered schedule against the reference's ga.cpp loop (fresh
    crossover child), same number of children: the device GA with two
    sub-batches of one child (pop 10, C = 2, each child bred one child behind,
    as two ga.cpp threads would) for 500 generations against the reference's
    one-thread loop for 1000 generations, 16 seeds, maxSteps 200 on sm. Same
    feasibility (Fisher), no shift of the final best (Mann-Whitney U, p >
    0.01), medians within 20 %."""
    from oracle_lib import ref
    R = ref()
    if R is None:
        pytest.skip("reference build oracle/_ref not present")
    stats = pytest.importorskip("scipy.stats")
    sys.path.insert(0, str(REPO / "tools"))
    from ga_quality import device_runs
    from oracle_lib import host_threads
    inst = sm[0]
    seeds = list(range(1, 17))
    _, _, rfeas, _, rtrace, _ = R.problem(inst).ga_run(seeds, 10, 1000, 200, 0, host_threads())
    dfinal, dfeas, dtrace, _ = device_runs(inst, seeds, 10, 500, 200, children=2, schedule="staggered")
    assert np.all(np.diff(dtrace, axis=1) <= 0)
    _assert_same_quality(stats, seeds, dfinal, dfeas, rtrace[:, -1], rfeas)


def _assert_same_quality(stats, seeds, dfinal, dfeas, rfinal, rfeas):
    """Same feasibility count (Fisher), no shift of the final best (Mann-Whitney
    U, p > 0.01), device median best within 20 % of the reference's."""
    table = [[int(dfeas.sum()), int(len(seeds) - dfeas.sum())], [int(rfeas.sum()), int(len(seeds) - rfeas.sum())]]
    assert stats.fisher_exact(table)[1] > 0.01
    p = stats.mannwhitneyu(dfinal, rfinal, alternative="two-sided").pvalue
    assert p > 0.01, (dfinal, rfinal, p)
    md, mr = float(np.median(dfinal)), float(np.median(rfinal))
    assert abs(md - mr) <= 0.2 * max(mr, 1.0), (md, mr)


@pytest.mark.parametrize("c", range(4))
def test_breed_selection5_vs_reference(sm, c):
    """tt_ga_breed's tournaments against the reference's own selection5
    (tests/golden/ga_ref.json, ga.cpp:129-145 compiled from the reference):
    with crossover always on, child k's slots follow parent a = winner 2k and
    parent b = winner 2k+1 of the golden sequence."""
    from test_json_parity import GOLD, selection_case_expectations
    from ttga.rng import ParkMiller
    inst, dp, o = sm
    case = GOLD["selection5"][c]
    N = case["N"]
    rng = np.random.default_rng(c)
    pop_slot = rng.integers(0, 45, (N, inst.E), dtype=np.uint8)
    pop_room = o.assign_rooms(pop_slot)
    seeds = selection_case_expectations(case)
    C = seeds.size
    gs, gr = dev(np.zeros((C, inst.E), np.uint8)), dev(np.zeros((C, inst.E), np.uint8))
    gf, grng = dev(np.zeros(C, np.uint8)), dev(seeds)
    dp.ga_breed(dev(pop_slot), dev(pop_room), dev(np.array(case["penalty"], np.int32)), grng, gs, gr, gf, 1.0, 0.0,
                False)
    got = host(gs)
    w = np.array(case["winners"])
    for k in range(C):
        pm = ParkMiller(int(seeds[k]))
        for _ in range(11):
            pm.next()
        take_a = np.array([pm.next() < 0.5 for _ in range(inst.E)])
        assert np.array_equal(got[k], np.where(take_a, pop_slot[w[2 * k]], pop_slot[w[2 * k + 1]])), k


def test_best_thread_with_lpt_dispatch(sm):
    """The logEntry threadID (Island.best_thread, from the source slot
    tt_ga_replace writes at tt_ga_work_source_offset) with LPT dispatch on
    (C >= 4096, tt_lpt_order sorts in the same work buffer): after each
    generation it names the child that became pop[0], or 0 when the old pop[0]
    stayed (it wins ties: lower merged position)."""
    inst, dp, o = sm
    N, C = 8192, 4096
    isl = Island(dp, pop_size=N, children=C, max_steps=50, seed=12)
    assert isl.lpt
    isl.initialize()
    changed = 0
    for _ in range(4):
        old0 = int(host(isl.pop["penalty"])[0])
        isl.step()
        cpen = host(isl.child["penalty"]).astype(np.uint32)
        c = int(np.argmin(cpen))
        exp = c if cpen[c] < np.uint32(old0) else 0
        got = isl.best_thread()
        assert got == exp
        if cpen[c] < np.uint32(old0):
            changed += 1
            assert np.array_equal(host(isl.pop["slot"][0]), host(isl.child["slot"][c]))
    assert changed > 0


def test_local_search_order_permutation_check():
    """tt_local_search_ordered flags a dispatch order that is not a
    permutation (status bit 3): a duplicate entry (one individual missing), an
    out-of-range entry, three duplicates replacing {1, 5, 6} by {2, 3, 7}
    (sum and sum of squares unchanged: only an exact check sees it); a true
    permutation leaves the status clean."""
    inst = ttga.config_instance("med")
    P = 64
    seeds = ttga.population_seeds(31, P)
    same_sums = np.arange(P)
    same_sums[[1, 5, 6]] = [2, 3, 7]
    assert same_sums.sum() == np.arange(P).sum() and (same_sums ** 2).sum() == (np.arange(P) ** 2).sum()
    for order, bad in ((np.random.default_rng(0).permutation(P), False),
                       (np.r_[np.arange(P - 1), 0], True),
                       (np.r_[np.arange(P - 1), P], True),
                       (np.random.default_rng(1).permutation(same_sums), True)):
        dp = native.DeviceProblem(inst)
        s = dev(ttga.random_slots(seeds, inst.E)[0])
        r = dp.assign_rooms(s)
        dp.local_search(s, r, dev(seeds), 50, order=dev(order.astype(np.int32)))
        assert bool(dp.status() & 8) == bad, order[-3:]
        dp.close()


def test_ga_trajectories_med_statistical():
    """The north star's statistical GA comparison at a 400-event size (reduced
    form of tools/ga_quality_program.py, whose full runs -- the reference
    program itself, 16 seeds x 2001 generations -- are in
    profiles/r03_ga_quality_{med,comp01}.json): the device GA (pop 10, one
    child per generation, maxSteps 1000 as -p 2) against the reference's own
    ga.cpp loop (oracle/_ref ref_ga_run, fresh crossover child) on the med
    instance, 16 seeds x 500 generations: same feasibility count (Fisher), no
    detectable shift of the final best (Mann-Whitney U, p > 0.01), medians
    within 20 %."""
    from oracle_lib import host_threads, ref
    R = ref()
    if R is None:
        pytest.skip("reference build oracle/_ref not present")
    stats = pytest.importorskip("scipy.stats")
    sys.path.insert(0, str(REPO / "tools"))
    from ga_quality import device_runs
    inst = ttga.config_instance("med")
    seeds, gens, steps = list(range(1, 17)), 500, 1000
    _, _, rfeas, _, rtrace, _ = R.problem(inst).ga_run(seeds, 10, gens, steps, 0, host_threads())
    dfinal, dfeas, dtrace, _ = device_runs(inst, seeds, 10, gens, steps)
    assert np.all(np.diff(dtrace, axis=1) <= 0)
    _assert_same_quality(stats, seeds, dfinal, dfeas, rtrace[:, -1], rfeas)