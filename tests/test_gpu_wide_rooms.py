"""GPU parity beyond the BASELINE instances' shapes: R > 16 rooms and E > 448
events through the local search, mutation, crossover, breed and replace,
against the CPU oracle. Bit-exact (slots, rooms, RNG states).

The local search has code that depends on R: the phase-1 room-pair bounds
(TT_LS_P1B) and the register matcher (TT_MATCH_REG) exist only for R <= 16, so
R = 17..64 runs the plain wave matcher with u32/u64 room masks and no pair
bounds. E > 448 widens every per-event structure past 7 64-bit words (EW64 > 7)
and the matcher tasks past one wave of events. Reference: Solution.cpp:357-469
(moves, mutation), 471-769 (localSearch), 772-891 (assignRooms), 893-910
(crossover); ga.cpp:129-153, 543-585 (selection5, replace-worst + sort).
"""
import numpy as np
import pytest

import ttga
from oracle_lib import oracle, split_rows

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")
from ttga import native  # noqa: E402
from ttga.ga import Island, stream_seeds  # noqa: E402

KEYS = ("slot", "room", "hcv", "scv", "feasible", "penalty")


def dev(a):
    return torch.from_numpy(np.ascontiguousarray(a)).cuda()


def host(t):
    torch.cuda.synchronize()
    return t.cpu().numpy()


@pytest.fixture(scope="module")
def orc():
    return oracle()


def _inst(E, R, F, S, seed, att=(4, 16)):
    """4..16 events per student by default: localSearch(300) from random init
    leaves every individual infeasible (phase 1) and (3000) makes them feasible
    (phase 2) at every R and E here; att=None: the generator's 5..20."""
    return ttga.generate(E, R, F, S, seed=seed, **(dict(min_att=att[0], max_att=att[1]) if att else {}))


def _ls_both(dp, o, s0, r0, seeds, steps):
    """tt_local_search and the oracle (host threads over row blocks) on the same
    inputs; asserts slots, rooms and RNG states equal; returns the oracle's."""
    s, r, g = dev(s0), dev(r0), dev(seeds)
    dp.local_search(s, r, g, steps)
    es, er, eg = split_rows(o.local_search, (s0, r0, seeds), steps)
    gs, gr, gg = host(s), host(r), host(g)
    bad = np.flatnonzero((gs != es).any(1) | (gr != er).any(1) | (gg != eg))
    assert bad.size == 0, f"{bad.size} individuals differ at maxSteps {steps}, first {bad[:8]}"
    return es, er, eg


# (E, R, F, S): R just past the pair bounds / register matcher (17), u32 room masks
# (24), u64 masks (40, 64); E past eval_tile5's 448 (EW64 = 8) and at ~1000 (EW64 = 16)
LS_SHAPES = [(400, 17, 4, 200), (400, 24, 5, 200), (449, 40, 5, 220), (449, 64, 6, 220),
             (1000, 24, 6, 300), (1000, 64, 6, 300)]


@pytest.mark.parametrize("dims", LS_SHAPES, ids=[f"E{d[0]}R{d[1]}" for d in LS_SHAPES])
def test_local_search_wide_rooms_phase1_then_phase2(orc, dims):
    """From RandomInitialSolution: localSearch(300) (phase 1), chained (3000)
    (most individuals reach feasibility), then (2000) started in phase 2 --
    slots, rooms and RNG states identical to the oracle after every call, and
    eval identical at the end."""
    inst = _inst(*dims, seed=dims[0] + dims[1])
    dp = native.DeviceProblem(inst)
    o = orc.problem(inst)
    P = 48
    s0, r0, _ = o.random_init(ttga.population_seeds(5000 + dims[1], P))
    seeds = ttga.population_seeds(6000 + dims[1], P)
    es, er, eg = _ls_both(dp, o, s0, r0, seeds, 300)
    feas0 = int(o.eval(es, er)[2].sum())
    es, er, eg = _ls_both(dp, o, es, er, eg, 3000)
    feas = int(o.eval(es, er)[2].sum())
    assert feas0 < P // 4 and feas >= P // 2          # phase 1 first, the last call mostly in phase 2
    es, er, eg = _ls_both(dp, o, es, er, eg, 2000)
    got = [host(t) for t in dp.eval(dev(es), dev(er))]
    for x, e in zip(got, o.eval(es, er)):
        assert np.array_equal(x, e)
    assert dp.status() == 0


@pytest.mark.parametrize("dims", [(449, 24, 5, 220), (1000, 64, 6, 400)], ids=["E449R24", "E1000R64"])
def test_local_search_wide_rooms_dense_students(orc, dims):
    """The generator's default attendances (5..20 events per student): dense
    correlations keep the whole call in phase 1 with many room clashes; random
    rooms (not assignRooms's) as the start on every other individual."""
    inst = _inst(*dims, seed=77, att=None)
    dp = native.DeviceProblem(inst)
    o = orc.problem(inst)
    P = 32
    s0, r0, _ = o.random_init(ttga.population_seeds(7100, P))
    r0[::2] = np.random.default_rng(3).integers(0, inst.R, size=(P // 2, inst.E), dtype=np.uint8)
    _ls_both(dp, o, s0, r0, ttga.population_seeds(7200, P), 400)
    assert dp.status() == 0


@pytest.mark.parametrize("dims", [(400, 40, 5, 200), (1000, 64, 6, 300), (449, 17, 5, 220)],
                         ids=["E400R40", "E1000R64", "E449R17"])
def test_local_search_wide_rooms_crowded_slots_redo(orc, dims):
    """Crowded slots (65-200 events in one slot) at R > 16: the first launch's
    64-event matcher tasks send those individuals to the redo launch, whose
    tasks hold up to 256 events (the lane-serial matcher past 64 events); every
    individual against the oracle, the device status clean."""
    inst = _inst(*dims, seed=91, att=(2, 8))
    dp = native.DeviceProblem(inst)
    o = orc.problem(inst)
    P = 24
    s0, _, _ = o.random_init(ttga.population_seeds(8100, P))
    rng = np.random.default_rng(4)
    for k in range(1, P, 2):
        n = int(rng.integers(65, 200 if inst.E >= 1000 else 150))
        s0[k, rng.choice(inst.E, size=n, replace=False)] = int(rng.integers(0, 45))
    r0 = o.assign_rooms(s0)
    assert np.array_equal(host(dp.assign_rooms(dev(s0))), r0)
    es, er, eg = _ls_both(dp, o, s0, r0, ttga.population_seeds(8200, P), 300)
    _ls_both(dp, o, es, er, eg, 1500)
    assert dp.status() == 0


@pytest.mark.parametrize("dims", [(1000, 40, 6, 300), (1000, 17, 5, 300), (1000, 16, 5, 300), (600, 10, 4, 200)],
                         ids=["E1000R40", "E1000R17", "E1000R16", "E600R10"])
def test_assign_rooms_slot_shapes_vs_oracle(orc, dims):
    """tt_assign_rooms and tt_mutation on rows built to hit every matcher path:
    the wave matcher (slots of 1-64 events), the lane-serial fallback (65-256
    events; at R > 16 two such slots of one individual, an even and an odd one,
    so both waves of the wide kernel take it at once), the register lanes of a
    whole row at R <= 16 (<= 32 events) beside the wave (33-64), empty slots.
    Rooms and mutated rows against the oracle, device status clean."""
    inst = _inst(*dims, seed=123, att=(2, 8))
    dp = native.DeviceProblem(inst)
    o = orc.problem(inst)
    E, P = inst.E, 48
    rng = np.random.default_rng(17)
    s0 = rng.integers(0, 45, size=(P, E), dtype=np.uint8)
    for k in range(P):
        kind = k % 4
        ev = rng.permutation(E)
        if kind == 0:                                   # two crowded slots, even and odd
            a, b = 2 * int(rng.integers(0, 22)), 2 * int(rng.integers(0, 22)) + 1
            s0[k, ev[:int(rng.integers(65, 257))]] = a
            s0[k, ev[300:300 + int(rng.integers(65, 257))]] = b
        elif kind == 1:                                 # slots of exactly 32, 33, 64 events; slot 44 empty
            s0[k][s0[k] == 44] = 0
            for t, n in ((3, 32), (4, 33), (5, 64)):
                s0[k][s0[k] == t] = 6
                s0[k, ev[100 * t:100 * t + n]] = t
        elif kind == 2:                                 # few slots of ~40-70 events
            s0[k] = rng.integers(0, max(1, E // 50), size=E).astype(np.uint8)
    r0 = o.assign_rooms(s0)
    assert np.array_equal(host(dp.assign_rooms(dev(s0))), r0)
    ms = ttga.population_seeds(9400, P)
    mslot, mroom, mrng = o.mutation(s0, r0, ms)
    gs, gr, gg = dev(s0), dev(r0), dev(ms)
    dp.mutation(gs, gr, gg)
    assert np.array_equal(host(gs), mslot) and np.array_equal(host(gr), mroom) and np.array_equal(host(gg), mrng)
    assert dp.status() == 0


@pytest.mark.parametrize("dims", [(449, 24, 5, 220), (1000, 64, 6, 300)], ids=["E449R24", "E1000R64"])
def test_variation_wide_rooms_vs_oracle(orc, dims):
    """RandomInitialSolution, crossover and mutation (Solution.cpp:48-61,
    441-469, 893-910) at R > 16 and E > 448: children, rooms and RNG states."""
    inst = _inst(*dims, seed=55)
    dp = native.DeviceProblem(inst)
    o = orc.problem(inst)
    P = 64
    seeds = ttga.population_seeds(9100, P)
    es, er, eg = o.random_init(seeds)
    s, r, g = (torch.empty((P, inst.E), dtype=torch.uint8, device="cuda"),
               torch.empty((P, inst.E), dtype=torch.uint8, device="cuda"), dev(seeds))
    dp.random_init(g, s, r)
    assert np.array_equal(host(s), es) and np.array_equal(host(r), er) and np.array_equal(host(g), eg)
    h = P // 2
    xs = ttga.population_seeds(9200, h)
    cs, cr, crng = o.crossover(es[:h], es[h:], xs)
    gs, gr, gg = dev(np.zeros((h, inst.E), np.uint8)), dev(np.zeros((h, inst.E), np.uint8)), dev(xs)
    dp.crossover(dev(es[:h]), dev(es[h:]), gg, gs, gr)
    assert np.array_equal(host(gs), cs) and np.array_equal(host(gr), cr) and np.array_equal(host(gg), crng)
    ms = ttga.population_seeds(9300, P)
    mslot, mroom, mrng = o.mutation(es, er, ms)
    gs, gr, gg = dev(es), dev(er), dev(ms)
    dp.mutation(gs, gr, gg)
    assert np.array_equal(host(gs), mslot) and np.array_equal(host(gr), mroom) and np.array_equal(host(gg), mrng)
    assert not np.array_equal(mslot, es)
    assert dp.status() == 0


def _oracle_population(o, N, seed, steps):
    s, r, g = o.random_init(stream_seeds(seed, 0, N))
    s, r, g = split_rows(o.local_search, (s, r, g), steps)
    h, sc, f, p = o.eval(s, r)
    pop = dict(slot=s, room=r, hcv=h, scv=sc, feasible=f, penalty=p)
    return o.ga_replace(pop, {k: v[:0] for k, v in pop.items()})


@pytest.mark.parametrize("dims", [(449, 24, 5, 220), (1000, 64, 6, 300)], ids=["E449R24", "E1000R64"])
def test_breed_replace_wide_rooms_vs_oracle(orc, dims):
    """tt_ga_breed (selection5 x 2, crossover or copy, mutation; wave per
    child) and tt_ga_replace (replace-worst + sort) at R > 16 and E > 448
    against the oracle's GA primitives."""
    inst = _inst(*dims, seed=57)
    dp = native.DeviceProblem(inst)
    o = orc.problem(inst)
    N, C = 96, 64
    pop = _oracle_population(o, N, 21, 150)
    seeds = stream_seeds(22, N, C)
    cs, cr, fl, crng = o.ga_breed(pop["slot"], pop["room"], pop["penalty"], seeds, C, 0.8, 0.5, 1)
    gs, gr = dev(np.zeros((C, inst.E), np.uint8)), dev(np.zeros((C, inst.E), np.uint8))
    gf, grng = dev(np.zeros(C, np.uint8)), dev(seeds)
    dp.ga_breed(dev(pop["slot"]), dev(pop["room"]), dev(pop["penalty"]), grng, gs, gr, gf, 0.8, 0.5, True)
    assert np.array_equal(host(gf), fl)
    assert np.array_equal(host(gs), cs) and np.array_equal(host(gr), cr) and np.array_equal(host(grng), crng)
    assert (fl & 1).any() and (fl & 2).any()
    h, sc, f, p = o.eval(cs, cr)
    child = dict(slot=cs, room=cr, hcv=h, scv=sc, feasible=f, penalty=p)
    exp = o.ga_replace(pop, child)
    gpop = {k: dev(v) for k, v in pop.items()}
    dp.ga_replace(gpop, {k: dev(v) for k, v in child.items()}, dp.ga_work(N))
    for k in KEYS:
        assert np.array_equal(host(gpop[k]), exp[k]), k


@pytest.mark.parametrize("dims,lpt", [((449, 40, 5, 220), False), ((1000, 64, 6, 300), True)],
                         ids=["E449R40", "E1000R64_lpt"])
def test_island_generations_wide_rooms_vs_oracle(orc, dims, lpt):
    """Whole island generations (breed -> localSearch -> eval -> replace, the
    ga.cpp:543-585 loop for C children at once) at R > 16 and E > 448, with and
    without longest-expected-first dispatch, against the oracle's GA."""
    inst = _inst(*dims, seed=59)
    dp = native.DeviceProblem(inst)
    o = orc.problem(inst)
    N, C, gens, steps, seed = 64, 48, 3, 300, 31
    isl = Island(dp, pop_size=N, children=C, max_steps=steps, seed=seed, lpt=lpt)
    isl.initialize()
    for _ in range(gens):
        isl.step()
    pop = _oracle_population(o, N, seed, steps)
    rng = stream_seeds(seed, N, C)
    for _ in range(gens):
        cs, cr, fl, rng = o.ga_breed(pop["slot"], pop["room"], pop["penalty"], rng, C, 0.8, 0.5, 1)
        cs, cr, rng = split_rows(o.local_search, (cs, cr, rng), steps)
        h, sc, f, p = o.eval(cs, cr)
        pop = o.ga_replace(pop, dict(slot=cs, room=cr, hcv=h, scv=sc, feasible=f, penalty=p))
    for k in KEYS:
        assert np.array_equal(host(isl.pop[k]), pop[k]), k
    assert np.array_equal(host(isl.rng_child), rng)
    assert dp.status() == 0


def test_local_search_syn_sample_vs_oracle(orc):
    """BASELINE configs[4]'s instance (2000 events, 40 rooms, 5000 students)
    through the local search: 32 individuals from RandomInitialSolution,
    localSearch(200), bit-exact against the oracle (slots, rooms, RNG
    states), then eval."""
    inst = ttga.config_instance("syn")
    dp = native.DeviceProblem(inst)
    o = orc.problem(inst)
    P = 32
    s0, r0, _ = o.random_init(ttga.population_seeds(9900, P))
    es, er, eg = _ls_both(dp, o, s0, r0, ttga.population_seeds(9901, P), 200)
    got = [host(t) for t in dp.eval(dev(es), dev(er))]
    for x, e in zip(got, o.eval(es, er)):
        assert np.array_equal(x, e)
    assert dp.status() == 0
