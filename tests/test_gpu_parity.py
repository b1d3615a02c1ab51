"""GPU parity: every kernel through the C-ABI vs the reference's golden vectors
and vs the CPU oracle on seeded inputs; size-independent properties at the
benchmark size. Bit-exact (integer/byte/index work)."""
import numpy as np
import pytest

import ttga
from oracle_lib import oracle

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")
from ttga import native  # noqa: E402

NAMES = ["sm", "med", "tight"]
# tt_eval kernels: 2 eval_block, 7/8 eval_tile5 (4/8 waves), 13 wide path (eval_lanes<16> + eval_corr)
EVAL_VARIANTS = [2, 7, 8, 13]


def load(golden_dir, name):
    z = np.load(golden_dir / f"{name}.npz")
    E, R, F, S = (int(x) for x in z["dims"])
    inst = ttga.Instance(E, R, F, S, z["room_size"], z["student_events"], z["room_features"], z["event_features"])
    return inst, z


def dev(a):
    return torch.from_numpy(np.ascontiguousarray(a)).cuda()


def host(t):
    torch.cuda.synchronize()
    return t.cpu().numpy()


@pytest.fixture(scope="module")
def orc():
    return oracle()


@pytest.fixture(scope="module")
def problems(golden_dir):
    out = {}
    for n in NAMES:
        inst, z = load(golden_dir, n)
        out[n] = (native.DeviceProblem(inst), inst, z)
    return out


@pytest.mark.parametrize("name", NAMES)
def test_derived_matches_reference(problems, name):
    dp, inst, z = problems[name]
    sn, corr, poss = dp.derived()
    assert np.array_equal(sn, z["ref_student_number"])
    assert np.array_equal(np.packbits(corr.astype(np.uint8), axis=1), z["ref_corr_bits"])
    assert np.array_equal(poss, z["ref_possible"])


@pytest.mark.parametrize("variant", EVAL_VARIANTS)
@pytest.mark.parametrize("name", NAMES)
@pytest.mark.parametrize("tag,sk,rk", [("canon", "slots", "rooms"), ("rand", "slots", "rand_rooms"),
                                       ("skew", "skew_slots", "skew_rooms"), ("edge", "edge_slots", "edge_rooms"),
                                       ("ls3", "ls3_slots", "ls3_rooms")])
def test_eval_golden(problems, name, tag, sk, rk, variant):
    dp, inst, z = problems[name]
    hcv, scv, feas, pen = (host(t) for t in dp.eval(dev(z[sk]), dev(z[rk]), variant=variant))
    assert np.array_equal(hcv, z[f"eval_{tag}_hcv"])
    assert np.array_equal(scv, z[f"eval_{tag}_scv"])
    assert np.array_equal(feas, z[f"eval_{tag}_feasible"])
    assert np.array_equal(pen, z[f"eval_{tag}_penalty"])


@pytest.mark.parametrize("variant", EVAL_VARIANTS)
@pytest.mark.parametrize("dims", [(333, 9, 6, 170), (320, 24, 5, 150), (250, 40, 4, 120), (448, 11, 5, 300)],
                         ids=["E333R9", "E320R24", "E250R40", "E448R11"])
def test_eval_random_vs_oracle(orc, variant, dims):
    """Ragged P; E not a multiple of 16 (byte staging path) or of 64; room masks
    packed with studentNumber (R <= 16), u32 (R <= 32) and u64 (R = 40)."""
    inst = ttga.generate(*dims, seed=11)
    dp = native.DeviceProblem(inst)
    P = 203                                            # ragged last wave
    slots, _ = ttga.random_slots(ttga.population_seeds(4242, P), inst.E)
    rng = np.random.default_rng(5)
    rooms = rng.integers(0, inst.R, size=(P, inst.E), dtype=np.uint8)
    rooms[::3] = orc.problem(inst).assign_rooms(slots[::3])
    got = [host(t) for t in dp.eval(dev(slots), dev(rooms), variant=variant)]
    exp = orc.problem(inst).eval(slots, rooms)
    for g, e in zip(got, exp):
        assert np.array_equal(g, e)


@pytest.mark.parametrize("dims", [(1000, 20, 6, 700), (1531, 64, 8, 900), (2430, 33, 5, 600), (449, 10, 5, 200)],
                         ids=["E1000R20", "E1531R64", "E2430R33", "E449R10"])
def test_eval_wide_vs_oracle(orc, dims):
    """Instances beyond eval_tile5 (E > 448): the wide path (variant 13, the
    automatic choice there) and the workgroup kernel against the oracle; E not a
    multiple of 4 (byte row loads), R = 64 (full room masks), E = 2430 (more
    chunk pairs than waves: eval_corr reloads its words per round), and the
    first E past eval_tile5."""
    inst = ttga.generate(*dims, seed=13)
    dp = native.DeviceProblem(inst)
    assert dp.eval_variant() == 13
    P = 133
    slots, _ = ttga.random_slots(ttga.population_seeds(777, P), inst.E)
    rng = np.random.default_rng(9)
    rooms = rng.integers(0, inst.R, size=(P, inst.E), dtype=np.uint8)
    rooms[::2] = orc.problem(inst).assign_rooms(slots[::2])
    exp = orc.problem(inst).eval(slots, rooms)
    slots[5, inst.E - 1] = 45                          # invalid gene in the last (partial) chunk: sentinels
    slots[6, 0] = 255                                  # and at the first event
    rooms[7, inst.E // 2] = inst.R                     # an invalid room
    for q in (5, 6, 7):
        exp[0][q] = exp[1][q] = exp[3][q] = -1
        exp[2][q] = 0
    for v in (2, 13):
        got = [host(t) for t in dp.eval(dev(slots), dev(rooms), variant=v)]
        for g, e in zip(got, exp):
            assert np.array_equal(g, e), v


def test_eval_invalid_individual_flagged(problems):
    dp, inst, z = problems["sm"]
    s = z["slots"][:3].copy()
    r = z["rooms"][:3].copy()
    s[1, 7] = 45
    r[2, 3] = inst.R
    for variant in EVAL_VARIANTS:
        hcv, scv, feas, pen = (host(t) for t in dp.eval(dev(s), dev(r), variant=variant))
        assert hcv[0] == z["eval_canon_hcv"][0]
        assert list(hcv[1:]) == [-1, -1] and list(pen[1:]) == [-1, -1] and list(feas[1:]) == [0, 0]


def test_eval_empty_population(problems):
    dp, inst, z = problems["sm"]
    e = torch.empty((0, inst.E), dtype=torch.uint8, device="cuda")
    dp.eval(e, e)


def test_eval_bench_size_properties(orc):
    """P = 65536 on the headline instance: the eval kernels (tile5, the wide
    path, the workgroup kernel) agree on every individual, a strided sample matches the oracle, and feasibility
    <=> hcv == 0 with penalty = feasible ? scv : 1e6 + hcv."""
    inst = ttga.config_instance("med")
    dp = native.DeviceProblem(inst)
    P = 65536
    g = torch.Generator(device="cuda").manual_seed(0)
    slot = torch.randint(0, 45, (P, inst.E), dtype=torch.uint8, device="cuda", generator=g)
    room = dp.assign_rooms(slot)
    a = [host(t) for t in dp.eval(slot, room, variant=8)]
    # plus eval_tile5's two grids forced: 8 | 64 << 4 persistent (the default with the
    # second tile buffer), 8 | 128 << 4 one tile per workgroup
    for v in [v for v in EVAL_VARIANTS if v != 8] + [8 | (64 << 4), 8 | (128 << 4)]:
        b = [host(t) for t in dp.eval(slot, room, variant=v)]
        for x, y in zip(a, b):
            assert np.array_equal(x, y)
    hcv, scv, feas, pen = a
    assert np.array_equal(feas.astype(bool), hcv == 0)
    assert np.array_equal(pen, np.where(hcv == 0, scv, 1000000 + hcv))
    idx = np.arange(0, P, 1021)
    s_np, r_np = host(slot)[idx], host(room)[idx]
    exp = orc.problem(inst).eval(s_np, r_np)
    assert np.array_equal(orc.problem(inst).assign_rooms(s_np), r_np)
    for x, e in zip(a, exp):
        assert np.array_equal(x[idx], e)
    assert dp.status() == 0


@pytest.mark.parametrize("name", NAMES)
def test_assign_rooms_golden(problems, name):
    dp, inst, z = problems[name]
    assert np.array_equal(host(dp.assign_rooms(dev(z["slots"]))), z["rooms"])
    assert np.array_equal(host(dp.assign_rooms(dev(z["skew_slots"]))), z["skew_rooms"])   # N > 64 per slot
    assert dp.status() == 0


def test_assign_rooms_random_vs_oracle(orc):
    # R = 16 / 17 and slots of exactly 32 / 33 events sit on the register
    # matcher's limits (N <= 32, R <= 16, TT_MATCH_REG), crowded slots past them
    for seed, dims in [(21, (250, 12, 4, 150)), (22, (600, 30, 6, 300)), (23, (300, 16, 4, 150)),
                       (24, (300, 17, 4, 150))]:
        inst = ttga.generate(*dims, seed=seed)
        dp = native.DeviceProblem(inst)
        slots, _ = ttga.random_slots(ttga.population_seeds(seed, 97), inst.E)
        slots[:10] = (slots[:10] % 4) * 11     # crowded slots
        for r, n in ((10, 32), (11, 33), (12, 31)):
            slots[r, :n] = 7
            slots[r, n:] = np.where(slots[r, n:] == 7, 8, slots[r, n:])
        assert np.array_equal(host(dp.assign_rooms(dev(slots))), orc.problem(inst).assign_rooms(slots))


@pytest.mark.parametrize("name", NAMES)
def test_random_init_crossover_mutation_golden(problems, name):
    dp, inst, z = problems[name]
    n = z["init_seeds"].size
    rng = dev(z["init_seeds"]); s = dev(np.zeros((n, inst.E), np.uint8)); r = dev(np.zeros((n, inst.E), np.uint8))
    dp.random_init(rng, s, r)
    assert np.array_equal(host(s), z["init_slots"]) and np.array_equal(host(r), z["init_rooms"])
    assert np.array_equal(host(rng), z["init_rng"])
    h = n // 2
    rng = dev(z["xover_seeds"]); cs = dev(np.zeros((h, inst.E), np.uint8)); cr = dev(np.zeros((h, inst.E), np.uint8))
    dp.crossover(dev(z["init_slots"][:h]), dev(z["init_slots"][h:]), rng, cs, cr)
    assert np.array_equal(host(cs), z["xover_slots"]) and np.array_equal(host(cr), z["xover_rooms"])
    assert np.array_equal(host(rng), z["xover_rng"])
    rng = dev(z["mut_seeds"]); ms = dev(z["init_slots"]); mr = dev(z["init_rooms"])
    dp.mutation(ms, mr, rng)
    assert np.array_equal(host(ms), z["mut_slots"]) and np.array_equal(host(mr), z["mut_rooms"])
    assert np.array_equal(host(rng), z["mut_rng"])


def test_syn_scale_instance(orc):
    """Synthetic 2000/40/10/5000 instance (BASELINE configs[4]): tt_eval takes the
    wide path; it agrees with the workgroup kernel on every individual and with
    the oracle (rooms and all four outputs) on 64 of them."""
    inst = ttga.config_instance("syn")
    dp = native.DeviceProblem(inst)
    assert dp.eval_variant() == 13
    P = 512
    slots, _ = ttga.random_slots(ttga.population_seeds(31, P), inst.E)
    room = dp.assign_rooms(dev(slots))
    hcv, scv, feas, pen = (host(t) for t in dp.eval(dev(slots), room))
    for x, y in zip((hcv, scv, feas, pen), (host(t) for t in dp.eval(dev(slots), room, variant=2))):
        assert np.array_equal(x, y)
    idx = np.arange(0, P, 8)                             # 64 individuals against the oracle
    o = orc.problem(inst)
    r_np = host(room)[idx]
    assert np.array_equal(o.assign_rooms(slots[idx]), r_np)
    exp = o.eval(slots[idx], r_np)
    for x, e in zip((hcv, scv, feas, pen), exp):
        assert np.array_equal(x[idx], e)


@pytest.mark.parametrize("name", NAMES)
def test_local_search_golden(problems, name):
    """Solution::localSearch replayed on the GPU: phase 1 from random init
    (200 steps), chained to 1000 and 2000 steps (phase 2 once feasible), and a
    Move3-enabled run (prob3 = 1) — slots, rooms and final RNG state exact."""
    dp, inst, z = problems[name]
    n = z["ls_seeds"].size
    s, r, g = dev(z["init_slots"][:n]), dev(z["init_rooms"][:n]), dev(z["ls_seeds"])
    for steps, tag in ((200, "ls"), (1000, "ls2"), (2000, "ls3")):
        dp.local_search(s, r, g, steps)
        assert np.array_equal(host(s), z[f"{tag}_slots"]), tag
        assert np.array_equal(host(r), z[f"{tag}_rooms"]), tag
        assert np.array_equal(host(g), z[f"{tag}_rng"]), tag
    s, r = dev(z["init_slots"][:4]), dev(z["init_rooms"][:4])
    g = dev(ttga.population_seeds(9500, 4))
    dp.local_search(s, r, g, 60, 1.0, 1.0, 1.0)
    assert np.array_equal(host(s), z["lsp3_slots"]) and np.array_equal(host(r), z["lsp3_rooms"])
    assert np.array_equal(host(g), z["lsp3_rng"])
    assert dp.status() == 0


def test_local_search_random_vs_oracle(orc):
    inst = ttga.generate(180, 7, 4, 140, seed=17)
    dp = native.DeviceProblem(inst)
    o = orc.problem(inst)
    P = 24
    s0, r0, _ = o.random_init(ttga.population_seeds(606, P))
    seeds = ttga.population_seeds(707, P)
    s, r, g = dev(s0), dev(r0), dev(seeds)
    dp.local_search(s, r, g, 500)
    es, er, eg = o.local_search(s0, r0, seeds, 500)
    assert np.array_equal(host(s), es) and np.array_equal(host(r), er) and np.array_equal(host(g), eg)
    # chained into phase 2
    dp.local_search(s, r, g, 3000)
    es, er, eg = o.local_search(es, er, eg, 3000)
    assert np.array_equal(host(s), es) and np.array_equal(host(r), er) and np.array_equal(host(g), eg)


@pytest.mark.parametrize("name", ["tight", "med"])
def test_local_search_noncanonical_rooms_vs_oracle(orc, problems, name):
    """The phase-1 room-pair bounds (TT_LS_P1B) use a slot's rooms as a maximum
    matching only after checking that no augmenting path exists: localSearch
    from random slots with rooms that assignRooms would not give (random, and
    all room 0), on the tight instance (27 events without a possible room) and
    med, against the oracle."""
    dp, inst, z = problems[name]
    o = orc.problem(inst)
    P = 32
    slots, _ = ttga.random_slots(ttga.population_seeds(3131, P), inst.E)
    rng = np.random.default_rng(9)
    rooms = rng.integers(0, inst.R, size=(P, inst.E), dtype=np.uint8)
    rooms[::2] = 0
    seeds = ttga.population_seeds(3232, P)
    s, r, g = dev(slots), dev(rooms), dev(seeds)
    dp.local_search(s, r, g, 300)
    es, er, eg = o.local_search(slots, rooms, seeds, 300)
    assert np.array_equal(host(s), es) and np.array_equal(host(r), er) and np.array_equal(host(g), eg)
    assert dp.status() == 0


def test_local_search_med_population_vs_oracle(orc):
    """BASELINE configs[1] at a parity size: the med instance, 96 individuals
    from RandomInitialSolution, localSearch(200), then chained localSearch(1000)
    and (3000) into phase 2, then eval -- every slot, room, RNG state and output
    against the oracle (Solution.cpp:471-769)."""
    inst = ttga.config_instance("med")
    dp = native.DeviceProblem(inst)
    o = orc.problem(inst)
    P = 96
    s0, r0, _ = o.random_init(ttga.population_seeds(4242, P))
    seeds = ttga.population_seeds(4343, P)
    s, r, g = dev(s0), dev(r0), dev(seeds)
    es, er, eg = s0, r0, seeds
    for steps in (200, 1000, 3000):
        dp.local_search(s, r, g, steps)
        es, er, eg = o.local_search(es, er, eg, steps)
        assert np.array_equal(host(s), es) and np.array_equal(host(r), er) and np.array_equal(host(g), eg), steps
    got = [host(t) for t in dp.eval(s, r)]
    for x, e in zip(got, o.eval(es, er)):
        assert np.array_equal(x, e)
    assert 0 < int(got[2].sum()) < P          # both phases met (some individuals feasible, some not)
    assert dp.status() == 0


def test_local_search_ordered_dispatch():
    """tt_local_search_ordered: any dispatch order gives tt_local_search's
    results (slots, rooms, RNG states), on the small-task + redo path too."""
    for name, P in (("med", 150), ("sm", 70)):
        inst = ttga.config_instance(name)
        dp = native.DeviceProblem(inst)
        seeds = ttga.population_seeds(515, P)
        s0 = dev(ttga.random_slots(seeds, inst.E)[0])
        r0 = dp.assign_rooms(s0)
        runs = []
        for order in (None, torch.randperm(P, generator=torch.Generator().manual_seed(3)).int().cuda()):
            s, r, g = s0.clone(), r0.clone(), dev(ttga.population_seeds(616, P))
            dp.local_search(s, r, g, 400, order=order)
            runs.append((host(s), host(r), host(g)))
        for a, b in zip(*runs):
            assert np.array_equal(a, b), name


def test_local_search_mask_policy_same_results(orc):
    """The phase-2 student masks of call k on a stream are launched or not by
    the phase-2 share of call k - 2's steps (tt_local_search_stats), waited for
    if needed, so the launch shape depends only on the call sequence: on med at
    8,192 individuals (where the masks cost resident waves) the first two calls
    on a fresh stream have no share to go by and run without them, the third,
    after a phase-2-heavy first call, with them; all three give the same slots,
    rooms and RNG states, and a strided sample matches the oracle. The
    statistics count phase-2 steps only for individuals that reached phase 2."""
    inst = ttga.config_instance("med")
    dp = native.DeviceProblem(inst)
    P = 8192
    s0 = dev(ttga.random_slots(ttga.population_seeds(321, P), inst.E)[0])
    r0 = dp.assign_rooms(s0)
    dp.local_search(s0, r0, dev(ttga.population_seeds(432, P)), 3000)
    feas = np.flatnonzero(host(dp.eval(s0, r0)[2]))
    assert len(feas) > 0
    pick = torch.from_numpy(feas[np.arange(P) % len(feas)]).cuda()     # feasible individuals only: phase 2 heavy
    s0, r0 = s0[pick].contiguous(), r0[pick].contiguous()
    st = torch.cuda.Stream()
    st.wait_stream(torch.cuda.current_stream())
    runs, masks = [], []
    with torch.cuda.stream(st):
        assert dp.local_search_stats(st) == (0, 0) and dp.local_search_masks(st) == -1
        for k in range(3):
            s, r, g = s0.clone(), r0.clone(), dev(ttga.population_seeds(543, P))
            dp.local_search(s, r, g, 1000)          # no synchronisation between the calls
            masks.append(dp.local_search_masks(st))
            runs.append((s, r, g))
        st.synchronize()
        ph2, allsteps = dp.local_search_stats(st)
        assert 0 < ph2 <= allsteps
        assert ph2 >= 0.5 * allsteps                       # phase-2 heavy: call 3 takes the masks
    assert masks == [0, 0, inst.S], masks
    runs = [tuple(host(t) for t in x) for x in runs]
    for other in runs[1:]:
        for a, b in zip(runs[0], other):
            assert np.array_equal(a, b)
    idx = np.arange(0, P, 257)
    es, er, eg = orc.problem(inst).local_search(host(s0)[idx], host(r0)[idx], ttga.population_seeds(543, P)[idx], 1000)
    assert np.array_equal(runs[2][0][idx], es) and np.array_equal(runs[2][1][idx], er)
    assert np.array_equal(runs[2][2][idx], eg)
    assert dp.status() == 0


def test_local_search_crowded_slots_redo(orc):
    """tt_local_search runs a first launch whose matcher tasks hold 64 events per
    slot; an individual whose trial touches a slot with more events is redone
    from its untouched input by the full-size launch. Crowded individuals (70 to
    150 events in one slot) mixed with ordinary ones must match the oracle
    exactly, with the device status clean."""
    inst = ttga.generate(400, 10, 5, 200, seed=23)
    dp = native.DeviceProblem(inst)
    o = orc.problem(inst)
    P = 12
    s0, _, _ = o.random_init(ttga.population_seeds(808, P))
    rng = np.random.default_rng(3)
    for k, n in ((1, 70), (4, 100), (7, 150), (10, 65)):
        idx = rng.choice(inst.E, size=n, replace=False)
        s0[k, idx] = 3 + k                                # one crowded slot
    r0 = o.assign_rooms(s0)
    seeds = ttga.population_seeds(909, P)
    s, r, g = dev(s0), dev(r0), dev(seeds)
    dp.local_search(s, r, g, 300)
    es, er, eg = o.local_search(s0, r0, seeds, 300)
    assert np.array_equal(host(s), es) and np.array_equal(host(r), er) and np.array_equal(host(g), eg)
    assert dp.status() == 0


def test_local_search_redo_list_reuse(orc):
    """The per-stream redo list persists across calls: the redo launch resets
    its count and arrival counter on the device, and a call with a larger
    population regrows it. Three chained calls on one stream -- crowded
    individuals at P = 12, again at P = 12, then at P = 40 (regrown) -- each
    equal the oracle, with the status clean after every call."""
    inst = ttga.generate(400, 10, 5, 200, seed=23)
    dp = native.DeviceProblem(inst)
    o = orc.problem(inst)
    rng = np.random.default_rng(5)
    for call, P in enumerate((12, 12, 40)):
        s0, _, _ = o.random_init(ttga.population_seeds(1808 + call, P))
        for k in range(1, P, 3):
            idx = rng.choice(inst.E, size=int(rng.integers(65, 150)), replace=False)
            s0[k, idx] = int(rng.integers(0, 45))           # one crowded slot
        r0 = o.assign_rooms(s0)
        seeds = ttga.population_seeds(1909 + call, P)
        s, r, g = dev(s0), dev(r0), dev(seeds)
        dp.local_search(s, r, g, 250)
        es, er, eg = o.local_search(s0, r0, seeds, 250)
        assert np.array_equal(host(s), es) and np.array_equal(host(r), er) and np.array_equal(host(g), eg), call
        assert dp.status() == 0, call


@pytest.mark.parametrize("p1,p2", [(1.0, 1.0), (0.7, 0.4)])
def test_local_search_phase2_vs_oracle(orc, p1, p2):
    """Mostly-feasible individuals (3000 steps from random init), then a chained
    run that starts in phase 2 (Solution.cpp:619-768): the lazy matching of the
    trial neighbours (exact lower-bound rejection before the target slot is
    matched, the old slot matched only for an accepted Move1) must keep slots,
    rooms and RNG states identical to the oracle."""
    inst = ttga.generate(300, 12, 4, 150, seed=31)
    dp = native.DeviceProblem(inst)
    o = orc.problem(inst)
    P = 32
    s0, r0, _ = o.random_init(ttga.population_seeds(1201, P))
    seeds = ttga.population_seeds(1301, P)
    s, r, g = dev(s0), dev(r0), dev(seeds)
    dp.local_search(s, r, g, 3000, p1, p2)
    es, er, eg = o.local_search(s0, r0, seeds, 3000, p1, p2)
    assert np.array_equal(host(s), es) and np.array_equal(host(r), er) and np.array_equal(host(g), eg)
    assert int(o.eval(es, er)[2].sum()) >= P // 2          # phase 2 is exercised below
    dp.local_search(s, r, g, 2000, p1, p2)
    es, er, eg = o.local_search(es, er, eg, 2000, p1, p2)
    assert np.array_equal(host(s), es) and np.array_equal(host(r), er) and np.array_equal(host(g), eg)
    assert dp.status() == 0


def _hot_events(inst, s, r):
    """Per individual: events with eventHcv > 0 (Solution.cpp:173-191: room
    clashes in its slot and room plus correlated events in its slot)."""
    A = inst.student_events.astype(np.int64)
    C = (A.T @ A) > 0
    np.fill_diagonal(C, False)
    out = []
    for sl, rm in zip(s, r):
        same_slot = sl[:, None] == sl[None, :]
        clash = same_slot & (rm[:, None] == rm[None, :])
        np.fill_diagonal(clash, False)
        out.append(int(((clash | (C & same_slot)).any(axis=1)).sum()))
    return np.array(out)


def test_local_search_flagged_events_vs_oracle(orc):
    """GA-child-like starts: feasible individuals with one to three events moved
    to random slots, so only a few events have eventHcv > 0 and phase 1 visits
    them through the eventHcv flags (TT_LS_HOT: the unflagged events skipped 64
    scramble positions at a time, the flags refreshed after every accepted move).
    Slots, rooms and RNG states identical to the oracle's localSearch."""
    inst = ttga.generate(300, 12, 4, 150, seed=31)
    dp = native.DeviceProblem(inst)
    o = orc.problem(inst)
    P = 48
    s0, r0, _ = o.random_init(ttga.population_seeds(2201, P))
    s1, r1, _ = o.local_search(s0, r0, ttga.population_seeds(2301, P), 3000)
    feas = o.eval(s1, r1)[2].astype(bool)
    assert feas.sum() >= P // 2
    rng = np.random.default_rng(7)
    s2 = s1[feas].copy()
    for k in range(s2.shape[0]):
        idx = rng.choice(inst.E, size=int(rng.integers(1, 4)), replace=False)
        s2[k, idx] = rng.integers(0, 45, size=idx.size)
    r2 = o.assign_rooms(s2)
    hot = _hot_events(inst, s2, r2)
    assert (hot > 0).sum() >= s2.shape[0] // 2 and (4 * hot <= inst.E).all()   # the flagged path runs
    seeds = ttga.population_seeds(2401, s2.shape[0])
    for steps in (200, 1000):
        s, r, g = dev(s2), dev(r2), dev(seeds)
        dp.local_search(s, r, g, steps)
        es, er, eg = o.local_search(s2, r2, seeds, steps)
        assert np.array_equal(host(s), es) and np.array_equal(host(r), er) and np.array_equal(host(g), eg), steps
        assert dp.status() == 0


def test_rng_edge_seeds_vs_oracle(orc):
    """Park-Miller states outside [0, 2^31 - 1) take the 64-bit Schrage path on
    their first draw (Random.cc:27-37; every later state is in range and takes
    the 32-bit path): zero, negative, 2^31 and beyond, through random init and
    local search, against the oracle."""
    inst = ttga.generate(120, 6, 4, 90, seed=41)
    dp = native.DeviceProblem(inst)
    o = orc.problem(inst)
    # (seeds whose first draw leaves [0, 2^31 - 1), e.g. 2^40, give the reference
    # negative or >= 1 draws and out-of-range slots: undefined there, not tested)
    seeds = np.array([0, 1, -1, -123456789, -2_000_000_000, 2**31 - 2, 2**31 - 1, 2**31, 2**31 + 5,
                      3_000_000_000, 4_000_000_000, 42], dtype=np.int64)
    es, er, eg = o.random_init(seeds.copy())
    s = torch.empty((seeds.size, inst.E), dtype=torch.uint8, device="cuda")
    r = torch.empty_like(s)
    g = dev(seeds.copy())
    dp.random_init(g, s, r)
    assert np.array_equal(host(s), es) and np.array_equal(host(r), er) and np.array_equal(host(g), eg)
    g = dev(seeds.copy())
    dp.local_search(s, r, g, 300)
    ls, lr, lg = o.local_search(es, er, seeds.copy(), 300)
    assert np.array_equal(host(s), ls) and np.array_equal(host(r), lr) and np.array_equal(host(g), lg)


@pytest.mark.parametrize("dims,p1,p2", [((50, 5, 4, 40), 1.0, 1.0), ((120, 6, 4, 90), 0.9, 0.35)],
                         ids=["E50", "E120_p"])
def test_local_search_step_budget_windows(orc, dims, p1, p2):
    """The local search screens up to 64 trials per pass (one per lane, with
    Park-Miller jump-ahead draws) and must stop exactly where the reference's
    step budget stops it: many small maxSteps values, so the budget runs out
    inside a window at every offset, from random init (phase 1) and from
    mostly feasible individuals (phase 2); E < 64 (windows wrapping the event
    ring more than once) and draw probabilities below 1."""
    inst = ttga.generate(*dims, seed=19)
    dp = native.DeviceProblem(inst)
    o = orc.problem(inst)
    P = 16
    s0, r0, _ = o.random_init(ttga.population_seeds(2101, P))
    f_s, f_r, _ = o.local_search(s0, r0, ttga.population_seeds(2201, P), 4000, p1, p2)
    for start_s, start_r in ((s0, r0), (f_s, f_r)):
        for steps in (1, 2, 5, 9, 17, 33, 64, 65, 130):
            seeds = ttga.population_seeds(2301 + steps, P)
            s, r, g = dev(start_s), dev(start_r), dev(seeds)
            dp.local_search(s, r, g, steps, p1, p2)
            es, er, eg = o.local_search(start_s, start_r, seeds, steps, p1, p2)
            assert np.array_equal(host(s), es) and np.array_equal(host(r), er) and np.array_equal(host(g), eg), steps
    assert dp.status() == 0


@pytest.mark.parametrize("dims,crowd,steps", [((50, 5, 4, 40), False, 300), ((400, 10, 5, 200), True, 400),
                                              ((300, 12, 4, 150), False, 3000), ((449, 40, 5, 220), True, 300)],
                         ids=["E50_small_path", "E400_redo", "E300_phase2", "E449R40_redo"])
def test_local_search_eval_outputs_vs_eval(orc, dims, crowd, steps):
    """tt_local_search_eval: the searched individuals' hcv, scv, feasible and
    penalty computed at the end of the search launch (localSearch then
    computePenalty, ga.cpp:574-575) equal tt_eval of the searched rows and the
    oracle, on the one-launch path (E <= 64), through the redo launch
    (crowded slots), into phase 2, with R > 16, and with an invalid genome
    (left untouched, -1 sentinels); slots, rooms and RNG states equal
    tt_local_search's."""
    inst = ttga.generate(*dims, seed=47)
    dp = native.DeviceProblem(inst)
    o = orc.problem(inst)
    P = 40
    s0, r0, _ = o.random_init(ttga.population_seeds(4700, P))
    if crowd:
        rng = np.random.default_rng(2)
        for k in range(1, P, 5):
            s0[k, rng.choice(inst.E, size=int(rng.integers(65, 120)), replace=False)] = int(rng.integers(0, 45))
        r0 = o.assign_rooms(s0)
    s0[7, 3] = 45                                          # an invalid genome
    seeds = ttga.population_seeds(4800, P)
    s, r, g = dev(s0), dev(r0), dev(seeds)
    out = (torch.empty(P, dtype=torch.int32, device="cuda"), torch.empty(P, dtype=torch.int32, device="cuda"),
           torch.empty(P, dtype=torch.uint8, device="cuda"), torch.empty(P, dtype=torch.int32, device="cuda"))
    dp.local_search(s, r, g, steps, out=out)
    s2, r2, g2 = dev(s0), dev(r0), dev(seeds)
    dp.local_search(s2, r2, g2, steps)
    for a, b in zip((s, r, g), (s2, r2, g2)):
        assert np.array_equal(host(a), host(b))
    got = [host(t) for t in out]
    ev = [host(t) for t in dp.eval(s, r)]
    for x, e in zip(got, ev):
        assert np.array_equal(x, e)
    assert got[0][7] == -1 and got[3][7] == -1 and got[2][7] == 0
    ok = np.arange(P) != 7
    es, er, eg = o.local_search(s0[ok], r0[ok], seeds[ok], steps)
    assert np.array_equal(host(s)[ok], es) and np.array_equal(host(r)[ok], er)
    for x, e in zip(got, o.eval(es, er)):
        assert np.array_equal(x[ok], e)
    assert dp.status() == 2                                # bit 1: the invalid genome met by the search
