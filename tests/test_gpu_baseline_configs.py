"""BASELINE.json configurations at (or from) their full sizes on the GPU,
checked against the CPU oracle (and the reference's own per-child path):

* configs[2] ITC-2002 comp01 / comp10 / comp20: whole island generations
  (Island.step: breed, LPT-ordered localSearch(1000), eval, replace-worst +
  sort) into the phase-2 regime (feasible children), bit-exact with the oracle
  GA (ga.cpp:543-585); and 256 device children of a comp01 generation against
  the reference's own per-child path (oracle/_ref ref_ga_children,
  ga.cpp:543-577) on the same streams;
* configs[1] medium01-size, population 4096: localSearch(200) then (1000),
  then a chained (3000) into phase 2, on the whole population, a 16-strided
  sample of 256 against the oracle
  (Solution.cpp:471-769), whole-population properties;
* configs[4] synthetic 2000/40/10/5000, population 262,144: RandomInitialSolution
  and tt_eval on the whole population, a 512-strided sample against the
  oracle (Solution.cpp:48-170), whole-population properties.

The oracle runs on host threads (tests/oracle_lib.split_rows).
"""
import numpy as np
import pytest

import ttga
from oracle_lib import oracle, ref, split_rows

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


def o_local_search(o, s, r, g, steps):
    return split_rows(lambda a, b, c: o.local_search(a, b, c, steps), (s, r, g))


def o_eval(o, s, r):
    return split_rows(o.eval, (s, r))


def o_breed(o, pop, seeds, C, p_cross=0.8, p_mut=0.5):
    return split_rows(lambda g: o.ga_breed(pop["slot"], pop["room"], pop["penalty"], g, g.size, p_cross, p_mut, 1),
                      (seeds,))


# ---------------------------------------------------------------- configs[2]
@pytest.mark.parametrize("name", ["comp01", "comp10", "comp20"])
def test_comp_ga_generations_vs_oracle(orc, name):
    """Island generations on a comp instance (N = 64, C = 32, maxSteps 1000,
    LPT dispatch forced on) from a population of long local searches
    (random init + localSearch(20000), near feasible), for at least 8
    generations and until feasible (phase-2) children have occurred (at most
    32): the population, its order and every child stream equal the oracle
    GA's after every generation."""
    inst = ttga.config_instance(name)
    dp = native.DeviceProblem(inst)
    o = orc.problem(inst)
    N, C, min_gens, max_gens, seed, init_steps = 64, 32, 8, 32, 7, 20000
    isl = Island(dp, pop_size=N, children=C, max_steps=init_steps, seed=seed, lpt=True)
    isl.initialize()
    isl.max_steps = 1000
    # the oracle's initial population: ga.cpp:429-434 with the same streams, then sorted
    s, r, g = o.random_init(stream_seeds(seed, 0, N))
    s, r, g = o_local_search(o, s, r, g, init_steps)
    h, sc, f, p = o_eval(o, s, r)
    pop = dict(slot=s, room=r, hcv=h, scv=sc, feasible=f, penalty=p)
    pop = o.ga_replace(pop, {k: v[:0] for k, v in pop.items()})
    for k in KEYS:
        assert np.array_equal(host(isl.pop[k]), pop[k]), ("init", k)
    assert np.array_equal(host(isl.rng_init), g)
    rng = stream_seeds(seed, N, C)
    feasible_children = 0
    gen = 0
    while gen < min_gens or (feasible_children == 0 and gen < max_gens):
        isl.step()
        cs, cr, fl, rng = o_breed(o, pop, rng, C)
        cs, cr, rng = o_local_search(o, cs, cr, rng, 1000)
        h, sc, f, p = o_eval(o, cs, cr)
        feasible_children += int(f.sum())
        assert np.array_equal(host(isl.child["penalty"]), p), (gen, "children")
        pop = o.ga_replace(pop, dict(slot=cs, room=cr, hcv=h, scv=sc, feasible=f, penalty=p))
        for k in KEYS:
            assert np.array_equal(host(isl.pop[k]), pop[k]), (gen, k)
        assert np.array_equal(host(isl.rng_child), rng), gen
        gen += 1
    assert feasible_children > 0, "no phase-2 child met: the test did not reach the GA's phase-2 regime"
    assert np.all(np.diff(pop["penalty"].astype(np.int64)) >= 0)
    assert dp.status() == 0


def test_comp01_children_vs_reference_per_child_path():
    """256 children of one comp01 generation (maxSteps 1000) bred, searched and
    evaluated on the device (tt_ga_breed with the 3E discarded draws,
    tt_local_search, tt_eval) equal the reference's own per-child path of
    ga.cpp:543-577 run by its Solution objects (oracle/_ref ref_ga_children:
    three RandomInitialSolution, two selection5, copies, crossover into a
    fresh child or copy, mutation, localSearch, computePenalty) on the same
    per-child streams: slots, rooms, hcv, scv, feasible, penalty, final RNG."""
    R = ref()
    if R is None:
        pytest.skip("reference build oracle/_ref not present")
    inst = ttga.config_instance("comp01")
    dp = native.DeviceProblem(inst)
    N, C, steps = 512, 256, 1000
    isl = Island(dp, pop_size=N, children=C, max_steps=3000, seed=99)
    isl.initialize()
    pop = {k: host(v) for k, v in isl.pop.items()}
    seeds = stream_seeds(99, N, C)
    c = {k: torch.empty_like(v[:C]) for k, v in isl.pop.items()}
    flags, g = torch.zeros(C, dtype=torch.uint8, device="cuda"), dev(seeds)
    dp.ga_breed(isl.pop["slot"], isl.pop["room"], isl.pop["penalty"], g, c["slot"], c["room"], flags, 0.8, 0.5, True)
    dp.local_search(c["slot"], c["room"], g, steps)
    dp.eval(c["slot"], c["room"], out=(c["hcv"], c["scv"], c["feasible"], c["penalty"]))
    fl = host(flags)
    assert (fl & 1).any() and (fl & 1 == 0).any() and (fl & 2).any()
    exp, erng, _ = R.problem(inst).ga_children(pop["slot"], pop["room"], pop["penalty"], seeds, steps,
                                                threads=__import__("oracle_lib").host_threads())
    for k in KEYS:
        assert np.array_equal(host(c[k]), exp[k]), k
    assert np.array_equal(host(g), erng)


# ---------------------------------------------------------------- configs[1]
def test_med_local_search_pop4096_sampled(orc):
    """configs[1] at its full size: 4096 med individuals from
    RandomInitialSolution, localSearch(200), then localSearch(1000) on the
    device (phase 1: 1,200 steps from random init reach no feasible
    individual), then a chained localSearch(3000) into phase 2; every 16th
    individual (256) against the oracle after each call (slots, rooms, RNG),
    then eval; whole population: eval equals the workgroup kernel, feasible
    <=> hcv == 0, penalty formula, status clean."""
    inst = ttga.config_instance("med")
    dp = native.DeviceProblem(inst)
    o = orc.problem(inst)
    P, stride = 4096, 16
    seeds = ttga.population_seeds(8080, P)
    g = dev(seeds)
    s = torch.empty((P, inst.E), dtype=torch.uint8, device="cuda")
    r = torch.empty_like(s)
    dp.random_init(g, s, r)
    idx = np.arange(0, P, stride)
    es, er, eg = o.random_init(seeds[idx])
    assert np.array_equal(host(s)[idx], es) and np.array_equal(host(r)[idx], er) and np.array_equal(host(g)[idx], eg)
    for steps in (200, 1000, 3000):
        dp.local_search(s, r, g, steps)
        es, er, eg = o_local_search(o, es, er, eg, steps)
        hs, hr, hg = host(s), host(r), host(g)
        assert np.array_equal(hs[idx], es) and np.array_equal(hr[idx], er) and np.array_equal(hg[idx], eg), steps
    out = [host(t) for t in dp.eval(s, r)]
    for x, e in zip(out, o_eval(o, es, er)):
        assert np.array_equal(x[idx], e)
    for x, y in zip(out, (host(t) for t in dp.eval(s, r, variant=2))):
        assert np.array_equal(x, y)
    hcv, scv, feas, pen = out
    assert np.array_equal(feas.astype(bool), hcv == 0)
    assert np.array_equal(pen, np.where(feas != 0, scv, 1000000 + hcv))
    assert feas.any() and not feas.all()
    assert dp.status() == 0


# ---------------------------------------------------------------- configs[4]
def test_syn_eval_pop262144_sampled(orc):
    """configs[4] at its full size: 262,144 syn individuals (E = 2000, R = 40)
    from RandomInitialSolution on the device, tt_eval (wide path) on the whole
    population; every 512th individual (512) against the oracle (slots, rooms,
    RNG, hcv, scv, feasible, penalty); whole population: a second launch is
    identical, outputs consistent (penalty formula, scv >= 0)."""
    inst = ttga.config_instance("syn")
    dp = native.DeviceProblem(inst)
    assert dp.eval_variant() == 13
    o = orc.problem(inst)
    P, stride = 262144, 512
    seeds = ttga.population_seeds(262144, P)
    g = dev(seeds)
    s = torch.empty((P, inst.E), dtype=torch.uint8, device="cuda")
    r = torch.empty_like(s)
    dp.random_init(g, s, r)
    out = [host(t) for t in dp.eval(s, r)]
    again = [host(t) for t in dp.eval(s, r)]
    for x, y in zip(out, again):
        assert np.array_equal(x, y)
    idx = np.arange(0, P, stride)
    hs, hr = host(s[::stride]), host(r[::stride])
    es, er, eg = split_rows(o.random_init, (seeds[idx],))
    assert np.array_equal(hs, es) and np.array_equal(hr, er) and np.array_equal(host(g)[idx], eg)
    for x, e in zip(out, o_eval(o, es, er)):
        assert np.array_equal(x[idx], e)
    hcv, scv, feas, pen = out
    assert (scv >= 0).all() and (hcv >= 0).all()
    assert np.array_equal(pen, np.where(feas != 0, scv, 1000000 + hcv))
    assert dp.status() == 0
