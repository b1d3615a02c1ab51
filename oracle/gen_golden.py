"""Generate the golden vectors under tests/golden/ — TEST INFRASTRUCTURE ONLY.

Every expected output here is produced by the REFERENCE's own code
(oracle/_ref/libttref.so: Problem.cpp, Solution.cpp, Random.cc, Timer.C and
util.cpp from /root/reference compiled unmodified, F1 neutralised by
-ftrivial-auto-var-init=zero, see oracle/Makefile). Inputs are seeded
synthetic instances and populations (real .tim files are unavailable offline).

    make -C oracle && python oracle/gen_golden.py

The fixtures are data only (inputs + reference outputs, compressed npz).
"""
from __future__ import annotations

import pathlib
import sys

import numpy as np

REPO = pathlib.Path(__file__).resolve().parent.parent
sys.path.insert(0, str(REPO / "timetabling-ga-mpi-openmp_amd"))
sys.path.insert(0, str(REPO / "tests"))

import ttga  # noqa: E402
from oracle_lib import ref  # noqa: E402

OUT = REPO / "tests" / "golden"

INSTANCES = {
    "sm": dict(E=100, R=5, F=5, S=80, seed=1),
    "med": dict(E=400, R=10, F=5, S=200, seed=1),
    # rooms too small / too featured on purpose: events without possible rooms,
    # many unmatched events (the lessBusy carry-over path of assignRooms)
    "tight": dict(E=120, R=4, F=3, S=100, seed=7, size_lo=0.5, size_span=0.8, repair=False, p_event_feature=0.3),
}
RNG_SEEDS = [1, 2, 42, 12345, 2147483646, 0, -1, -123456789, 987654321, 16807]


def pm_stream(seed, n, k):
    r = ttga.ParkMiller(seed)
    return np.array([r.pick(k) for _ in range(n)], dtype=np.uint8)


def main():
    R = ref()
    if R is None:
        sys.exit("oracle/_ref/libttref.so not built (needs /root/reference): make -C oracle ref")
    OUT.mkdir(parents=True, exist_ok=True)

    draws, finals = [], []
    for s in RNG_SEEDS:
        d, f = R.rand(s, 64)
        draws.append(d)
        finals.append(f)
    np.savez_compressed(OUT / "rng.npz", seeds=np.array(RNG_SEEDS, np.int64), draws=np.array(draws),
                        finals=np.array(finals, np.int64))

    for name, kw in INSTANCES.items():
        kw = dict(kw)
        E, Rm, F, S = kw.pop("E"), kw.pop("R"), kw.pop("F"), kw.pop("S")
        inst = ttga.generate(E, Rm, F, S, **kw)
        if name == "sm":
            ttga.write_tim(inst, OUT / "sm.tim")
        h = R.problem(inst)
        sn, corr, poss = h.derived()
        data = dict(dims=np.array([E, Rm, F, S], np.int32), room_size=inst.room_size,
                    student_events=inst.student_events.astype(np.uint8),
                    room_features=inst.room_features.astype(np.uint8),
                    event_features=inst.event_features.astype(np.uint8),
                    ref_student_number=sn, ref_corr_bits=np.packbits(corr.astype(np.uint8), axis=1),
                    ref_possible=poss.astype(np.uint8))

        P = 64 if name == "med" else 128
        slots, _ = ttga.random_slots(ttga.population_seeds(12345, P), E)
        rooms = h.assign_rooms(slots)
        rrooms = np.stack([pm_stream(777 + i, E, Rm) for i in range(P)])
        # skewed populations: events crowded into a few slots (large matchings, N > 64)
        k = 3 if name == "med" else 2
        skew = np.stack([pm_stream(99 + i, E, k) * (45 // k) for i in range(8)]).astype(np.uint8)
        skew_rooms = h.assign_rooms(skew)
        # evaluation edge cases: one slot for everything, last slots only
        edge = np.stack([np.zeros(E, np.uint8), np.full(E, 44, np.uint8), np.full(E, 8, np.uint8),
                         (np.arange(E) % 45).astype(np.uint8), (np.arange(E) % 9 * 5 % 45).astype(np.uint8)])
        edge_rooms = np.stack([pm_stream(31 + i, E, Rm) for i in range(edge.shape[0])])
        data.update(slots=slots, rooms=rooms, rand_rooms=rrooms, skew_slots=skew, skew_rooms=skew_rooms,
                    edge_slots=edge, edge_rooms=edge_rooms)
        for tag, (s_, r_) in dict(canon=(slots, rooms), rand=(slots, rrooms), skew=(skew, skew_rooms),
                                  edge=(edge, edge_rooms)).items():
            hcv, scv, feas, pen = h.eval(s_, r_)
            data.update({f"eval_{tag}_hcv": hcv, f"eval_{tag}_scv": scv, f"eval_{tag}_feasible": feas,
                         f"eval_{tag}_penalty": pen})

        # RandomInitialSolution
        nin = 32
        iseeds = ttga.population_seeds(1000, nin)
        islot, iroom, irng = h.random_init(iseeds)
        data.update(init_seeds=iseeds, init_slots=islot, init_rooms=iroom, init_rng=irng)
        # crossover of the two halves of the initial population
        xseeds = ttga.population_seeds(5000, nin // 2)
        xs, xr, xrng = h.crossover(islot[: nin // 2], islot[nin // 2:], xseeds)
        data.update(xover_seeds=xseeds, xover_slots=xs, xover_rooms=xr, xover_rng=xrng)
        # mutation
        mseeds = ttga.population_seeds(7000, nin)
        ms, mr, mrng = h.mutation(islot, iroom, mseeds)
        data.update(mut_seeds=mseeds, mut_slots=ms, mut_rooms=mr, mut_rng=mrng)
        # local search from the initial population (phase 1), then chained (phase 2 once feasible)
        nls = 8 if name == "med" else 16
        steps = 200
        lseeds = ttga.population_seeds(9000, nls)
        ls_s, ls_r, ls_rng = h.local_search(islot[:nls], iroom[:nls], lseeds, steps)
        ls2_s, ls2_r, ls2_rng = h.local_search(ls_s, ls_r, ls_rng, 1000)
        ls3_s, ls3_r, ls3_rng = h.local_search(ls2_s, ls2_r, ls2_rng, 2000)
        data.update(ls_seeds=lseeds, ls_slots=ls_s, ls_rooms=ls_r, ls_rng=ls_rng,
                    ls2_slots=ls2_s, ls2_rooms=ls2_r, ls2_rng=ls2_rng,
                    ls3_slots=ls3_s, ls3_rooms=ls3_r, ls3_rng=ls3_rng)
        # Move3 enabled (prob3 = 1), small budget
        p3s, p3r, p3rng = h.local_search(islot[:4], iroom[:4], ttga.population_seeds(9500, 4), 60, 1.0, 1.0, 1.0)
        data.update(lsp3_slots=p3s, lsp3_rooms=p3r, lsp3_rng=p3rng)
        # evaluation of the LS outputs (some feasible)
        for tag, (s_, r_) in dict(ls3=(ls3_s, ls3_r)).items():
            hcv, scv, feas, pen = h.eval(s_, r_)
            data.update({f"eval_{tag}_hcv": hcv, f"eval_{tag}_scv": scv, f"eval_{tag}_feasible": feas,
                         f"eval_{tag}_penalty": pen})
        np.savez_compressed(OUT / f"{name}.npz", **data)
        f3 = data["eval_ls3_feasible"]
        print(f"{name}: E={E} R={Rm} S={S} ls3 feasible {int(f3.sum())}/{f3.size}, "
              f"unmatched-possible rooms {int((poss.sum(1) == 0).sum())} events without a room")


if __name__ == "__main__":
    main()
