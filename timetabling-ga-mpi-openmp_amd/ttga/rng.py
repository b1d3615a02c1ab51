"""Park-Miller "minimal standard" generator (Random.h:15-19, Random.cc:27-37).

Schrage's method on a signed 64-bit state, C truncating division, then the
fp64 product ``AM * state`` exactly as the reference computes it.
"""
from __future__ import annotations

import numpy as np

IA, IM, IQ, IR = 16807, 2147483647, 127773, 2836
AM = 1.0 / IM


def _cdiv(a: int, b: int) -> int:
    q = abs(a) // abs(b)
    return q if (a >= 0) == (b >= 0) else -q


def step(s: int) -> int:
    k = _cdiv(s, IQ)
    s = IA * (s - k * IQ) - IR * k
    if s < 0:
        s += IM
    return s


class ParkMiller:
    def __init__(self, seed: int):
        self.seed = int(seed)

    def next(self) -> float:
        self.seed = step(self.seed)
        return AM * self.seed

    def pick(self, n: int) -> int:
        """(int)(next() * n), the reference's index draw (Solution.cpp:52)."""
        return int(self.next() * n)


def island_seed(seed: int, i: int) -> int:
    """Per-rank seed abs(seed + i*(seed/10)) with C int division (ga.cpp:412)."""
    return abs(seed + i * _cdiv(seed, 10))


def population_seeds(base: int, n: int) -> np.ndarray:
    """Random(base + i) per individual (SURVEY 8d population recipe)."""
    return (np.arange(n, dtype=np.int64) + np.int64(base)).astype(np.int64)


def random_slots(seeds: np.ndarray, E: int) -> tuple[np.ndarray, np.ndarray]:
    """slot_e = (int)(next()*45) for e ascending, per individual; vectorised over
    individuals with exact int64/fp64 arithmetic. Returns (slots[P][E] uint8, final states)."""
    s = np.asarray(seeds, dtype=np.int64).copy()
    out = np.empty((s.size, E), dtype=np.uint8)
    for e in range(E):
        k = np.where(s >= 0, s // IQ, -((-s) // IQ))
        s = IA * (s - k * IQ) - IR * k
        s = np.where(s < 0, s + IM, s)
        out[:, e] = (AM * s.astype(np.float64) * 45.0).astype(np.int64)
    return out, s
