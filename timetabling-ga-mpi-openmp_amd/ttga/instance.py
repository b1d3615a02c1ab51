"""Problem instances: the .tim format of the reference and a seeded generator.

`.tim` token order follows Problem::Problem(istream&) (Problem.cpp:3-84):
``E R F S``, R room sizes, the S x E attendance matrix (student-major), the
R x F room-feature matrix, the E x F event-feature matrix; whitespace separated.

The real small01/medium01/large01 and ITC-2002 comp01-20 files are not
available offline, so the generator builds seeded synthetic instances with the
same (E, R, F, S): each student attends U[5, 20] distinct events,
room features / event requirements are Bernoulli, and rooms are repaired so
every event has at least one possible room. All draws come from the
reference's own Park-Miller generator, so the C++ driver can reproduce them.
"""
from __future__ import annotations

import dataclasses
import pathlib

import numpy as np

from .rng import ParkMiller

# Named configurations of BASELINE.json (E, R, F, S), generator seeds fixed.
CONFIGS = {
    "sm": (100, 5, 5, 80),       # small01-like
    "med": (400, 10, 5, 200),    # medium01-like (headline instance size)
    "lg": (400, 10, 10, 400),    # large01-like
    "syn": (2000, 40, 10, 5000), # synthetic scaling instance
}


@dataclasses.dataclass
class Instance:
    """Parsed .tim matrices (Problem.h:35-44), int32 numpy arrays."""

    E: int
    R: int
    F: int
    S: int
    room_size: np.ndarray        # [R]
    student_events: np.ndarray   # [S, E] 0/1
    room_features: np.ndarray    # [R, F] 0/1
    event_features: np.ndarray   # [E, F] 0/1

    def __post_init__(self):
        self.room_size = np.ascontiguousarray(self.room_size, dtype=np.int32).reshape(self.R)
        self.student_events = np.ascontiguousarray(self.student_events, dtype=np.int32).reshape(self.S, self.E)
        self.room_features = np.ascontiguousarray(self.room_features, dtype=np.int32).reshape(self.R, self.F)
        self.event_features = np.ascontiguousarray(self.event_features, dtype=np.int32).reshape(self.E, self.F)

    # -- derived data, Problem.cpp:33-95 (numpy restatement, used by tests and the CLI)
    def student_number(self) -> np.ndarray:
        return self.student_events.sum(axis=0).astype(np.int32)

    def correlations(self) -> np.ndarray:
        a = self.student_events.astype(np.int64)
        return ((a.T @ a) > 0).astype(np.int32)

    def possible_rooms(self) -> np.ndarray:
        sn = self.student_number()
        size_ok = self.room_size[None, :] >= sn[:, None]
        missing = (self.event_features[:, None, :] == 1) & (self.room_features[None, :, :] == 0)
        return (size_ok & ~missing.any(axis=2)).astype(np.int32)

    def to_tim(self) -> str:
        parts = [f"{self.E} {self.R} {self.F} {self.S}"]
        for arr in (self.room_size, self.student_events, self.room_features, self.event_features):
            parts.append("\n".join(map(str, arr.reshape(-1).tolist())))
        return "\n".join(p for p in parts if p) + "\n"


def parse_tim(text: str) -> Instance:
    """Problem::Problem(istream&) token order (Problem.cpp:7-74)."""
    tok = np.array(text.split(), dtype=np.int64)
    if tok.size < 4:
        raise ValueError("truncated .tim header")
    E, R, F, S = (int(x) for x in tok[:4])
    need = 4 + R + S * E + R * F + E * F
    if tok.size < need:
        raise ValueError(f".tim file has {tok.size} tokens, expected {need}")
    o = 4
    room_size = tok[o:o + R]; o += R
    A = tok[o:o + S * E]; o += S * E
    rf = tok[o:o + R * F]; o += R * F
    ef = tok[o:o + E * F]
    return Instance(E, R, F, S, room_size, A, rf, ef)


def read_tim(path) -> Instance:
    return parse_tim(pathlib.Path(path).read_text())


def write_tim(inst: Instance, path) -> None:
    pathlib.Path(path).write_text(inst.to_tim())


def generate(E: int, R: int, F: int, S: int, seed: int = 1, min_att: int = 5, max_att: int = 20,
             p_room_feature: float = 0.5, p_event_feature: float = 0.2, size_lo: float = 0.4,
             size_span: float = 0.8, repair: bool = True) -> Instance:
    """Seeded synthetic instance with the given dimensions."""
    rng = ParkMiller(seed)
    A = np.zeros((S, E), dtype=np.int32)
    span = max_att - min_att + 1
    for s in range(S):
        k = min(E, min_att + int(rng.next() * span))
        row = A[s]
        c = 0
        while c < k:
            e = int(rng.next() * E)
            if row[e] == 0:
                row[e] = 1
                c += 1
    sn = A.sum(axis=0)
    rf = np.array([[1 if rng.next() < p_room_feature else 0 for _ in range(F)] for _ in range(R)],
                  dtype=np.int32).reshape(R, F)
    ef = np.array([[1 if rng.next() < p_event_feature else 0 for _ in range(F)] for _ in range(E)],
                  dtype=np.int32).reshape(E, F)
    top = max(int(sn.max()) if E else 1, 1)
    sizes = np.array([max(1, int(top * (size_lo + size_span * rng.next()))) for _ in range(R)], dtype=np.int32)
    for e in range(E if repair else 0):
        ok = (sizes >= sn[e]) & ~((ef[e][None, :] == 1) & (rf == 0)).any(axis=1)
        if not ok.any():
            r = int(rng.next() * R)
            rf[r] |= ef[e]
            sizes[r] = max(sizes[r], sn[e])
    return Instance(E, R, F, S, sizes, A, rf, ef)


def comp_dims(k: int) -> tuple[int, int, int, int]:
    """(E, R, F, S) of the ITC-2002-like instance compK (k = 1..20): E in
    [350, 440], R in {10, 11}, F = 10, S in [200, 350], drawn from
    Park-Miller seeded with 7919 * k."""
    rng = ParkMiller(7919 * int(k))
    E = 350 + int(rng.next() * 91)
    R = 10 + int(rng.next() * 2)
    S = 200 + int(rng.next() * 151)
    return E, R, 10, S


def config_instance(name: str, seed: int = 1) -> Instance:
    """sm / med / lg / syn (CONFIGS) or comp01 .. comp20 (seed k)."""
    if name.startswith("comp"):
        k = int(name[4:])
        if not 1 <= k <= 20:
            raise ValueError("comp instances are comp01 .. comp20")
        return generate(*comp_dims(k), seed=k)
    E, R, F, S = CONFIGS[name]
    return generate(E, R, F, S, seed=seed)
