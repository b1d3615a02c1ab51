"""f1: the Problem's derived data on the device (Problem.cpp:33-58,
76-95). tt_problem_create derives eventCorrelations = (AᵀA > 0) with an int8
MFMA contraction over the students, studentNumber from the diagonal of the same
product and possibleRooms in the same launch (csrc/tt_derive.hip);
tt_problem_derived reads that device image back. Bit-equal to the CPU oracle's
derivation (oracle/ttga_oracle.cpp derive, pinned to the goldens) on every
BASELINE configuration -- sm, med, lg, comp01..comp20, syn -- and on shapes at
the kernel's edges: E and S not multiples of 32/64, no students, a student
attending every event, more than 64 features, 64 rooms, events without
students or possible rooms."""
import numpy as np
import pytest

import ttga
from oracle_lib import oracle

pytestmark = pytest.mark.gpu
torch = pytest.importorskip("torch")
from ttga import native  # noqa: E402

CONFIGS = ["sm", "med", "lg", "syn"] + [f"comp{k:02d}" for k in range(1, 21)]


@pytest.fixture(scope="module")
def orc():
    return oracle()


def check(orc, inst):
    dp = native.DeviceProblem(inst)
    sn, corr, poss = dp.derived()
    osn, ocorr, oposs = orc.problem(inst).derived()
    assert np.array_equal(sn, osn)
    assert np.array_equal(corr, ocorr)
    assert np.array_equal(poss, oposs)
    dp.close()
    return sn, corr, poss


@pytest.mark.parametrize("name", CONFIGS)
def test_derived_configs_vs_oracle(orc, name):
    inst = ttga.config_instance(name)
    sn, corr, _ = check(orc, inst)
    # independent restatement: the dense product, exact in float32 for counts < 2^24
    a = inst.student_events.astype(np.float32)
    c = a.T @ a
    assert np.array_equal(corr, (c > 0).astype(np.int32))
    assert np.array_equal(sn, np.diag(c).astype(np.int32))


@pytest.mark.parametrize("dims", [(1, 1, 0, 1), (31, 3, 2, 17), (33, 4, 1, 65), (65, 7, 3, 63), (127, 9, 70, 129),
                                  (200, 64, 5, 0), (450, 13, 6, 333), (1531, 40, 10, 700)],
                         ids=["E1", "E31S17", "E33S65", "E65S63", "E127F70", "S0R64", "E450", "E1531"])
def test_derived_edge_shapes_vs_oracle(orc, dims):
    E, R, F, S = dims
    inst = ttga.generate(E, R, F, S, seed=E + S, min_att=1, max_att=min(E, 9)) if S else \
        ttga.Instance(E, R, F, S, np.full(R, 5), np.zeros((0, E)), np.zeros((R, F)), np.zeros((E, F)))
    check(orc, inst)


def test_derived_dense_and_empty_events(orc):
    """Student 0 attends every event (every pair correlated, counts up to S);
    the last 70 events have no student (zero rows and columns, zero diagonal);
    a few events require a feature no room has (no possible room)."""
    E, R, F, S = 300, 12, 8, 260
    rng = np.random.default_rng(7)
    A = (rng.random((S, E)) < 0.03).astype(np.int32)
    A[0, :] = 1
    A[:, E - 70:] = 0
    A[1:, 5] = 1                                            # event 5 attended by all
    rf = (rng.random((R, F)) < 0.6).astype(np.int32)
    rf[:, F - 1] = 0
    ef = (rng.random((E, F)) < 0.2).astype(np.int32)
    ef[[3, 77, 150], F - 1] = 1
    inst = ttga.Instance(E, R, F, S, rng.integers(1, S + 2, R), A, rf, ef)
    sn, corr, poss = check(orc, inst)
    assert sn[5] == S and corr[:E - 70, :E - 70].all() and not corr[E - 70:].any()
    assert not poss[[3, 77, 150]].any()
