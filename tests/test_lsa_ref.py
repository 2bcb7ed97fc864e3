"""The assignment oracle (oracle/lsa_ref.py) pinned against the reference's
own dependency: scipy.optimize.linear_sum_assignment (requirements.txt:101;
called per step by simple_formation.py / simple_line.py, SOURCES.txt:24-25).

Also checks the lane-parallel formulation the HIP kernel uses
(gsm_ragged_kernels.hip: wave_lsa) — same recurrence, but the sequential
column scan is replaced by (exact min, position-in-`remaining` tie-break) —
so a kernel/oracle mismatch cannot hide behind the tie rule.
"""
import math

import numpy as np
import pytest
from scipy.optimize import linear_sum_assignment as scipy_lsa

from oracle.lsa_ref import linear_sum_assignment


def _matrices(seed, count):
    rng = np.random.default_rng(seed)
    for t in range(count):
        n = int(rng.integers(1, 33))
        kind = t % 5
        if kind == 0:
            c = rng.random((n, n))
        elif kind == 1:
            c = rng.integers(0, 3, (n, n)).astype(np.float64)        # heavy ties
        elif kind == 2:
            c = rng.integers(0, 10, (n, n)).astype(np.float64)
        elif kind == 3:
            c = np.full((n, n), 0.5)                                 # all equal
        else:
            # fp32 distances of agents to polygon slots, some agents stacked
            p = rng.random((n, 2)).astype(np.float32)
            p[: n // 2] = p[0]
            a = np.array([[math.cos(2 * math.pi * j / n), math.sin(2 * math.pi * j / n)]
                          for j in range(n)], dtype=np.float32) * np.float32(0.5)
            d = p[:, None, :] - a[None, :, :]
            c = np.sqrt(d[..., 0] * d[..., 0] + d[..., 1] * d[..., 1]).astype(np.float32).astype(np.float64)
        yield c


def lane_parallel_lsa(cost):
    """The kernel's formulation in NumPy: per step, exact min over the
    remaining columns, then the last unassigned minimum in `remaining` order
    if any, else the first."""
    c = np.asarray(cost, np.float64)
    n = c.shape[0]
    u = np.zeros(n)
    v = np.zeros(n)
    col4row = np.full(n, -1)
    row4col = np.full(n, -1)
    for cur in range(n):
        spc = np.full(n, np.inf)
        path = np.full(n, -1)
        SR = np.zeros(n, bool)
        SC = np.zeros(n, bool)
        rpos = n - 1 - np.arange(n)
        nrem = n
        min_val = 0.0
        i, sink = cur, -1
        while sink < 0:
            SR[i] = True
            rem = ~SC
            r = ((min_val + c[i]) - u[i]) - v
            upd = rem & (r < spc)
            path[upd] = i
            spc[upd] = r[upd]
            m = spc[rem].min()
            cand = rem & (spc == m)
            fre = cand & (row4col == -1)
            if fre.any():
                j = int(np.flatnonzero(fre)[np.argmax(rpos[fre])])
            else:
                j = int(np.flatnonzero(cand)[np.argmin(rpos[cand])])
            min_val = m
            at = rpos[j]
            SC[j] = True
            nrem -= 1
            mv = rem & (np.arange(n) != j) & (rpos == nrem)
            rpos[mv] = at
            if row4col[j] < 0:
                sink = j
            else:
                i = row4col[j]
        spc_c = spc[np.maximum(col4row, 0)]
        for k in range(n):
            if k == cur:
                u[k] += min_val
            elif SR[k]:
                u[k] += min_val - spc_c[k]
        v[SC] -= min_val - spc[SC]
        j = sink
        while True:
            i = path[j]
            row4col[j] = i
            col4row[i], j = j, col4row[i]
            if i == cur:
                break
    return col4row


@pytest.mark.parametrize("seed", [0, 1, 2])
def test_restatement_matches_scipy(seed):
    for c in _matrices(seed, 1500):
        _, col = scipy_lsa(c)
        assert np.array_equal(linear_sum_assignment(c), col), c


def test_lane_parallel_formulation_matches_scipy():
    for c in _matrices(7, 800):
        _, col = scipy_lsa(c)
        assert np.array_equal(lane_parallel_lsa(c), col), c


def test_constant_matrix_gives_identity():
    # scipy fills `remaining` in reverse precisely so this holds (scipy #11602)
    for n in (1, 2, 5, 24, 32):
        assert np.array_equal(linear_sum_assignment(np.ones((n, n))), np.arange(n))


def test_rejects_bad_input():
    with pytest.raises(ValueError):
        linear_sum_assignment(np.array([[np.nan]]))
    with pytest.raises(ValueError):
        linear_sum_assignment(np.zeros((2, 3)))
    assert linear_sum_assignment(np.zeros((0, 0))).shape == (0,)
