"""Linear sum assignment restated from scipy's shortest-augmenting-path solver.

TEST INFRASTRUCTURE ONLY (the checker); see oracle/batch_ref.py's header.

The reference's polygon/line scenarios (``simple_formation.py``,
``simple_line.py``: GSMARL.egg-info/SOURCES.txt:24-25; readme.md:89-90) call
``scipy.optimize.linear_sum_assignment`` every step (scipy pinned at 1.7.3,
requirements.txt:101). That solver is scipy's ``rectangular_lsap.cpp``
(Crouse, "On implementing 2D rectangular assignment algorithms", 2016), the
same algorithm in every release 1.4 .. 1.15 (this container ships 1.15.3).
This module restates its published algorithm step for step, including the
two details that decide ties:

* the column scan order of every augmenting-path search is the list
  ``remaining = [n-1, ..., 1, 0]``, from which the chosen column is removed by
  swapping in the list's last element;
* among columns of equal reduced cost the scan keeps the first minimum unless
  a later equal one is unassigned (``row4col == -1``), so the result is the
  LAST unassigned minimum in scan order if there is one, else the FIRST.

All arithmetic is float64 in scipy's operation order
(``r = minVal + C[i][j] - u[i] - v[j]`` evaluated left to right), so with the
same float64 cost matrix the assignment is identical, ties included.
``tests/test_lsa_ref.py`` pins this restatement against scipy itself on
random, integer (tie-heavy) and constant matrices; the HIP kernel
(gsm_ragged_kernels.hip) runs the same recurrence one column per lane.
"""
from __future__ import annotations

import math

import numpy as np


def _augmenting_path(n, cost, u, v, path, row4col, spc, i, SR, SC, remaining):
    """One shortest augmenting path from free row i. Returns (sink, minVal)."""
    min_val = 0.0
    num_remaining = n
    for it in range(n):
        remaining[it] = n - it - 1
    for k in range(n):
        SR[k] = False
        SC[k] = False
        spc[k] = math.inf
    sink = -1
    while sink == -1:
        index = -1
        lowest = math.inf
        SR[i] = True
        for it in range(num_remaining):
            j = remaining[it]
            r = min_val + cost[i][j] - u[i] - v[j]
            if r < spc[j]:
                path[j] = i
                spc[j] = r
            if spc[j] < lowest or (spc[j] == lowest and row4col[j] == -1):
                lowest = spc[j]
                index = it
        min_val = lowest
        if min_val == math.inf:
            raise ValueError("cost matrix is infeasible")
        j = remaining[index]
        if row4col[j] == -1:
            sink = j
        else:
            i = row4col[j]
        SC[j] = True
        num_remaining -= 1
        remaining[index] = remaining[num_remaining]
    return sink, min_val


def linear_sum_assignment(cost):
    """Square float64 cost matrix -> col4row (int64 [n]): row i gets column
    col4row[i], minimising the total cost (scipy's tie-breaking)."""
    c = np.asarray(cost, dtype=np.float64)
    n = c.shape[0]
    if c.ndim != 2 or c.shape[1] != n:
        raise ValueError("square matrices only (the scenarios assign N agents to N slots)")
    if n == 0:
        return np.zeros(0, np.int64)
    if np.isnan(c).any() or (c == -np.inf).any():
        raise ValueError("cost matrix contains NaN or -inf")
    cost_l = c.tolist()          # Python floats are IEEE float64
    u = [0.0] * n
    v = [0.0] * n
    spc = [math.inf] * n
    path = [-1] * n
    col4row = [-1] * n
    row4col = [-1] * n
    SR = [False] * n
    SC = [False] * n
    remaining = [0] * n
    for cur in range(n):
        sink, min_val = _augmenting_path(n, cost_l, u, v, path, row4col, spc, cur, SR, SC, remaining)
        u[cur] += min_val
        for i in range(n):
            if SR[i] and i != cur:
                u[i] += min_val - spc[col4row[i]]
        for j in range(n):
            if SC[j]:
                v[j] -= min_val - spc[j]
        j = sink
        while True:
            i = path[j]
            row4col[j] = i
            col4row[i], j = j, col4row[i]
            if i == cur:
                break
    return np.asarray(col4row, dtype=np.int64)
