"""Kuhn-Munkres assignment (native ``_vodacore.linear_assignment``, pure-Python fallback).

The reference calls ``munkres.ComputeMunkresMax`` on a size x size integer score matrix
(pkg/placement/placement_manager.go:492-522).  ``assign_max(scores)`` returns the column
chosen for every row of a square or rectangular matrix, maximising the total score.
"""
from __future__ import annotations

from typing import Sequence

from ..ops import _native


def _py_min_assign(cost: list[list[float]]) -> list[int]:
    """O(n^2 m) Hungarian with potentials (rows <= cols)."""
    n, m = len(cost), len(cost[0]) if cost else 0
    INF = float("inf")
    u, v = [0.0] * (n + 1), [0.0] * (m + 1)
    p, way = [0] * (m + 1), [0] * (m + 1)
    for i in range(1, n + 1):
        p[0] = i
        j0 = 0
        minv = [INF] * (m + 1)
        used = [False] * (m + 1)
        while True:
            used[j0] = True
            i0, delta, j1 = p[j0], INF, -1
            for j in range(1, m + 1):
                if not used[j]:
                    cur = cost[i0 - 1][j - 1] - u[i0] - v[j]
                    if cur < minv[j]:
                        minv[j], way[j] = cur, j0
                    if minv[j] < delta:
                        delta, j1 = minv[j], j
            for j in range(m + 1):
                if used[j]:
                    u[p[j]] += delta
                    v[j] -= delta
                else:
                    minv[j] -= delta
            j0 = j1
            if p[j0] == 0:
                break
        while True:
            j1 = way[j0]
            p[j0] = p[j1]
            j0 = j1
            if j0 == 0:
                break
    ans = [-1] * n
    for j in range(1, m + 1):
        if p[j]:
            ans[p[j] - 1] = j - 1
    return ans


def linear_assignment(scores: Sequence[Sequence[float]], maximize: bool = True) -> list[int]:
    rows = len(scores)
    if rows == 0:
        return []
    cols = len(scores[0])
    flat = [float(x) for r in scores for x in r]
    if len(flat) != rows * cols:
        raise ValueError("ragged score matrix")
    if _native.core_available():
        return list(_native.core().linear_assignment(flat, rows, cols, maximize))
    sgn = -1.0 if maximize else 1.0
    if rows <= cols:
        return _py_min_assign([[sgn * float(x) for x in r] for r in scores])
    t = [[sgn * float(scores[i][j]) for i in range(rows)] for j in range(cols)]
    colrow = _py_min_assign(t)
    ans = [-1] * rows
    for j, i in enumerate(colrow):
        if i >= 0:
            ans[i] = j
    return ans


def assign_max(scores: Sequence[Sequence[float]]) -> list[int]:
    return linear_assignment(scores, maximize=True)
