"""FfDL Optimizer (IBM FfDL dynamic program; reference pkg/algorithm/ffdl_optimizer.go:32-130).

Jobs are FIFO-trimmed to the first ``K = total_gpu`` and a DP over (jobs x GPUs)
maximises the summed speedup:
``P[j][k] = max_{g} speedup_j[g] + P[j-1][k-g]``, ``P[0][*] = 0``, others -10000.
Fixes: ``g`` ranges over ``[Min, Max]`` instead of ``[1, Max]`` (the
reference can hand a job fewer than its minimum); when that makes the trimmed set
infeasible, the DP is re-run allowing ``g = 0`` (job waits) instead of panicking.
The O(J*K*Max) DP runs in the native ``_vodacore`` module when available.
"""
from __future__ import annotations

from ..common.trainingjob import TrainingJob
from .base import SchedulerAlgorithm, by_submit_time, info_of

NEG = -10000.0


def ffdl_dp(speedups: list[list[float]], mins: list[int], maxs: list[int], K: int,
            allow_zero: bool) -> tuple[float, list[int]]:
    """Pure-Python DP.  ``speedups[j][g]`` for g in 0..maxs[j]; returns (best, alloc)."""
    J = len(speedups)
    P = [[0.0] * (K + 1)] + [[NEG] * (K + 1) for _ in range(J)]
    SOL = [[0] * (K + 1) for _ in range(J + 1)]
    for j in range(1, J + 1):
        sp, lo, hi = speedups[j - 1], mins[j - 1], maxs[j - 1]
        for k in range(0, K + 1):
            if allow_zero and P[j - 1][k] > P[j][k]:
                P[j][k] = P[j - 1][k]
                SOL[j][k] = 0
            for g in range(max(lo, 1), hi + 1):
                if k - g < 0:
                    break
                prev = P[j - 1][k - g]
                if prev <= NEG / 2:
                    continue
                p = sp[g] + prev
                if p > P[j][k]:
                    P[j][k] = p
                    SOL[j][k] = g
    # best over k <= K (the reference reads P[J][K]; with P[0][*] = 0 that already
    # includes "leave GPUs idle", identical here)
    best = P[J][K]
    alloc = [0] * J
    k = K
    for j in range(J, 0, -1):
        alloc[j - 1] = SOL[j][k]
        k -= SOL[j][k]
    return best, alloc


def _dp(speedups, mins, maxs, K, allow_zero):
    try:
        from ..ops._native import core

        c = core()
        return c.ffdl_dp(speedups, mins, maxs, K, allow_zero)
    except RuntimeError:
        return ffdl_dp(speedups, mins, maxs, K, allow_zero)


class FfDLOptimizer(SchedulerAlgorithm):
    name = "FfDLOptimizer"
    need_job_info = True

    def _schedule(self, jobs: list[TrainingJob], total_gpu: int) -> dict[str, int]:
        res = {j.name: 0 for j in jobs}
        if not jobs or total_gpu == 0:
            return res
        K = total_gpu
        feasible = by_submit_time(jobs)[:K]
        sps, mins, maxs = [], [], []
        for j in feasible:
            inf = info_of(j)
            hi = min(j.config.max_num_proc, K)
            sps.append([inf.s(g) for g in range(hi + 1)])
            mins.append(j.config.min_num_proc)
            maxs.append(hi)
        best, alloc = _dp(sps, mins, maxs, K, False)
        if best <= 0:
            best, alloc = _dp(sps, mins, maxs, K, True)
        for j, g in zip(feasible, alloc):
            res[j.name] = int(g)
        return res
