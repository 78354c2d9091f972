"""AFS-L (Hwang et al., "Elastic Resource Sharing for Distributed Deep Learning", NSDI'21).

Reference: pkg/algorithm/afsl.go:31-106.  GPUs are handed out one at a time to the
"top priority" job, chosen by a pairwise scan: between two waiting jobs the shorter
remaining time wins; otherwise, with ``j`` the job that would finish sooner and ``jb`` the
longer one, ``jb`` wins iff its relative marginal gain beats ``j``'s.
Fixes: a job at 0 GPUs receives its ``Min`` at once (or is skipped
when ``Min`` no longer fits) instead of a single GPU; ``jobLength(jb, ...)`` uses ``jb``'s
own worker count (the reference passes ``j``'s, afsl.go:82).
"""
from __future__ import annotations

import math

from ..common.trainingjob import TrainingJob
from .base import SchedulerAlgorithm, by_submit_time, info_of


def _next(job: TrainingJob, w: int) -> int:
    return job.config.min_num_proc if w == 0 else w + 1


def _div(a: float, b: float) -> float:
    if b == 0:
        return math.inf if a > 0 else (-math.inf if a < 0 else math.nan)
    return a / b


class AFSL(SchedulerAlgorithm):
    name = "AFS-L"
    need_job_info = True

    @staticmethod
    def job_length(job: TrainingJob, workers: int) -> float:
        if workers == 0:
            return math.inf
        inf = info_of(job)
        return _div(inf.estimate_remainning_time_seconds, inf.s(workers))

    @staticmethod
    def evaluate(j: TrainingJob, jb: TrainingJob, res: dict[str, int]) -> bool:
        """True if the longer job ``jb`` should get the next GPU(s) instead of ``j``."""
        sj, sb = info_of(j), info_of(jb)
        wj, wb = res[j.name], res[jb.name]
        nb, nj = _next(jb, wb), _next(j, wj)
        left = _div(sb.s(nb) - sb.s(wb), sb.s(nb))
        right = _div(sj.s(nj) - sj.s(wj), sj.s(wj))
        return left > right  # NaN compares False, like Go

    def top_priority(self, jobs: list[TrainingJob], res: dict[str, int]) -> TrainingJob:
        j = jobs[0]
        for jb in jobs[1:]:
            if res[j.name] == 0 and res[jb.name] == 0:
                if info_of(j).estimate_remainning_time_seconds >= info_of(jb).estimate_remainning_time_seconds:
                    j = jb
            else:
                a, b = j, jb
                if self.job_length(a, res[a.name]) >= self.job_length(b, res[b.name]):
                    a, b = b, a  # a: shorter job, b: longer job
                j = b if self.evaluate(a, b, res) else a
        return j

    def _schedule(self, jobs, total_gpu):
        res = {j.name: 0 for j in jobs}
        free = total_gpu
        cand = by_submit_time(jobs)
        while free > 0 and cand:
            j = self.top_priority(cand, res)
            need = _next(j, res[j.name]) - res[j.name]
            if need > free:
                cand.remove(j)  # cannot start (Min does not fit) / cannot grow further
                continue
            res[j.name] += need
            free -= need
            if res[j.name] >= j.config.max_num_proc:
                cand.remove(j)
        return res
