"""Tiresias (2-queue discretized LAS) and Elastic-Tiresias.

Reference: pkg/algorithm/tiresias.go:17-119 and elastic_tiresias.go:18-190.  Priority
demotion / promotion runs in the scheduler's time-metrics tick (scheduler.go:786-802 ->
:meth:`vodascheduler_amd.scheduler.core.SchedulerCore.update_time_metrics`).
"""
from __future__ import annotations

import math

from ..common.trainingjob import TrainingJob
from .base import SchedulerAlgorithm, info_of

TIRESIAS_QUEUE_NUM = 2
TIRESIAS_THRESHOLDS_SEC = {0: 3600.0, 1: math.inf}  # tiresias.go:27-30
TIRESIAS_PROMOTE_KNOB = 8                            # tiresias.go:35
ELASTIC_TIRESIAS_COMPACTION_THRESHOLD = 10           # elastic_tiresias.go:21


def demote_priority(p: int) -> int:
    return p + 1 if p < TIRESIAS_QUEUE_NUM - 1 else p


def promote_priority(p: int) -> int:
    return 0


def _queue_of(job: TrainingJob) -> int:
    # out-of-range priorities (e.g. JOB_PRIORITY=5) would be silently dropped by the
    # reference's map-of-queues; clamp them into the last queue instead
    return min(max(int(job.priority), 0), TIRESIAS_QUEUE_NUM - 1)


def tiresias_queues(jobs: list[TrainingJob]) -> list[list[TrainingJob]]:
    qs: list[list[TrainingJob]] = [[] for _ in range(TIRESIAS_QUEUE_NUM)]
    for j in jobs:
        qs[_queue_of(j)].append(j)
    # FirstStartTime order (not submit time) to avoid needless preemption (tiresias.go:62-70)
    return [sorted(q, key=lambda j: j.metrics.first_start_timestamp) for q in qs]


class Tiresias(SchedulerAlgorithm):
    name = "Tiresias"
    need_job_info = False

    def _schedule(self, jobs, total_gpu):
        free = total_gpu
        res: dict[str, int] = {}
        for q in tiresias_queues(jobs):
            for j in q:
                res[j.name] = 0
                if free >= j.config.num_proc:
                    res[j.name] = j.config.num_proc
                    free -= j.config.num_proc
        return res


def _next_gain(job: TrainingJob, workers: int) -> float:
    inf = info_of(job)
    return inf.s(workers + 1) - inf.s(workers)


class ElasticTiresias(SchedulerAlgorithm):
    """Tiresias base allocation (``NumProc``), compaction of priority>=1 jobs to ``Min``
    when more than 10 jobs are pending, then greedy allocation by marginal speedup gain."""

    name = "ElasticTiresias"
    need_job_info = True

    def _schedule(self, jobs, total_gpu):
        free = total_gpu
        pendings = len(jobs)
        res: dict[str, int] = {j.name: 0 for j in jobs}
        gain: dict[str, float] = {}
        for j in jobs:
            mn = j.config.min_num_proc
            gain[j.name] = info_of(j).s(mn) / mn  # elastic_tiresias.go:58
        queues = tiresias_queues(jobs)
        for q in queues:
            for j in q:
                if free >= j.config.num_proc:
                    res[j.name] = j.config.num_proc
                    free -= j.config.num_proc
                    pendings -= 1
                    gain[j.name] = _next_gain(j, res[j.name])
        if pendings > ELASTIC_TIRESIAS_COMPACTION_THRESHOLD:
            for q in queues[1:]:
                for j in q:
                    if res[j.name] != 0:
                        free += res[j.name] - j.config.min_num_proc
                        res[j.name] = j.config.min_num_proc
                        gain[j.name] = _next_gain(j, res[j.name])
        cand = [j for j in jobs if not (res[j.name] >= j.config.max_num_proc or free < j.config.min_num_proc)]
        while free > 0 and cand:
            cand.sort(key=lambda j: _queue_of(j))
            cand.sort(key=lambda j: -gain[j.name])
            j = cand[0]
            if gain[j.name] <= 0:
                break
            if res[j.name] == 0:
                if free >= j.config.min_num_proc:
                    res[j.name] = j.config.min_num_proc
                    free -= j.config.min_num_proc
                    gain[j.name] = _next_gain(j, res[j.name])
                    if res[j.name] >= j.config.max_num_proc:
                        cand.remove(j)
                else:
                    cand.remove(j)
            else:
                res[j.name] += 1
                free -= 1
                gain[j.name] = _next_gain(j, res[j.name])
                if res[j.name] >= j.config.max_num_proc:
                    cand.remove(j)
        return res
