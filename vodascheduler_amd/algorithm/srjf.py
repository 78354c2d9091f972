"""SRJF and Elastic-SRJF (reference pkg/algorithm/srjf.go:25-52, elastic_srjf.go:25-72).

Order: estimated remaining time ascending (needs job info).
"""
from __future__ import annotations

from ..common.trainingjob import TrainingJob
from .base import SchedulerAlgorithm, info_of
from .fifo import elastic_phase2


def by_remaining_time(jobs: list[TrainingJob]) -> list[TrainingJob]:
    return sorted(jobs, key=lambda j: info_of(j).estimate_remainning_time_seconds)


class SRJF(SchedulerAlgorithm):
    name = "SRJF"
    need_job_info = True

    def _schedule(self, jobs, total_gpu):
        free = total_gpu
        res: dict[str, int] = {}
        for j in by_remaining_time(jobs):
            res[j.name] = 0
            if free >= j.config.min_num_proc:
                res[j.name] = j.config.min_num_proc
                free -= j.config.min_num_proc
        return res


class ElasticSRJF(SchedulerAlgorithm):
    """Phase 1 marks ``Min == Max`` jobs satisfied (the reference forgets to, so phase 2
    pushes them past ``Max``: SURVEY.md §2.10 #2); phase 2 as Elastic-FIFO."""

    name = "ElasticSRJF"
    need_job_info = True

    def _schedule(self, jobs, total_gpu):
        free = total_gpu
        res: dict[str, int] = {}
        sat: dict[str, bool] = {}
        order = by_remaining_time(jobs)
        for j in order:
            res[j.name] = 0
            sat[j.name] = False
            if free >= j.config.min_num_proc:
                res[j.name] = j.config.min_num_proc
                free -= j.config.min_num_proc
                if res[j.name] == j.config.max_num_proc:
                    sat[j.name] = True
            else:
                sat[j.name] = True
        elastic_phase2(order, res, sat, free)
        return res
