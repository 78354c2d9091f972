"""FIFO and Elastic-FIFO (reference pkg/algorithm/fifo.go:25-52, elastic_fifo.go:25-75)."""
from __future__ import annotations

from ..common.trainingjob import TrainingJob
from .base import SchedulerAlgorithm, all_true, by_submit_time


class FIFO(SchedulerAlgorithm):
    """Non-elastic: submit order, each job gets ``MinNumProc`` if it fits (fifo.go:38-45)."""

    name = "FIFO"
    need_job_info = False

    def _schedule(self, jobs: list[TrainingJob], total_gpu: int) -> dict[str, int]:
        free = total_gpu
        res: dict[str, int] = {}
        for j in by_submit_time(jobs):
            res[j.name] = 0
            if free >= j.config.min_num_proc:
                res[j.name] = j.config.min_num_proc
                free -= j.config.min_num_proc
        return res


def elastic_phase2(order: list[TrainingJob], res: dict[str, int], sat: dict[str, bool], free: int) -> int:
    """Round-robin +1 GPU over unsatisfied jobs in ``order`` until max or out of GPUs.

    The reference tests ``res < Max || !sat`` (elastic_fifo.go:59, elastic_srjf.go:56), which
    hands single GPUs to jobs that could not even get their minimum and then trips
    ``validateResult``.  Intended rule: only jobs that already run
    (``res > 0``) and are below ``Max`` grow.
    """
    while free > 0 and not all_true(sat):
        progressed = False
        for j in order:
            if not sat[j.name] and 0 < res[j.name] < j.config.max_num_proc:
                res[j.name] += 1
                free -= 1
                progressed = True
                if res[j.name] >= j.config.max_num_proc:
                    sat[j.name] = True
                if free == 0:
                    break
        if not progressed:
            break
    return free


class ElasticFIFO(SchedulerAlgorithm):
    """Default policy. Phase 1: ``Min`` in submit order; phase 2: round-robin +1 up to ``Max``."""

    name = "ElasticFIFO"
    need_job_info = False

    def _schedule(self, jobs: list[TrainingJob], total_gpu: int) -> dict[str, int]:
        free = total_gpu
        res: dict[str, int] = {}
        sat: dict[str, bool] = {}
        order = by_submit_time(jobs)
        for j in order:
            res[j.name] = 0
            sat[j.name] = False
            if free >= j.config.min_num_proc:
                res[j.name] = j.config.min_num_proc
                free -= j.config.min_num_proc
                if res[j.name] == j.config.max_num_proc:
                    sat[j.name] = True
            else:
                sat[j.name] = True  # unable to allocate Min to the job
        elastic_phase2(order, res, sat, free)
        return res
