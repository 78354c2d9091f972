"""Scheduling-algorithm framework (reference pkg/algorithm/types.go:16-47, utils.go:9-42).

``SchedulerAlgorithm.schedule(ready_jobs, total_gpu) -> {job_name: num_gpus}``.  Every
policy validates its result with :func:`validate_result` (the reference panics; we raise
:class:`AllocationError`).  Policies never mutate the caller's job list.
"""
from __future__ import annotations

from abc import ABC, abstractmethod
from typing import Iterable, Sequence

from ..common.trainingjob import JobInfo, TrainingJob, new_base_job_info

ReadyJobs = Sequence[TrainingJob]


class AllocationError(RuntimeError):
    """An allocation violated the min/max/total invariants (``validateResult``)."""


class SchedulerAlgorithm(ABC):
    name: str = ""
    need_job_info: bool = False

    def __init__(self, scheduler_id: str = ""):
        self.scheduler_id = scheduler_id

    @abstractmethod
    def _schedule(self, jobs: list[TrainingJob], total_gpu: int) -> dict[str, int]:
        ...

    def schedule(self, jobs: ReadyJobs, total_gpu: int) -> dict[str, int]:
        if total_gpu < 0:
            raise ValueError("total_gpu must be >= 0")
        jobs = list(jobs)
        names = [j.name for j in jobs]
        if len(set(names)) != len(names):
            raise ValueError("duplicate job names in ready jobs")
        result = self._schedule(list(jobs), total_gpu)
        for j in jobs:
            result.setdefault(j.name, 0)
        validate_result(total_gpu, result, jobs)
        return result

    def get_name(self) -> str:
        return self.name

    def __repr__(self) -> str:
        return f"{type(self).__name__}(scheduler_id={self.scheduler_id!r})"


def info_of(job: TrainingJob) -> JobInfo:
    """Job info, falling back to the linear-speedup base info when the allocator could not
    provide one (the reference dereferences a nil Info here)."""
    if job.info is None:
        return new_base_job_info(job.name, job.job_category, job.gpu_type)
    return job.info


def all_true(d: dict[str, bool]) -> bool:
    return all(d.values())


def validate_result(total_gpu: int, result: dict[str, int], jobs: Iterable[TrainingJob]) -> None:
    """Invariants of every allocation (utils.go:18-42)."""
    mx = {j.name: j.config.max_num_proc for j in jobs}
    mn = {j.name: j.config.min_num_proc for j in jobs}
    used = 0
    for job, n in result.items():
        if job not in mx:
            raise AllocationError(f"allocation for unknown job {job!r}")
        if n < 0:
            raise AllocationError("Invalid GPU allocations: can't be negative")
        if 0 < n < mn[job]:
            raise AllocationError(f"Invalid GPU allocations: less than job min gpu ({job}: {n} < {mn[job]})")
        if n > mx[job]:
            raise AllocationError(f"Invalid GPU allocations: exceeded job max gpu ({job}: {n} > {mx[job]})")
        used += n
    if used > total_gpu:
        raise AllocationError(f"Invalid GPU allocations: exceeded total GPUs ({used} > {total_gpu})")


def by_submit_time(jobs: list[TrainingJob]) -> list[TrainingJob]:
    return sorted(jobs, key=lambda j: j.submit_timestamp)  # Python's sort is stable, like sort.SliceStable
