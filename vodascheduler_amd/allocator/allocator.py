"""Resource allocator (reference pkg/allocator/allocator/resource_allocator.go:31-136,
types.go:5-10).

Stateless: takes ``AllocationRequest{SchedulerID, NumGpu, AlgorithmName, ReadyJobs}``,
optionally loads job info from the store, runs the policy, returns ``{job: num_gpus}``.
Fix: job info IS attached to the jobs handed to the policy (the
reference assigns to a loop copy, so every info-driven policy dereferences nil); jobs without
a record fall back to linear speedup.
"""
from __future__ import annotations

import time
from dataclasses import dataclass, field
from typing import Any

from ..algorithm import new_algorithm
from ..common.store import JobStore, NotFound
from ..common.trainingjob import TrainingJob, job_info_from_record, new_base_job_info
from ..utils.metrics import AllocatorMetrics


@dataclass
class AllocationRequest:
    scheduler_id: str
    num_gpu: int
    algorithm_name: str
    ready_jobs: list[TrainingJob] = field(default_factory=list)

    def to_dict(self) -> dict[str, Any]:
        # field names of the reference's JSON (types.go:5-10)
        return {"SchedulerID": self.scheduler_id, "NumGpu": self.num_gpu, "AlgorithmName": self.algorithm_name,
                "ReadyJobs": [j.to_dict() for j in self.ready_jobs]}

    @classmethod
    def from_dict(cls, d: dict[str, Any]) -> "AllocationRequest":
        return cls(scheduler_id=d["SchedulerID"], num_gpu=int(d["NumGpu"]), algorithm_name=d["AlgorithmName"],
                   ready_jobs=[TrainingJob.from_dict(j) for j in d.get("ReadyJobs") or []])


class ResourceAllocator:
    def __init__(self, store: JobStore | None = None, metrics: AllocatorMetrics | None = None):
        self.store = store
        self.metrics = metrics or AllocatorMetrics()

    def get_jobs_info(self, jobs: list[TrainingJob]) -> None:
        """Attach ``JobInfo`` to every job from ``job_info.<category>`` (in place)."""
        t0 = time.perf_counter()
        for j in jobs:
            rec = None
            if self.store is not None:
                try:
                    rec = self.store.find_job_info(j.job_category, j.name)
                except NotFound:
                    rec = None
            j.info = (job_info_from_record(rec, j.job_category, j.gpu_type) if rec is not None
                      else new_base_job_info(j.name, j.job_category, j.gpu_type))
        self.metrics.db_duration.observe(time.perf_counter() - t0)

    def allocate(self, req: AllocationRequest) -> dict[str, int]:
        algo = new_algorithm(req.algorithm_name, req.scheduler_id)
        jobs = [j.clone() for j in req.ready_jobs]
        if algo.need_job_info:
            self.get_jobs_info(jobs)
        t0 = time.perf_counter()
        result = algo.schedule(jobs, req.num_gpu)
        dt = time.perf_counter() - t0
        m = self.metrics
        m.num_ready_jobs.observe(len(jobs))
        m.num_gpus.observe(req.num_gpu)
        m.algo_duration.observe(dt)
        m.num_ready_jobs_l.labels(req.algorithm_name).observe(len(jobs))
        m.num_gpus_l.labels(req.algorithm_name).observe(req.num_gpu)
        m.algo_duration_l.labels(req.algorithm_name).observe(dt)
        return result


class HttpAllocatorClient:
    """Calls a remote allocator's ``POST /allocation`` (scheduler.go:377-430)."""

    def __init__(self, base_url: str, timeout: float = 30.0):
        self.base_url = base_url.rstrip("/")
        self.timeout = timeout

    def allocate(self, req: AllocationRequest) -> dict[str, int]:
        import json
        import urllib.request

        body = json.dumps(req.to_dict()).encode()
        r = urllib.request.Request(self.base_url + "/allocation", data=body, method="POST",
                                   headers={"Content-Type": "application/json"})
        with urllib.request.urlopen(r, timeout=self.timeout) as resp:
            out = json.loads(resp.read())
        if not isinstance(out, dict):
            raise RuntimeError(f"allocator returned {out!r}")
        return {k: int(v) for k, v in out.items()}
