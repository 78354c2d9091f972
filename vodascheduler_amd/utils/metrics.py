"""Prometheus series with the reference's exact names.

Full names are ``<namespace>_<subsystem>_<name>`` with namespace ``voda_scheduler`` and, for
per-GPU-type components, subsystem = GPU type with ``-`` -> ``_`` (reference
pkg/scheduler/scheduler/metrics.go:29-126, pkg/placement/metrics.go:18-50,
pkg/allocator/allocator/metrics.go:24-80, pkg/service/service/metrics.go:21-69,
doc/prometheus-metrics-exposed.md).  Each component owns a private CollectorRegistry so
several instances can live in one process (tests, simulator).
"""
from __future__ import annotations

from typing import Callable

from prometheus_client import CollectorRegistry, Counter, Gauge, Summary, generate_latest

from ..common.types import NAMESPACE, VERSION

NS = NAMESPACE.replace("-", "_")


def subsystem_of(gpu_type: str) -> str:
    return gpu_type.replace("-", "_")


class _Base:
    def __init__(self):
        self.registry = CollectorRegistry()

    def exposition(self) -> bytes:
        return generate_latest(self.registry)


class SchedulerMetrics(_Base):
    def __init__(self, scheduler_id: str, jobs_ready: Callable[[], float], jobs_waiting: Callable[[], float],
                 jobs_running: Callable[[], float], gpus: Callable[[], float], gpus_inuse: Callable[[], float]):
        super().__init__()
        sub, r = subsystem_of(scheduler_id), self.registry
        kw = dict(namespace=NS, subsystem=sub, registry=r)
        self.info = Gauge("scheduler_info", "Information about the scheduler.",
                          ["version", "namespace", "scheduler"], **kw)
        self.info.labels(VERSION, NAMESPACE, scheduler_id).set(1)
        # prometheus_client appends "_total" to counters itself
        self.jobs_created = Counter("scheduler_jobs_created", "Counts number of training jobs created.", **kw)
        self.jobs_deleted = Counter("scheduler_jobs_deleted", "Counts number of training jobs deleted.", **kw)
        self.jobs_completed = Counter("scheduler_jobs_completed", "Counts number of training jobs completed.", **kw)
        self.jobs_failed = Counter("scheduler_jobs_failed", "Counts number of training jobs failed.", **kw)
        self.resched = Counter("scheduler_resched", "Counts number of rescheduling.", **kw)
        self.resched_duration = Summary("scheduler_resched_duration_seconds",
                                        "A summary of the duration of rescheduling.", **kw)
        self.resched_allocator_duration = Summary(
            "scheduler_resched_allocator_duration_seconds",
            "A summary of the duration of getting scheduling result from resource allocator.", **kw)
        for name, helptext, fn in (("scheduler_jobs_ready", "Number of ready jobs.", jobs_ready),
                                   ("scheduler_jobs_waiting", "Number of waiting jobs.", jobs_waiting),
                                   ("scheduler_jobs_running", "Number of running jobs.", jobs_running),
                                   ("scheduler_gpus", "Number of schedulable GPUs.", gpus),
                                   ("scheduler_gpus_inuse", "Number of GPUs in use.", gpus_inuse)):
            Gauge(name, helptext, **kw).set_function(fn)


class PlacementMetrics(_Base):
    def __init__(self, scheduler_id: str):
        super().__init__()
        kw = dict(namespace=NS, subsystem=subsystem_of(scheduler_id), registry=self.registry)
        self.algo_duration = Summary("scheduler_placement_algorithm_duration_seconds",
                                     "A summary of the duration of placement algorithm.", **kw)
        self.workers_migrated = Gauge("scheduler_placement_workers_migrated",
                                      "Number of deleted worker pods for migration in last rescheduling.", **kw)
        self.launchers_deleted = Gauge("scheduler_placement_launchers_deleted",
                                       "Number of deleted launcher pods in last rescheduling.", **kw)
        self.jobs_cross_node = Gauge("scheduler_placement_jobs_cross_node",
                                     "Number of job that need cross-node communication.", **kw)


class AllocatorMetrics(_Base):
    def __init__(self):
        super().__init__()
        kw = dict(namespace=NS, registry=self.registry)
        self.info = Gauge("resource_allocator_info", "Information about the resource allocator.",
                          ["version", "namespace"], **kw)
        self.info.labels(VERSION, NAMESPACE).set(1)
        self.db_duration = Summary("resource_allocator_database_duration_seconds",
                                   "A summary of the duration of accessing database.", **kw)
        self.num_ready_jobs = Summary("resource_allocator_num_ready_jobs",
                                      "A summary of the number of ready jobs.", **kw)
        self.num_gpus = Summary("resource_allocator_num_gpus", "A summary of the number of GPUs.", **kw)
        self.algo_duration = Summary("resource_allocator_scheduling_algorithm_duration_seconds",
                                     "A summary of the duration of scheduling algorithm.", **kw)
        self.num_ready_jobs_l = Summary("resource_allocator_labeled_num_ready_jobs",
                                        "A summary of the number of ready jobs labeled by algorithm.",
                                        ["algorithm"], **kw)
        self.num_gpus_l = Summary("resource_allocator_labeled_num_gpus",
                                  "A summary of the number of GPUs labeled by algorithm.", ["algorithm"], **kw)
        self.algo_duration_l = Summary("resource_allocator_labeled_scheduling_algorithm_duration_seconds",
                                       "A summary of the duration of scheduling algorithm labeled by algorithm.",
                                       ["algorithm"], **kw)


class ServiceMetrics(_Base):
    def __init__(self):
        super().__init__()
        kw = dict(namespace=NS, registry=self.registry)
        self.info = Gauge("training_service_info", "Information about the training service.",
                          ["version", "namespace"], **kw)
        self.info.labels(VERSION, NAMESPACE).set(1)
        self.jobs_created = Counter("training_service_jobs_created", "Counts number of training jobs created.",
                                    **kw)
        self.jobs_deleted = Counter("training_service_jobs_deleted", "Counts number of training jobs deleted.",
                                    **kw)
        self.create_duration = Summary("training_service_create_job_duration_seconds",
                                       "A summary of the duration of creating training job.", **kw)
        self.create_success_duration = Summary("training_service_create_job_success_duration_seconds",
                                               "A summary of the duration of successfully creating training job.",
                                               **kw)
        self.delete_duration = Summary("training_service_delete_job_duration_seconds",
                                       "A summary of the duration of deleting training job.", **kw)
        self.delete_success_duration = Summary("training_service_delete_job_success_duration_seconds",
                                               "A summary of the duration of successfully deleting training job.",
                                               **kw)
