"""Scheduler core: one instance per GPU type, a single-writer state machine.

Reference: pkg/scheduler/scheduler/scheduler.go (``Scheduler`` 74-114, ``Run`` 271-324,
``resched`` 326-364, ``compareResults`` 448-480, start/scale/halt 495-589, completion
611-687, node events 689-747, ``updateTimeMetrics`` 757-813, create/delete 845-958,
``GetAllTrainingJob`` 968-998, ``constructStatusOnRestart`` 1009-1072).

Design (MI355X-first, not a translation):
* all state mutations happen through this object on ONE thread (``SchedulerRunner``) or in
  virtual time (``Simulator``) -- no lock-free writes from HTTP handlers (the reference
  races on ``Algorithm`` / rate limit);
* time is injected (``Clock``); ``poll()`` executes whatever is due and ``next_wakeup()``
  says when to call it again, so the same code runs in real time and in simulation;
* rate limiting keeps the reference semantics (requests issued before a reschedule started
  are satisfied by it; at most one reschedule per ``rate_limit`` seconds) but uses request
  sequence numbers, so coalescing is exact in virtual time, and never busy-waits
  (reference ``time.Sleep(2)`` = 2 ns, §2.10 #6);
* placement runs whenever counts changed OR the GPU topology changed (drained GPU), so
  migrations off a drained GPU happen even if no job's GPU count changes.
"""
from __future__ import annotations

import bisect
import logging
import time
from typing import Callable, Protocol

from ..algorithm import (ALGORITHMS, DEFAULT_ALGORITHM, TIRESIAS_PROMOTE_KNOB, TIRESIAS_THRESHOLDS_SEC,
                         demote_priority, promote_priority)
from ..allocator.allocator import AllocationRequest
from ..backend.base import (EV_FINISHED, EV_NODES, HALT, MIGRATE, SCALE_IN, SCALE_OUT, START, Backend, JobAction)
from ..common import mpijob
from ..common.store import JobStore, NotFound
from ..common.trainingjob import TrainingJob
from ..common.types import RESCHED_RATE_LIMIT_SEC, TIME_METRICS_TICK_SEC, JobStatus
from ..placement.manager import PlacementManager
from ..utils.clock import Clock, RealClock
from ..utils.metrics import SchedulerMetrics

log = logging.getLogger("vodascheduler_amd.scheduler")


class Allocator(Protocol):
    def allocate(self, req: AllocationRequest) -> dict[str, int]: ...


class SchedulerCore:
    def __init__(self, scheduler_id: str, store: JobStore, allocator: Allocator, backend: Backend,
                 placement: PlacementManager | None = None, clock: Clock | None = None,
                 algorithm: str = DEFAULT_ALGORITHM, rate_limit_sec: float = RESCHED_RATE_LIMIT_SEC,
                 tick_sec: float = TIME_METRICS_TICK_SEC, resume: bool = False, use_placement: bool = True,
                 work_conserving: bool = True):
        if algorithm not in ALGORITHMS:
            raise KeyError(f"Not found: algorithm {algorithm!r}")
        self.scheduler_id = scheduler_id
        self.store = store
        self.allocator = allocator
        self.backend = backend
        self.clock = clock or RealClock()
        self.algorithm = algorithm
        self.rate_limit_sec = float(rate_limit_sec)
        # Work-conserving rescheduling (documented deviation): a reschedule requested because
        # GPUs were FREED (job completed / failed / deleted), or by an arrival while GPUs sit
        # idle, runs immediately instead of waiting out the rate limit -- the reference
        # rate-limits every trigger (scheduler.go:300-316), which leaves GPUs idle for up to
        # ``rate_limit`` seconds.  Arrivals on a fully allocated cluster and priority changes
        # are still rate-limited, so bursts of submissions still coalesce.
        self.work_conserving = work_conserving
        self._urgent = False
        self.tick_sec = float(tick_sec)
        self.use_placement = use_placement
        self.placement = placement if placement is not None else (
            PlacementManager(scheduler_id) if use_placement else None)

        self.ready_jobs: dict[str, TrainingJob] = {}
        self.done_jobs: dict[str, TrainingJob] = {}
        self.job_num_gpu: dict[str, int] = {}
        self.job_workers: dict[str, list] = {}
        self.nodes: dict[str, list[int]] = {}
        self.total_gpus = 0

        now = self.clock.now()
        self._seq = 0
        self._requests: list[tuple[float, int]] = []  # (due time, seq), sorted
        self.last_resched = float("-inf")
        self.resched_blocked_until = float("-inf")
        self.next_tick = now + self.tick_sec
        self._topology_dirty = True
        self.resched_count = 0
        self.listeners: list[Callable[[str, dict], None]] = []  # event hooks (sim/bench/tracing)

        self.metrics = SchedulerMetrics(
            scheduler_id,
            jobs_ready=lambda: len(self.ready_jobs),
            jobs_waiting=lambda: sum(1 for j in self.ready_jobs.values() if j.status == JobStatus.WAITING),
            jobs_running=lambda: sum(1 for j in self.ready_jobs.values() if j.status == JobStatus.RUNNING),
            gpus=lambda: self.total_gpus,
            gpus_inuse=lambda: sum(self.job_num_gpu.values()))

        backend.set_event_sink(self.handle_backend_event)
        self.set_nodes(backend.nodes(), trigger=False)
        if resume:
            self.construct_status_on_restart()
        self.trigger_resched()

    # ------------------------------------------------------------------ events
    def _emit(self, kind: str, **data) -> None:
        for fn in self.listeners:
            fn(kind, dict(data, t=self.clock.now()))

    def trigger_resched(self, at: float | None = None) -> None:
        self._seq += 1
        due = self.clock.now() if at is None else at
        bisect.insort(self._requests, (due, self._seq))

    def handle_backend_event(self, kind: str, *args) -> None:
        if kind == EV_FINISHED:
            name, ok = args[0], bool(args[1])
            self.handle_job_finished(name, ok)
        elif kind == EV_NODES:
            self.set_nodes(args[0])

    # ------------------------------------------------------------------ timing
    def next_wakeup(self) -> float:
        t = self.next_tick
        if self._requests:
            block = float("-inf") if self._urgent else self.resched_blocked_until
            t = min(t, max(self._requests[0][0], block))
        return t

    def poll(self) -> None:
        """Run everything due at the current clock time."""
        now = self.clock.now()
        while now >= self.next_tick:
            self.next_tick += self.tick_sec
            self.update_time_metrics()
        block = float("-inf") if self._urgent else self.resched_blocked_until
        if self._requests and now >= max(self._requests[0][0], block):
            self._urgent = False
            seq_at_start = self._seq
            self.resched()
            t = self.clock.now()
            self.last_resched = t
            self.resched_blocked_until = t + self.rate_limit_sec
            # every request issued before this reschedule started is satisfied by it;
            # future-dated retries and requests raised meanwhile stay queued
            self._requests = [r for r in self._requests if r[0] > now or r[1] > seq_at_start]

    # ------------------------------------------------------------------ rescheduling
    def make_ready_jobs_list(self) -> list[TrainingJob]:
        return [j.clone() for j in self.ready_jobs.values()]

    def resched(self) -> bool:
        t0 = time.perf_counter()
        self.resched_count += 1
        old = dict(self.job_num_gpu)
        req = AllocationRequest(self.scheduler_id, self.total_gpus, self.algorithm, self.make_ready_jobs_list())
        ta = time.perf_counter()
        try:
            new = self.allocator.allocate(req)
        except Exception as e:  # retry after rate limit + 1 s (scheduler.go:338-346)
            log.error("allocation failed (%s); retrying in %.0fs", e, self.rate_limit_sec + 1)
            self.trigger_resched(at=self.clock.now() + self.rate_limit_sec + 1)
            self.metrics.resched.inc()
            return False
        self.metrics.resched_allocator_duration.observe(time.perf_counter() - ta)
        new = {j: int(new.get(j, 0)) for j in self.ready_jobs}
        self.job_num_gpu = new
        changed = self.apply_scheduler_results(old)
        self.metrics.resched_duration.observe(time.perf_counter() - t0)
        self.metrics.resched.inc()
        self._emit("resched", allocation=dict(new), changed=changed)
        return changed

    def compare_results(self, old: dict[str, int]) -> tuple[list[str], list[str], list[str], list[str]]:
        halts, scale_ins, scale_outs, starts = [], [], [], []
        for job in sorted(set(old) | set(self.job_num_gpu)):
            n_old, n_new = old.get(job, 0), self.job_num_gpu.get(job, 0)
            if n_old > n_new:
                if n_new == 0:
                    st = self.get_job_status(job)
                    if st is not None and st not in (JobStatus.COMPLETED, JobStatus.FAILED):
                        halts.append(job)
                else:
                    scale_ins.append(job)
            elif n_old < n_new:
                (starts if n_old == 0 else scale_outs).append(job)
        return halts, scale_ins, scale_outs, starts

    def apply_scheduler_results(self, old: dict[str, int]) -> bool:
        halts, scale_ins, scale_outs, starts = self.compare_results(old)
        changed = bool(halts or scale_ins or scale_outs or starts)
        workers: dict[str, list] = {}
        plan = None
        if self.placement is not None and (changed or self._topology_dirty):
            plan = self.placement.place({j: n for j, n in self.job_num_gpu.items() if n > 0})
            workers = plan.workers
            self._topology_dirty = False
        actions: list[JobAction] = []
        for j in halts:
            actions.append(JobAction(HALT, self.ready_jobs[j], 0, [], self.job_workers.get(j, [])))
        for kind, jobs in ((SCALE_IN, scale_ins), (START, starts), (SCALE_OUT, scale_outs)):
            for j in jobs:
                actions.append(JobAction(kind, self.ready_jobs[j], self.job_num_gpu[j], workers.get(j),
                                         self.job_workers.get(j, [])))
        touched = set(halts) | set(scale_ins) | set(starts) | set(scale_outs)
        if plan is not None:
            for j, locs in workers.items():
                if j not in touched and j in self.ready_jobs and locs != self.job_workers.get(j):
                    actions.append(JobAction(MIGRATE, self.ready_jobs[j], len(locs), locs,
                                             self.job_workers.get(j, [])))
        if not actions:
            return False
        self.backend.apply(actions)
        now = self.clock.now()
        for a in actions:
            job = a.job
            # close the waiting/running interval at the switch, charged at the allocation the
            # job held DURING it (job_num_gpu already holds the new one)
            self._accumulate(job, now, old.get(job.name, 0))
            if a.kind == HALT:
                job.status = JobStatus.WAITING.value
                job.time_metrics.last_waiting_time = 0.0
                self.job_workers.pop(job.name, None)
            else:
                if a.workers is not None:
                    self.job_workers[job.name] = list(a.workers)
                if a.kind == START:
                    job.status = JobStatus.RUNNING.value
                    job.time_metrics.last_gpu_time = 0.0
                    job.time_metrics.last_running_time = 0.0
                    if job.time_metrics.running_time == 0:
                        job.time_metrics.first_start_timestamp = now
            if job.spec is not None:
                try:
                    mpijob.set_worker_replicas(job.spec, a.num_workers)
                except (KeyError, TypeError):
                    pass
            self._persist(job)
        self._emit("actions", actions=[(a.kind, a.job.name, a.num_workers) for a in actions],
                   migrated=(plan.num_migrated if plan else 0))
        return changed

    # ------------------------------------------------------------------ job lifecycle
    def get_job_status(self, name: str) -> JobStatus | None:
        j = self.ready_jobs.get(name) or self.done_jobs.get(name)
        return JobStatus(j.status) if j is not None else None

    def _persist(self, job: TrainingJob) -> None:
        try:
            self.store.update_metadata(job.name, self.scheduler_id, job.to_dict())
        except NotFound:
            pass

    def create_training_job(self, name: str) -> bool:
        if self.get_job_status(name) is not None:
            log.warning("job %s already exists", name)
            return False
        try:
            doc = self.store.find_metadata(name, self.scheduler_id)
        except NotFound:
            log.error("job %s: metadata not found", name)
            return False
        job = TrainingJob.from_dict(doc)
        if job.spec is not None:
            mpijob.preprocess(job.spec, job.gpu_type)
        job.status = JobStatus.WAITING.value
        job.time_metrics.last_update_timestamp = self.clock.now()
        self._persist(job)
        self.ready_jobs[name] = job
        self.job_num_gpu[name] = 0
        if self.work_conserving and sum(self.job_num_gpu.values()) < self.total_gpus:
            self._urgent = True  # idle GPUs: start the arrival now, nothing has to shrink
        self.trigger_resched()
        self.metrics.jobs_created.inc()
        self._emit("created", job=name)
        return True

    def delete_training_job(self, name: str) -> bool:
        st = self.get_job_status(name)
        if st is None:
            return False
        running = st == JobStatus.RUNNING
        if name in self.ready_jobs:
            del self.ready_jobs[name]
            self.job_num_gpu.pop(name, None)
        else:
            self.done_jobs.pop(name, None)
        self.job_workers.pop(name, None)
        if running or st.done:
            self.backend.delete_job(name)
        if running:
            self._urgent = self._urgent or self.work_conserving
            self.trigger_resched()
        self.metrics.jobs_deleted.inc()
        self._emit("deleted", job=name)
        return True

    def handle_job_finished(self, name: str, succeeded: bool) -> None:
        job = self.ready_jobs.get(name)
        if job is None:
            return  # already done / deleted: first event wins
        self._accumulate(job, self.clock.now())
        job.status = (JobStatus.COMPLETED if succeeded else JobStatus.FAILED).value
        job.finish_timestamp = self.clock.now()
        self._persist(job)
        self.done_jobs[name] = job
        del self.ready_jobs[name]
        self.job_num_gpu.pop(name, None)
        self.job_workers.pop(name, None)
        (self.metrics.jobs_completed if succeeded else self.metrics.jobs_failed).inc()
        self._emit("finished", job=name, succeeded=succeeded)
        self._urgent = self._urgent or self.work_conserving
        self.trigger_resched()

    # ------------------------------------------------------------------ nodes
    def set_nodes(self, nodes: dict[str, list[int]], trigger: bool = True) -> None:
        """Declarative node/GPU inventory (add/update/delete node, GPU drain)."""
        nodes = {k: sorted(v) for k, v in nodes.items()}
        if nodes == self.nodes:
            return
        if self.placement is not None:
            for n in list(self.placement.nodes):
                if n not in nodes:
                    self.placement.delete_node(n)
            for n, g in nodes.items():
                self.placement.update_node(n, g)
        grew = sum(len(v) for v in nodes.values()) > self.total_gpus and bool(self.nodes)
        self.nodes = nodes
        self.total_gpus = sum(len(v) for v in nodes.values())
        self._topology_dirty = True
        # capacity ARRIVED (autoscaler node addition, a drained GPU back): like freed GPUs,
        # idle capacity is used at once instead of after the rate limit (work-conserving)
        if self.work_conserving and grew:
            self._urgent = True
        # a GPU that vanished under a running worker (drain, failure) leaves that job broken:
        # re-place it now instead of after the rate limit (work-conserving mode)
        alive = {(n, g) for n, gs in nodes.items() for g in gs}
        if self.work_conserving and any(tuple(loc) not in alive for locs in self.job_workers.values()
                                        for loc in locs):
            self._urgent = True
        if trigger:
            self.trigger_resched()
        self._emit("nodes", total_gpus=self.total_gpus)

    # ------------------------------------------------------------------ time metrics
    def _accumulate(self, job: TrainingJob, now: float, num_gpu: int | None = None) -> None:
        """Close the interval since the last update; ``num_gpu`` = GPUs held during it
        (default: the current allocation)."""
        m = job.time_metrics
        dt = max(0.0, now - m.last_update_timestamp)
        n = self.job_num_gpu.get(job.name, 0) if num_gpu is None else num_gpu
        if job.status == JobStatus.RUNNING:
            m.running_time += dt
            m.gpu_time += dt * n
            m.total_time += dt
            m.last_running_time += dt
            m.last_gpu_time += dt * n
        elif job.status == JobStatus.WAITING:
            m.waiting_time += dt
            m.total_time += dt
            m.last_waiting_time += dt
        m.last_update_timestamp = now

    def update_time_metrics(self) -> bool:
        now = self.clock.now()
        changed = False
        tiresias = self.algorithm in ("Tiresias", "ElasticTiresias")
        for job in self.ready_jobs.values():
            self._accumulate(job, now)
            if tiresias and job.status in (JobStatus.RUNNING, JobStatus.WAITING):
                m = job.time_metrics
                thr = TIRESIAS_THRESHOLDS_SEC.get(job.priority, float("inf"))
                if m.last_gpu_time > thr:
                    np_ = demote_priority(job.priority)
                    if np_ != job.priority:
                        job.priority = np_
                        changed = True
                elif m.last_waiting_time >= m.last_running_time * TIRESIAS_PROMOTE_KNOB and job.priority > 0:
                    job.priority = promote_priority(job.priority)
                    changed = True
        if changed:
            self.trigger_resched()
        return changed

    # ------------------------------------------------------------------ config
    def set_algorithm(self, name: str) -> None:
        if name not in ALGORITHMS:
            raise KeyError(f"Not found: algorithm {name!r}")
        self.algorithm = name

    def set_rate_limit(self, seconds: float) -> None:
        if seconds < 0:
            raise ValueError("rate limit must be >= 0")
        self.rate_limit_sec = float(seconds)
        self.resched_blocked_until = self.last_resched + self.rate_limit_sec

    # ------------------------------------------------------------------ status
    def get_all_training_jobs(self) -> str:
        """The reference's fixed-width status table (scheduler.go:968-998)."""
        fmt = "%-60s %-10s %-10s %-25s %-10s %-10s %-10s\n"
        row_fmt = "%-60s %-10s %-10d %-25s %-10s %-10s %-10s\n"
        out = fmt % ("NAME", "STATUS", "WORKERS", "SCHEDULER", "WAITING", "RUNNING", "TOTAL")
        rows = []
        for job in list(self.ready_jobs.values()) + list(self.done_jobs.values()):
            m = job.time_metrics
            rows.append(row_fmt % (
                job.name, job.status, self.job_num_gpu.get(job.name, 0), self.scheduler_id,
                f"{round(m.waiting_time)}s", f"{round(m.running_time)}s", f"{round(m.total_time)}s"))
        return out + "".join(sorted(rows))

    # ------------------------------------------------------------------ resume
    def construct_status_on_restart(self) -> None:
        running = self.backend.list_running()
        for doc in self.store.list_metadata(self.scheduler_id):
            job = TrainingJob.from_dict(doc)
            st = JobStatus(job.status)
            if st in (JobStatus.WAITING, JobStatus.RUNNING):
                self.ready_jobs[job.name] = job
                locs = running.get(job.name, [])
                self.job_num_gpu[job.name] = len(locs)
                if locs:
                    job.status = JobStatus.RUNNING.value
                    self.job_workers[job.name] = list(locs)
                else:
                    job.status = JobStatus.WAITING.value
            elif st.done:
                self.done_jobs[job.name] = job
        if self.placement is not None:
            self.placement.construct_status_on_restart({j: v for j, v in self.job_workers.items()})
        for job in self.ready_jobs.values():
            job.time_metrics.last_update_timestamp = self.clock.now()
