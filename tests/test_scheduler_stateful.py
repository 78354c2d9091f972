"""Hypothesis stateful test of the scheduler core ("hypothesis stateful
tests" for a component the reference left untested and racy).

Random interleavings of job submissions (random min/max/np), clock advances, completions,
failures, deletions, GPU drains / returns and runtime algorithm switches are driven through
the real SchedulerCore + ResourceAllocator + PlacementManager with a recording backend.
After every step the invariants that make the system safe to run hold:

* no GPU is over-subscribed: sum of allocations <= schedulable GPUs, and the backend's
  worker locations are distinct healthy GPUs;
* every running job's allocation respects its [min, max] (validateResult semantics);
* status agrees with allocation (Running <=> > 0 GPUs), done jobs hold nothing;
* the backend's view (running workers per job) equals the scheduler's allocation.
"""
import json

from hypothesis import HealthCheck, settings
from hypothesis import strategies as st
from hypothesis.stateful import RuleBasedStateMachine, invariant, precondition, rule

from vodascheduler_amd.algorithm import ALGORITHMS
from vodascheduler_amd.allocator.allocator import ResourceAllocator
from vodascheduler_amd.backend.base import NullBackend
from vodascheduler_amd.common.mq import InProcQueue
from vodascheduler_amd.common.store import MemoryStore
from vodascheduler_amd.common.types import DEFAULT_GPU_TYPE, JobStatus
from vodascheduler_amd.scheduler.core import SchedulerCore
from vodascheduler_amd.service.service import TrainingService
from vodascheduler_amd.sim import make_spec
from vodascheduler_amd.utils.clock import ManualClock

GPUS = 6


class DrainableBackend(NullBackend):
    def drain(self, gpu: int) -> None:
        self._nodes["node0"] = [g for g in self._nodes["node0"] if g != gpu]

    def restore(self, gpu: int) -> None:
        if gpu not in self._nodes["node0"]:
            self._nodes["node0"] = sorted(self._nodes["node0"] + [gpu])


class SchedulerMachine(RuleBasedStateMachine):
    def __init__(self):
        super().__init__()
        self.clock = ManualClock(1000.0)
        self.store = MemoryStore()
        self.mq = InProcQueue()
        self.svc = TrainingService(self.store, self.mq, self.clock)
        self.backend = DrainableBackend({"node0": list(range(GPUS))})
        self.core = SchedulerCore(DEFAULT_GPU_TYPE, self.store, ResourceAllocator(self.store), self.backend,
                                  clock=self.clock, algorithm="ElasticFIFO", rate_limit_sec=5.0, tick_sec=5.0)
        self.limits: dict[str, tuple[int, int]] = {}
        self.n = 0

    # ------------------------------------------------------------------ rules
    @rule(mn=st.integers(1, 3), extra=st.integers(0, 4), np_extra=st.integers(0, 4), prio=st.sampled_from([None, 0, 1]))
    def submit(self, mn, extra, np_extra, prio):
        mx = mn + extra
        np_ = min(mx, mn + np_extra)
        self.n += 1
        name = self.svc.create_training_job(json.dumps(make_spec(f"j{self.n}", "resnet50", np_, mn, mx, 2, 10,
                                                                 priority=prio)))
        m = self.mq.get(DEFAULT_GPU_TYPE)
        self.core.create_training_job(m.job_name)
        self.limits[name] = (mn, mx)

    @rule(dt=st.floats(0.0, 40.0))
    def advance(self, dt):
        self.clock.advance(dt)
        self.core.poll()

    @precondition(lambda self: any(v > 0 for v in self.core.job_num_gpu.values()))
    @rule(data=st.data(), ok=st.booleans())
    def finish(self, data, ok):
        running = sorted(j for j, v in self.core.job_num_gpu.items() if v > 0)
        job = data.draw(st.sampled_from(running))
        self.backend.running.pop(job, None)  # the backend reports a job whose workers exited
        self.core.handle_job_finished(job, ok)
        self.core.poll()

    @precondition(lambda self: bool(self.core.ready_jobs))
    @rule(data=st.data())
    def delete(self, data):
        self.core.delete_training_job(data.draw(st.sampled_from(sorted(self.core.ready_jobs))))
        self.core.poll()

    @rule(gpu=st.integers(0, GPUS - 1), back=st.booleans())
    def drain_or_restore(self, gpu, back):
        (self.backend.restore if back else self.backend.drain)(gpu)
        self.core.set_nodes(self.backend.nodes())
        self.core.poll()

    @rule(algo=st.sampled_from(sorted(ALGORITHMS)))
    def switch_algorithm(self, algo):
        self.core.set_algorithm(algo)
        self.core.trigger_resched()
        self.core.poll()

    # ------------------------------------------------------------------ invariants
    @invariant()
    def capacity_respected(self):
        healthy = set(self.backend.nodes()["node0"])
        assert sum(self.core.job_num_gpu.values()) <= len(healthy)
        locs = [loc for j, ls in self.backend.running.items() for loc in ls]
        assert len(locs) == len(set(locs)), locs
        # after the reschedule that follows a drain, nobody runs on a drained GPU
        if not self.core._topology_dirty and not self.core._requests:
            assert all(g in healthy for _, g in locs), (locs, healthy)

    @invariant()
    def allocations_within_limits(self):
        for j, n in self.core.job_num_gpu.items():
            mn, mx = self.limits[j]
            assert n == 0 or mn <= n <= mx, (j, n, mn, mx)

    @invariant()
    def status_matches_allocation(self):
        for j, job in self.core.ready_jobs.items():
            n = self.core.job_num_gpu.get(j, 0)
            assert (job.status == JobStatus.RUNNING.value) == (n > 0), (j, job.status, n)
        for j in self.core.done_jobs:
            assert j not in self.core.job_num_gpu and j not in self.core.job_workers

    @invariant()
    def backend_matches_scheduler(self):
        for j, n in self.core.job_num_gpu.items():
            assert len(self.backend.running.get(j, [])) == n, (j, n, self.backend.running.get(j))


TestSchedulerStateful = SchedulerMachine.TestCase
TestSchedulerStateful.settings = settings(max_examples=60, stateful_step_count=40, deadline=None,
                                          suppress_health_check=[HealthCheck.too_slow])
