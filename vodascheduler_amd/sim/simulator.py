"""Discrete-event simulator: the real training service + scheduler + allocator + placement,
driven in virtual time against :class:`SimBackend` ("avg JCT and
makespan on the 32-job trace without GPUs").

    from vodascheduler_amd.sim import simulate, philly_trace
    r = simulate(philly_trace(32), algorithm="ElasticFIFO", gpus=8)
    print(r.avg_jct, r.makespan)
"""
from __future__ import annotations

import json
import statistics
from dataclasses import asdict, dataclass, field

from ..allocator.allocator import ResourceAllocator
from ..backend.sim import SimBackend
from ..common.mq import VERB_CREATE, VERB_DELETE, InProcQueue
from ..common.store import MemoryStore
from ..common.types import DEFAULT_GPU_TYPE, JobStatus
from ..scheduler.core import SchedulerCore
from ..service.service import TrainingService
from ..utils.clock import ManualClock
from .trace import TraceJob


@dataclass
class SimResult:
    algorithm: str
    gpus: int
    n_jobs: int
    avg_jct: float
    median_jct: float
    p95_jct: float
    makespan: float
    avg_wait: float
    utilization: float
    reschedules: int
    resizes: int
    migrations: int
    jct: dict[str, float] = field(default_factory=dict)
    peak_gpus: int = 0          # most GPUs schedulable at any time
    avg_gpus: float = 0.0       # time-averaged schedulable GPUs over [first submission, last completion]

    def summary(self) -> dict:
        d = asdict(self)
        d.pop("jct")
        return d

    def to_json(self) -> str:
        return json.dumps(self.summary())


def simulate(trace: list[TraceJob], algorithm: str = "ElasticFIFO", gpus: int = 8,
             nodes: dict[str, list[int]] | None = None, rate_limit_sec: float = 30.0, tick_sec: float = 5.0,
             resize_overhead_s: float = 5.0, restart_overhead_s: float = 15.0, use_placement: bool = True,
             drain: list[tuple[float, str, int]] | None = None, max_time: float = 1e9,
             gpu_type: str = DEFAULT_GPU_TYPE, trace_path: str | None = None,
             naive_placement: bool = False, info_mode: str = "online",
             collector_period_s: float = 60.0,
             capacity: list[tuple[float, dict[str, list[int]]]] | None = None) -> SimResult:
    """Run a trace to completion.  ``drain`` = [(time, node, gpu)] GPU drain events;
    ``trace_path`` writes the scheduler timeline (Chrome-trace JSON, virtual time);
    ``naive_placement``: best-fit without the Munkres bindings (placement/manager.py);
    ``info_mode``: what the info-driven policies see (backend/sim.py): ``online`` (default:
    submission-time estimates from the declared workload, then the collector every
    ``collector_period_s``, the reference cron's 1 min), ``oracle``, ``prior`` or
    ``placeholder`` (the reference as written: 1 s epochs, linear speedup).
    ``capacity`` = [(time, {node: [gpu, ...]})]: the schedulable inventory from ``time`` on
    -- nodes / GPUs added (a cluster autoscaler, spot capacity returning) or removed; an
    entry at time 0 is the starting inventory.  A drained GPU STAYS drained: every later
    capacity snapshot is applied minus the GPUs drained so far, and at equal times the
    capacity entry is applied first, then the drain.  Utilisation is measured against the
    GPUs present over time; ``gpus`` / ``peak_gpus`` report the most GPUs schedulable at
    once and ``avg_gpus`` the time average."""
    clock = ManualClock(0.0)
    store = MemoryStore()
    mq = InProcQueue(maxsize=10 ** 6)
    svc = TrainingService(store, mq, clock, seed_from_workload=info_mode not in ("placeholder", "mixed"))
    nodes = nodes or {"node0": list(range(gpus))}
    caps = sorted(capacity or [], key=lambda c: c[0])
    start_nodes = nodes
    if caps and caps[0][0] <= 0:
        start_nodes = caps.pop(0)[1]
    backend = SimBackend(clock, start_nodes, store, resize_overhead_s, restart_overhead_s, info_mode=info_mode,
                         collector_period_s=collector_period_s)
    placement = None
    if use_placement and naive_placement:
        from ..placement.manager import PlacementManager

        placement = PlacementManager(gpu_type, naive=True)
    core = SchedulerCore(gpu_type, store, ResourceAllocator(store), backend, placement=placement, clock=clock,
                         algorithm=algorithm, rate_limit_sec=rate_limit_sec, tick_sec=tick_sec,
                         use_placement=use_placement)
    tracer = None
    if trace_path:
        from ..utils.tracing import SchedulerTracer

        tracer = SchedulerTracer(core)
    pending = sorted(trace, key=lambda tj: tj.submit_time)
    drains = sorted(drain or [])
    drained: set[tuple[str, int]] = set()
    names: list[str] = []
    steps = 0
    while True:
        t_arr = pending[0].submit_time if pending else None
        t_drain = drains[0][0] if drains else None
        if caps and (t_drain is None or caps[0][0] < t_drain):
            t_drain = caps[0][0]
        t_done = backend.next_event()
        t_sched = core.next_wakeup()
        active = bool(core.ready_jobs) or bool(pending)
        if not active:
            break
        cands = [t for t in (t_arr, t_drain, t_done) if t is not None]
        # scheduler ticks only matter while something is queued or running
        cands.append(t_sched)
        t = max(clock.now(), min(cands))
        if t > max_time:
            raise RuntimeError("simulation exceeded max_time (livelock?)")
        clock.set(t)
        backend.advance(t)
        while pending and pending[0].submit_time <= t:
            tj = pending.pop(0)
            name = svc.create_training_job(json.dumps(tj.spec), submit_time=tj.submit_time)
            names.append(name)
            doc = store.find_metadata(name)
            backend.on_submit(name, doc["job_category"], doc["spec"], int(doc["config"]["epochs"]))
        while caps and caps[0][0] <= t:
            snap = caps.pop(0)[1]
            backend.set_nodes({n: [g for g in gs if (n, g) not in drained] for n, gs in snap.items()})
        while drains and drains[0][0] <= t:
            _, node, gpu = drains.pop(0)
            drained.add((node, gpu))
            cur = backend.nodes()
            cur[node] = [g for g in cur.get(node, []) if g != gpu]
            backend.set_nodes(cur)
        m = mq.get(gpu_type)
        while m is not None:
            if m.verb == VERB_CREATE:
                core.create_training_job(m.job_name)
            elif m.verb == VERB_DELETE:
                core.delete_training_job(m.job_name)
            m = mq.get(gpu_type)
        core.poll()
        steps += 1
        if steps > 10_000_000:
            raise RuntimeError("simulation did not converge")
    if tracer is not None:
        tracer.save(trace_path)
    jct = {}
    waits = []
    for n in names:
        j = core.done_jobs[n]
        assert j.status == JobStatus.COMPLETED.value, (n, j.status)
        jct[n] = j.finish_timestamp - j.submit_timestamp
        waits.append(j.time_metrics.waiting_time)
    first = min(tj.submit_time for tj in trace)
    last = max(core.done_jobs[n].finish_timestamp for n in names)
    vals = sorted(jct.values())
    peak = backend.max_gpus  # the starting inventory and every later set_nodes
    present = backend.gpu_present_seconds(first, last)
    return SimResult(algorithm=algorithm, gpus=peak, n_jobs=len(names), avg_jct=statistics.fmean(vals),
                     median_jct=statistics.median(vals), p95_jct=vals[min(len(vals) - 1, int(0.95 * len(vals)))],
                     makespan=last - first, avg_wait=statistics.fmean(waits),
                     utilization=backend.gpu_busy_seconds / max(1e-9, present),
                     reschedules=core.resched_count,
                     resizes=backend.total_resizes, migrations=backend.total_migrations, jct=jct,
                     peak_gpus=peak, avg_gpus=present / max(1e-9, last - first))
