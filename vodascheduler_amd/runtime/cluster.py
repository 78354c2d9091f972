"""Run a job trace end-to-end on a pool of real workers: training service -> scheduler
(policy + Munkres placement) -> PoolBackend -> warm per-GPU workers running elastic DP.

Used by ``bench.py`` (GPU pool = torchrun ranks, RCCL over xGMI) and by the CPU/gloo tests
(BASELINE config 1: "Elastic-FIFO, 2 toy MNIST jobs on CPU/gloo, simulated 2-slot cluster").
"""
from __future__ import annotations

import json
import logging
import socket
import statistics
import time

import torch

from ..allocator.allocator import ResourceAllocator
from ..common.mq import InProcQueue
from ..common.store import MemoryStore
from ..common.types import DEFAULT_GPU_TYPE, JobStatus
from ..scheduler.core import SchedulerCore
from ..scheduler.runner import SchedulerRunner
from ..service.service import TrainingService
from ..sim.trace import TraceJob
from .pool import PoolBackend, PoolWorker
from .rendezvous import connect_store

log = logging.getLogger("vodascheduler_amd.cluster")


def free_port() -> int:
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def run_trace(store, trace: list[TraceJob], worker_locs, algorithm: str = "ElasticFIFO",
              rate_limit_sec: float = 1.0, tick_sec: float = 1.0, train_defaults: dict | None = None,
              timeout: float = 3600.0, gpu_type: str = DEFAULT_GPU_TYPE, progress=None,
              collect_every_s: float = 2.0, trace_path: str | None = None,
              gpu_numa: dict[str, dict[int, int]] | None = None, stop_pool: bool = True,
              settle_timeout: float = 120.0, capacity_ramp: list[tuple[float, int]] | None = None) -> dict:
    """Submit ``trace`` in real time (``submit_time`` seconds after start) and wait until every
    job completed.  Returns JCT / makespan / resize-latency statistics.  ``gpu_numa``: node ->
    {GPU: NUMA domain} from topology discovery (placement tie-breaker).  ``stop_pool=False``
    leaves the pool workers serving (another trace follows on the same warm pool).
    ``capacity_ramp`` = [(t, k)]: the scheduler's inventory is the first ``k`` pool GPUs from
    ``t`` seconds on (node additions by an autoscaler; the first entry applies at start).
    On a timeout or error every job still running is deleted (its workers leave at their
    next commit), so the pool is free for whatever follows."""
    db = MemoryStore()
    mq = InProcQueue(maxsize=10 ** 6)
    svc = TrainingService(db, mq)
    ramp = sorted(capacity_ramp or [])

    def inventory(k: int) -> dict[str, list[int]]:
        inv: dict[str, list[int]] = {}
        for n, g in list(worker_locs)[:k]:
            inv.setdefault(n, []).append(g)
        return inv

    initial = inventory(ramp.pop(0)[1]) if ramp and ramp[0][0] <= 0 else None
    backend = PoolBackend(store, worker_locs, train_defaults, settle_timeout=settle_timeout,
                          initial_nodes=initial)
    timeline = [(0.0, sum(len(v) for v in backend.nodes().values()))]
    from ..placement.manager import PlacementManager

    core = SchedulerCore(gpu_type, db, ResourceAllocator(db), backend, algorithm=algorithm,
                         placement=PlacementManager(gpu_type, gpu_numa=gpu_numa),
                         rate_limit_sec=rate_limit_sec, tick_sec=tick_sec)
    tracer = None
    if trace_path:
        from ..utils.tracing import SchedulerTracer

        tracer = SchedulerTracer(core)
    runner = SchedulerRunner(core, mq).start()
    collector = None
    mdir = (train_defaults or {}).get("metrics_dir")
    if mdir:
        from ..collector.collector import MetricsCollector

        collector = MetricsCollector(db, mdir)
    t0 = time.time()
    names: list[str] = []
    pending = sorted(trace, key=lambda tj: tj.submit_time)
    last_report = last_collect = t0
    ok = False
    try:
        while True:
            now = time.time()
            while ramp and now - t0 >= ramp[0][0]:
                _, k = ramp.pop(0)
                backend.set_nodes(inventory(k))
                timeline.append((round(now - t0, 2), k))
                log.info("capacity: %d GPUs at t=%.1fs", k, now - t0)
                if progress is not None:
                    progress(f"t={now - t0:.0f}s capacity -> {k} GPUs")
            if collector is not None and now - last_collect > collect_every_s:
                last_collect = now
                collector.update_info_all(list(names))
            while pending and now - t0 >= pending[0].submit_time:
                tj = pending.pop(0)
                names.append(svc.create_training_job(json.dumps(tj.spec)))
            done = runner.call(lambda: {n: j.status for n, j in core.done_jobs.items()})
            if not pending and names and all(n in done for n in names):
                break
            if now - t0 > timeout:
                raise TimeoutError(f"trace did not finish within {timeout}s ({len(done)}/{len(trace)} done)")
            if progress is not None and now - last_report > 30:
                last_report = now
                progress(f"t={now - t0:.0f}s done={len(done)}/{len(trace)} running="
                         f"{runner.call(lambda: {n: v for n, v in core.job_num_gpu.items() if v})}")
            time.sleep(0.05)
        t1 = time.time()
        jobs = runner.call(lambda: {n: core.done_jobs[n].clone() for n in names})
        ok = True
    finally:
        runner.stop()
        if not ok:  # cut the trace off: running jobs' workers leave at their next commit
            for n in list(backend.active):
                try:
                    backend.delete_job(n)
                except Exception:
                    log.exception("deleting %s after the aborted trace failed", n)
        backend.shutdown(stop_pool)
        if tracer is not None:
            tracer.save(trace_path)
    failed = [n for n, j in jobs.items() if j.status != JobStatus.COMPLETED.value]
    jct = {n: j.finish_timestamp - j.submit_timestamp for n, j in jobs.items()}
    lat = classify_latencies(backend.events, backend.resize_latency)
    vals = sorted(jct.values())
    q = lambda xs, p: xs[min(len(xs) - 1, int(p * len(xs)))] if xs else None  # noqa: E731
    return {
        "n_jobs": len(names), "failed": failed, "avg_jct_s": statistics.fmean(vals), "p50_jct_s": q(vals, 0.5),
        "p95_jct_s": q(vals, 0.95), "makespan_s": max(j.finish_timestamp for j in jobs.values()) - t0,
        "wall_s": t1 - t0, "resize_events": len(backend.events),
        "n_starts": len(lat["start"]), "n_resizes": len(lat["resize"]), "n_shrinks_to_1": len(lat["to_one"]),
        "start_latency_p50_s": q(lat["start"], 0.5), "start_latency_p95_s": q(lat["start"], 0.95),
        "resize_latency_p50_s": q(lat["resize"], 0.5), "resize_latency_p95_s": q(lat["resize"], 0.95),
        "reschedules": core.resched_count, "jct": jct, "forced_abort_epochs": backend.forced_epochs,
        "forced_abort_log": backend.forced_log,
        "events": backend.events, "resize_latency": backend.resize_latency,
        "capacity_timeline": timeline if len(timeline) > 1 else None,
    }


def classify_latencies(events: list[dict], synced: list[dict]) -> dict[str, list[float]]:
    """Split membership-change latencies (request -> new epoch synced and training) into
    * ``start``: the job had no workers (first start, or restart after a halt);
    * ``resize``: a running job moves to a world of >= 2 (scale-in/out or migration): an RCCL
      communicator rebuild (or cache hit) + state broadcast;
    * ``to_one``: a running job shrinks to one worker (no communicator)."""
    by_key = {(e["job"], e["epoch"]): e for e in events}
    out: dict[str, list[float]] = {"start": [], "resize": [], "to_one": []}
    for r in synced:
        e = by_key.get((r["job"], r["epoch"]))
        if e is None:
            continue
        if e["prev_world"] == 0:
            out["start"].append(r["latency_s"])
        elif e["world"] >= 2:
            out["resize"].append(r["latency_s"])
        elif e["world"] == 1:
            out["to_one"].append(r["latency_s"])
    for v in out.values():
        v.sort()
    return out


def cpu_worker_main(host: str, port: int, wid: str, threads: int = 1) -> None:
    """Entry point of a CPU pool worker process (tests / simulated cluster)."""
    torch.set_num_threads(threads)
    store = connect_store(host, port)
    watch = connect_store(host, port)
    PoolWorker(store, watch, wid, torch.device("cpu"), backend="gloo", timeout=120.0).serve()
