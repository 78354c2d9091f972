"""Scheduler REST API on :55588 (reference scheduler.go:256-261,1127-1183; doc/apis.md).

``GET /training`` status table, ``PUT /algorithm`` (JSON string), ``PUT /ratelimit`` (JSON
int seconds), ``GET /metrics``; plus ``GET /trace``: the scheduler timeline as Chrome-trace
JSON (utils/tracing.py; no reference counterpart).  Every call is executed on the scheduler
thread.
"""
from __future__ import annotations

import json

from ..algorithm import ALGORITHMS
from ..common.types import ENTRY_POINT
from ..utils.http import Router, text
from .runner import SchedulerRunner


def scheduler_router(runner: SchedulerRunner, tracer=None) -> Router:
    core = runner.core
    r = Router()

    def get_jobs(_b, _q):
        return text(200, runner.call(core.get_all_training_jobs))

    def put_algorithm(body, _q):
        try:
            name = json.loads(body)
        except json.JSONDecodeError as e:
            return text(400, f"{e}\n")
        if not isinstance(name, str) or name not in ALGORITHMS:
            return text(400, f"unknown algorithm {name!r}; known: {sorted(ALGORITHMS)}\n")
        runner.call(core.set_algorithm, name)
        runner.call(core.trigger_resched)
        return text(200, f"Scheduling algorithm set to: {name}\n")

    def put_ratelimit(body, _q):
        try:
            sec = json.loads(body)
            if isinstance(sec, bool) or not isinstance(sec, (int, float)) or sec < 0:
                raise ValueError("rate limit must be a non-negative number of seconds")
        except (ValueError, json.JSONDecodeError) as e:
            return text(400, f"{e}\n")
        runner.call(core.set_rate_limit, float(sec))
        return text(200, f"Rescheduling rate limit set to: {sec} seconds\n")

    def metrics(_b, _q):
        out = core.metrics.exposition()
        if core.placement is not None:
            out += core.placement.metrics.exposition()
        return 200, "text/plain; version=0.0.4", out

    r.add("GET", ENTRY_POINT, get_jobs)
    r.add("PUT", "/algorithm", put_algorithm)
    r.add("PUT", "/ratelimit", put_ratelimit)
    def trace(_b, _q):
        if tracer is None:
            return text(404, "tracing is not enabled on this scheduler\n")
        return 200, "application/json", runner.call(tracer.to_json).encode()

    r.add("GET", "/metrics", metrics)
    r.add("GET", "/trace", trace)
    return r
