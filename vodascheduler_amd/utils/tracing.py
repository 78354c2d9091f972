"""Tracing: roctx ranges for rocprofv3 timelines + an in-process Chrome-trace recorder.

The reference has no tracing at all -- only Prometheus duration summaries
(scheduler.go:330-347, placement_manager.go:311,328,
resource_allocator.go:98-108), which this framework keeps (``utils/metrics.py``).  On top
of them:

* :func:`trace_range` -- a context manager around the phases worth seeing on a GPU
  timeline: training step, communicator bootstrap, state sync, elastic commit.  It pushes a
  **roctx** range (``libroctx64`` via ctypes; rocprofv3 ``--marker-trace`` shows it next to
  the kernels and RCCL calls) when roctx is enabled, and records a Chrome-trace complete
  event when the recorder is on.  Both are off by default and cost one test each.
* :class:`TraceRecorder` -- a bounded, thread-safe buffer of Chrome trace events
  (``chrome://tracing`` / Perfetto JSON).  ``VODA_TRACE=<path>`` turns the process-wide
  recorder on and writes the file at exit (``{pid}`` in the path is replaced);
  ``VODA_ROCTX=1`` turns on roctx ranges.
* :class:`SchedulerTracer` -- subscribes to ``SchedulerCore.listeners`` and renders the
  scheduler's life as a timeline: one lane per job whose slices are the job's GPU
  allocation intervals (labelled with the worker count), reschedule / migration instants,
  and a GPUs-in-use counter track.  Served by the scheduler's ``GET /trace`` endpoint and
  written by the simulator / bench on request.
"""
from __future__ import annotations

import atexit
import ctypes
import json
import os
import threading
import time
from collections import deque
from contextlib import contextmanager
from typing import Any

_PID = os.getpid()


# ------------------------------------------------------------------------------ roctx
class _Roctx:
    """Lazy ctypes binding of roctx (ROCm's NVTX)."""

    def __init__(self) -> None:
        self.enabled = os.environ.get("VODA_ROCTX", "0") == "1"
        self._lib = None
        self._tried = False

    def _load(self):
        if not self._tried:
            self._tried = True
            rocm = os.environ.get("ROCM_PATH", "/opt/rocm")
            for name in ("libroctx64.so", os.path.join(rocm, "lib", "libroctx64.so"),
                         "librocprofiler-sdk-roctx.so", os.path.join(rocm, "lib", "librocprofiler-sdk-roctx.so")):
                try:
                    lib = ctypes.CDLL(name)
                    lib.roctxRangePushA.argtypes = [ctypes.c_char_p]
                    lib.roctxRangePushA.restype = ctypes.c_int
                    lib.roctxRangePop.restype = ctypes.c_int
                    lib.roctxMarkA.argtypes = [ctypes.c_char_p]
                    self._lib = lib
                    break
                except (OSError, AttributeError):
                    continue
        return self._lib

    @property
    def available(self) -> bool:
        return self._load() is not None

    def push(self, name: str) -> None:
        lib = self._load()
        if lib is not None:
            lib.roctxRangePushA(name.encode())

    def pop(self) -> None:
        lib = self._load()
        if lib is not None:
            lib.roctxRangePop()

    def mark(self, name: str) -> None:
        lib = self._load()
        if lib is not None:
            lib.roctxMarkA(name.encode())


ROCTX = _Roctx()


def enable_roctx(on: bool = True) -> bool:
    """Turn roctx ranges on/off; returns whether the library is loadable."""
    ROCTX.enabled = on
    return ROCTX.available if on else False


# ------------------------------------------------------------------------------ recorder
class TraceRecorder:
    """Bounded buffer of Chrome trace events; timestamps in microseconds since ``t0``."""

    def __init__(self, max_events: int = 200_000, clock=time.perf_counter):
        self._ev: deque = deque(maxlen=max_events)
        self._lock = threading.Lock()
        self.clock = clock
        self.t0 = clock()
        self._tids: dict[str, int] = {}
        self._meta: list[dict] = []

    def us(self, t: float) -> float:
        return round((t - self.t0) * 1e6, 3)

    def lane(self, name: str) -> int:
        """Stable thread id for a named lane (a job, a worker, a subsystem)."""
        with self._lock:
            tid = self._tids.get(name)
            if tid is None:
                tid = self._tids[name] = len(self._tids) + 1
                self._meta.append({"ph": "M", "name": "thread_name", "pid": _PID, "tid": tid,
                                   "args": {"name": name}})
            return tid

    def _tid(self, lane: str | None) -> int:
        return self.lane(lane) if lane else self.lane(threading.current_thread().name)

    def add(self, ev: dict) -> None:
        with self._lock:
            self._ev.append(ev)

    def complete(self, name: str, start: float, end: float, cat: str = "voda", lane: str | None = None,
                 args: dict | None = None) -> None:
        self.add({"ph": "X", "name": name, "cat": cat, "pid": _PID, "tid": self._tid(lane), "ts": self.us(start),
                  "dur": round(max(0.0, end - start) * 1e6, 3), "args": args or {}})

    def instant(self, name: str, t: float | None = None, cat: str = "voda", lane: str | None = None,
                args: dict | None = None) -> None:
        self.add({"ph": "i", "s": "t", "name": name, "cat": cat, "pid": _PID, "tid": self._tid(lane),
                  "ts": self.us(self.clock() if t is None else t), "args": args or {}})

    def counter(self, name: str, values: dict[str, float], t: float | None = None) -> None:
        self.add({"ph": "C", "name": name, "pid": _PID, "ts": self.us(self.clock() if t is None else t),
                  "args": values})

    def events(self) -> list[dict]:
        with self._lock:
            return list(self._meta) + list(self._ev)

    def to_json(self) -> str:
        return json.dumps({"traceEvents": self.events(), "displayTimeUnit": "ms"})

    def save(self, path: str) -> str:
        return _write(path, self.to_json())


def _write(path: str, text: str) -> str:
    d = os.path.dirname(path)
    if d:
        os.makedirs(d, exist_ok=True)
    tmp = f"{path}.tmp{os.getpid()}"
    with open(tmp, "w") as f:
        f.write(text)
    os.replace(tmp, path)
    return path


_RECORDER: TraceRecorder | None = None


def recorder() -> TraceRecorder | None:
    return _RECORDER


def start_recording(path: str | None = None, max_events: int = 200_000) -> TraceRecorder:
    """Turn on the process-wide recorder (written to ``path`` at exit when given)."""
    global _RECORDER
    if _RECORDER is None:
        rec = _RECORDER = TraceRecorder(max_events)
        if path:
            atexit.register(rec.save, path)
    return _RECORDER


def stop_recording() -> None:
    global _RECORDER
    _RECORDER = None


if os.environ.get("VODA_TRACE"):
    start_recording(os.environ["VODA_TRACE"].replace("{pid}", str(_PID)))


@contextmanager
def trace_range(name: str, cat: str = "runtime", lane: str | None = None, **args: Any):
    """roctx range + Chrome complete event around the body (no-ops when both are off)."""
    rec = _RECORDER
    rx = ROCTX.enabled
    if rec is None and not rx:
        yield
        return
    if rx:
        ROCTX.push(name)
    t0 = time.perf_counter()
    try:
        yield
    finally:
        if rx:
            ROCTX.pop()
        if rec is not None:
            rec.complete(name, t0, time.perf_counter(), cat, lane, args or None)


def mark(name: str, cat: str = "runtime", **args: Any) -> None:
    if ROCTX.enabled:
        ROCTX.mark(name)
    rec = _RECORDER
    if rec is not None:
        rec.instant(name, cat=cat, args=args or None)


# ------------------------------------------------------------------------------ scheduler
def _label(n: int) -> str:
    return f"{n} GPU" + ("s" if n != 1 else "")


class SchedulerTracer:
    """Timeline of a :class:`~vodascheduler_amd.scheduler.core.SchedulerCore` (real or
    virtual time).  Attach with ``SchedulerTracer(core)``; read with ``to_json()``."""

    def __init__(self, core, max_events: int = 200_000):
        self.core = core
        # the scheduler's own clock (virtual in the simulator) drives the timestamps
        self.rec = TraceRecorder(max_events, clock=core.clock.now)
        self._open: dict[str, tuple[float, int]] = {}   # job -> (start, workers)
        core.listeners.append(self._on_event)

    def _close(self, job: str, t: float) -> None:
        o = self._open.pop(job, None)
        if o is not None:
            self.rec.complete(_label(o[1]), o[0], t, "job", lane=job, args={"workers": o[1]})

    def _gpus(self, t: float) -> None:
        self.rec.counter("gpus_in_use", {"gpus": sum(self.core.job_num_gpu.values())}, t)

    def _on_event(self, kind: str, data: dict) -> None:
        t = data.get("t", self.core.clock.now())
        if kind == "created":
            self.rec.instant("submitted", t, "job", lane=data["job"])
        elif kind == "resched":
            self.rec.instant("resched", t, "scheduler", lane="scheduler",
                             args={"algorithm": self.core.algorithm, "allocation": data.get("allocation", {}),
                                   "changed": data.get("changed")})
        elif kind == "actions":
            for kind_, job, n in data.get("actions", []):
                self._close(job, t)
                if n > 0:
                    self._open[job] = (t, int(n))
                self.rec.instant(kind_, t, "job", lane=job, args={"workers": n})
            if data.get("migrated"):
                self.rec.instant("migration", t, "placement", lane="scheduler",
                                 args={"workers_migrated": data["migrated"]})
            self._gpus(t)
        elif kind in ("finished", "deleted"):
            self._close(data["job"], t)
            name = "deleted" if kind == "deleted" else ("completed" if data.get("succeeded") else "failed")
            self.rec.instant(name, t, "job", lane=data["job"])
            self._gpus(t)
        elif kind == "nodes":
            self.rec.instant("nodes", t, "scheduler", lane="scheduler", args={"total_gpus": data.get("total_gpus")})

    def events(self) -> list[dict]:
        """All events; allocation slices still open are rendered up to "now"."""
        now = self.core.clock.now()
        out = self.rec.events()
        for job, (t0, n) in list(self._open.items()):
            out.append({"ph": "X", "name": _label(n) + " (running)", "cat": "job", "pid": _PID,
                        "tid": self.rec.lane(job), "ts": self.rec.us(t0),
                        "dur": round(max(0.0, now - t0) * 1e6, 3), "args": {"workers": n}})
        return out

    def to_json(self) -> str:
        return json.dumps({"traceEvents": self.events(), "displayTimeUnit": "ms"})

    def save(self, path: str) -> str:
        return _write(path, self.to_json())
