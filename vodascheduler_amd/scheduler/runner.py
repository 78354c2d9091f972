"""Real-time driver of :class:`SchedulerCore`: one loop thread owns all scheduler state.

Replaces the reference's goroutines (``Run`` event loop, ``updateTimeMetrics`` ticker,
``readMsgs`` MQ consumer, informer callbacks; scheduler.go:271-324,757-843) with a single
writer: MQ messages, REST calls and backend events are *submitted* to the loop thread and
executed there, then ``core.poll()`` runs whatever is due.  The loop sleeps on a condition
variable until the next deadline or the next submitted command.
"""
from __future__ import annotations

import logging
import threading
from concurrent.futures import Future
from typing import Any, Callable

from ..common.mq import VERB_CONFIGURE, VERB_CREATE, VERB_DELETE, MessageQueue
from .core import SchedulerCore

log = logging.getLogger("vodascheduler_amd.scheduler")


class SchedulerRunner:
    def __init__(self, core: SchedulerCore, mq: MessageQueue | None = None, queue_name: str | None = None):
        self.core = core
        self.mq = mq
        self.queue_name = queue_name or core.scheduler_id
        self._cv = threading.Condition()
        self._cmds: list[tuple[Callable, tuple, Future]] = []
        self._stop = threading.Event()
        self._threads: list[threading.Thread] = []
        core.backend.set_event_sink(lambda *ev: self.submit(core.handle_backend_event, *ev))

    # ---------------------------------------------------------------- API
    def submit(self, fn: Callable, *args) -> Future:
        fut: Future = Future()
        with self._cv:
            self._cmds.append((fn, args, fut))
            self._cv.notify()
        return fut

    def call(self, fn: Callable, *args, timeout: float = 60.0) -> Any:
        """Run ``fn(*args)`` on the scheduler thread and wait for the result."""
        if threading.current_thread() in self._threads:
            return fn(*args)
        return self.submit(fn, *args).result(timeout=timeout)

    def start(self) -> "SchedulerRunner":
        t = threading.Thread(target=self._loop, name=f"scheduler-{self.core.scheduler_id}", daemon=True)
        self._threads.append(t)
        t.start()
        if self.mq is not None:
            c = threading.Thread(target=self._consume, name="scheduler-mq", daemon=True)
            self._threads.append(c)
            c.start()
        return self

    def stop(self, timeout: float = 10.0) -> None:
        self._stop.set()
        with self._cv:
            self._cv.notify_all()
        for t in self._threads:
            t.join(timeout)

    # ---------------------------------------------------------------- threads
    def _loop(self) -> None:
        while not self._stop.is_set():
            with self._cv:
                cmds, self._cmds = self._cmds, []
            for fn, args, fut in cmds:
                if fut.set_running_or_notify_cancel():
                    try:
                        fut.set_result(fn(*args))
                    except BaseException as e:  # surface to the caller, keep the loop alive
                        log.exception("scheduler command failed")
                        fut.set_exception(e)
            try:
                self.core.poll()
            except Exception:
                log.exception("scheduler poll failed")
            with self._cv:
                if self._cmds or self._stop.is_set():
                    continue
                delay = self.core.next_wakeup() - self.core.clock.now()
                if delay > 0:
                    self._cv.wait(timeout=min(delay, 1.0))

    def _consume(self) -> None:
        assert self.mq is not None
        for msg in self.mq.consume(self.queue_name, self._stop):
            if msg.verb == VERB_CREATE:
                self.submit(self.core.create_training_job, msg.job_name)
            elif msg.verb == VERB_DELETE:
                self.submit(self.core.delete_training_job, msg.job_name)
            elif msg.verb == VERB_CONFIGURE:
                log.info("configure message for %s ignored (not implemented in the reference either)",
                         msg.job_name)
