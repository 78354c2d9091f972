"""Injectable clocks: wall time for services, virtual time for the simulator and tests."""
from __future__ import annotations

import threading
import time


class Clock:
    def now(self) -> float:
        raise NotImplementedError


class RealClock(Clock):
    def now(self) -> float:
        return time.time()


class ManualClock(Clock):
    """Virtual time advanced explicitly (simulator, state-machine tests)."""

    def __init__(self, t0: float = 0.0):
        self._t = float(t0)
        self._lock = threading.Lock()

    def now(self) -> float:
        with self._lock:
            return self._t

    def advance(self, dt: float) -> float:
        if dt < 0:
            raise ValueError("time cannot go backwards")
        with self._lock:
            self._t += dt
            return self._t

    def set(self, t: float) -> None:
        with self._lock:
            if t < self._t:
                raise ValueError("time cannot go backwards")
            self._t = float(t)
