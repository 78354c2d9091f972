"""Node agent: starts, watches and restarts one warm worker process per GPU.

Replaces, on one MI355X node, what the reference gets from Kubernetes: the MPI-Operator
creates ``<job>-worker-<i>`` pods, the kubelet runs them, node informers report GPU
capacity, and Horovod elastic blacklists failed hosts with a 30-100 s cooldown
(reference pkg/scheduler/scheduler/scheduler.go:689-747, placement_manager.go:239-304,
examples/yaml/tensorflow2/*.yaml launcher args ``--blacklist-cooldown-range 30 100``).

Failure detection: a worker is *dead* when its process exited or its
heartbeat (``pool/<wid>/hb``, written every second by a side thread) is older than
``heartbeat_timeout``.  The agent reports the death to its listener (the LocalBackend,
which aborts the affected jobs' communicators and drains the GPU from the scheduler's
inventory), kills what is left of the process, and restarts it after a cooldown that
doubles on repeated failures (bounded by ``max_cooldown``, like Horovod's blacklist
cooldown range).  A restarted worker reports healthy again once it heartbeats.
"""
from __future__ import annotations

import logging
import os
import signal
import subprocess
import sys
import threading
import time
from dataclasses import dataclass, field
from typing import Callable

log = logging.getLogger("vodascheduler_amd.agent")

Listener = Callable[[str, str], None]   # (event, worker id); event in {"healthy", "dead"}


@dataclass
class WorkerProc:
    wid: str
    gpu: int
    proc: subprocess.Popen | None = None
    started: float = 0.0
    healthy: bool = False
    failures: int = 0
    restart_at: float = 0.0
    log_path: str | None = None
    _logf: object = field(default=None, repr=False)


class NodeAgent:
    def __init__(self, node: str, gpus: list[int], store_addr: str, device_type: str = "cuda",
                 python: str = sys.executable, log_dir: str | None = None, heartbeat_timeout: float = 30.0,
                 cooldown: float = 2.0, max_cooldown: float = 100.0, restart: bool = True,
                 backend: str = "auto", extra_env: dict | None = None, store=None, poll: float = 0.2):
        self.node = node
        self.store_addr = store_addr
        self.device_type = device_type
        self.python = python
        self.log_dir = log_dir
        self.heartbeat_timeout = heartbeat_timeout
        self.cooldown = cooldown
        self.max_cooldown = max_cooldown
        self.restart = restart
        self.backend = backend
        self.extra_env = dict(extra_env or {})
        self.store = store
        self.poll = poll
        self.workers = {f"{node}:{g}": WorkerProc(f"{node}:{g}", g) for g in gpus}
        self._listeners: list[Listener] = []
        self._lock = threading.Lock()
        self._stop = threading.Event()
        self._mon: threading.Thread | None = None

    # ---------------------------------------------------------------- API
    def add_listener(self, fn: Listener) -> None:
        self._listeners.append(fn)

    def start(self) -> "NodeAgent":
        for w in self.workers.values():
            self._spawn(w)
        self._mon = threading.Thread(target=self._monitor, daemon=True, name=f"agent-{self.node}")
        self._mon.start()
        return self

    def healthy_gpus(self) -> list[int]:
        with self._lock:
            return sorted(w.gpu for w in self.workers.values() if w.healthy)

    def wait_healthy(self, timeout: float = 300.0, n: int | None = None) -> list[int]:
        want = len(self.workers) if n is None else n
        deadline = time.time() + timeout
        while time.time() < deadline:
            g = self.healthy_gpus()
            if len(g) >= want:
                return g
            if self._stop.wait(0.1):
                break
        raise TimeoutError(f"node {self.node}: {len(self.healthy_gpus())}/{want} workers healthy after {timeout}s")

    def kill_worker(self, wid: str, sig: int = signal.SIGKILL) -> None:
        """Fault injection: kill one worker process (it is detected and restarted)."""
        w = self.workers[wid]
        if w.proc is not None and w.proc.poll() is None:
            w.proc.send_signal(sig)

    def shutdown(self, timeout: float = 20.0) -> None:
        self._stop.set()
        if self._mon is not None:
            self._mon.join(5)
        deadline = time.time() + timeout
        for w in self.workers.values():
            if w.proc is None:
                continue
            while w.proc.poll() is None and time.time() < deadline:
                time.sleep(0.05)
            if w.proc.poll() is None:
                w.proc.kill()
                w.proc.wait(5)
            if w._logf is not None:
                w._logf.close()

    # ---------------------------------------------------------------- internals
    def _cmd(self, w: WorkerProc) -> list[str]:
        dev = f"cuda:{w.gpu}" if self.device_type == "cuda" else "cpu"
        return [self.python, "-m", "vodascheduler_amd.agent.worker", "--store", self.store_addr, "--wid", w.wid,
                "--device", dev, "--backend", self.backend]

    def _spawn(self, w: WorkerProc) -> None:
        env = dict(os.environ)
        env.update(self.extra_env)
        env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
        root = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
        env["PYTHONPATH"] = root + (os.pathsep + env["PYTHONPATH"] if env.get("PYTHONPATH") else "")
        out = subprocess.DEVNULL
        if self.log_dir:
            os.makedirs(self.log_dir, exist_ok=True)
            w.log_path = os.path.join(self.log_dir, f"worker-{w.wid.replace(':', '-')}.log")
            w._logf = open(w.log_path, "ab")
            out = w._logf
        w.proc = subprocess.Popen(self._cmd(w), env=env, stdout=out, stderr=subprocess.STDOUT,
                                  start_new_session=True)
        w.started = time.time()
        w.healthy = False
        log.info("node %s: started worker %s (pid %d)", self.node, w.wid, w.proc.pid)

    def _heartbeat(self, w: WorkerProc) -> float | None:
        if self.store is None:
            return None
        try:
            if not self.store.check([f"pool/{w.wid}/hb"]):
                return None
            return float(self.store.get(f"pool/{w.wid}/hb").decode())
        except Exception:
            return None

    def _notify(self, event: str, wid: str) -> None:
        for fn in self._listeners:
            try:
                fn(event, wid)
            except Exception:
                log.exception("agent listener failed on %s %s", event, wid)

    def _monitor(self) -> None:
        while not self._stop.is_set():
            now = time.time()
            for w in list(self.workers.values()):
                if w.proc is None:
                    if self.restart and now >= w.restart_at and not self._stop.is_set():
                        self._spawn(w)
                    continue
                rc = w.proc.poll()
                hb = self._heartbeat(w)
                stale = (hb is not None and w.healthy and now - hb > self.heartbeat_timeout)
                if rc is None and not stale:
                    if not w.healthy and (self.store is None or (hb is not None and hb >= w.started - 1.0)):
                        with self._lock:
                            w.healthy = True
                        self._notify("healthy", w.wid)
                    continue
                if self._stop.is_set():
                    break
                # dead: exited, or alive but silent
                log.warning("node %s: worker %s %s", self.node, w.wid,
                            f"exited rc={rc}" if rc is not None else "missed heartbeats")
                if rc is None:
                    try:
                        os.killpg(w.proc.pid, signal.SIGKILL)
                    except (ProcessLookupError, PermissionError):
                        w.proc.kill()
                    w.proc.wait(10)
                was_healthy = w.healthy
                with self._lock:
                    w.healthy = False
                    w.failures += 1
                    w.proc = None
                    w.restart_at = now + min(self.max_cooldown, self.cooldown * (2 ** (w.failures - 1)))
                if was_healthy or rc is not None:
                    self._notify("dead", w.wid)
            self._stop.wait(self.poll)
