"""LocalBackend: the MI355X-native execution backend for one (or more) nodes.

``PoolBackend`` (runtime/pool.py) turns the scheduler's start / scale / halt / migrate
actions into membership epochs for warm per-GPU workers; this class adds the node agents
that own those worker processes, and the failure path the reference gets from Kubernetes
node informers + Horovod elastic (reference scheduler.go:689-747 ``add/update/deleteNode``,
placement_manager.go:239-304):

* a worker reported dead by its agent is removed from the schedulable inventory
  (``EV_NODES`` -> the scheduler's placement migrates its jobs off that GPU);
* every job that had the dead worker as a member gets an *abort* epoch listing the
  survivors, so their blocked collectives fail fast (the watchdog aborts the RCCL
  communicator), they restore the last commit and continue at the smaller world size;
  if nobody survives, the job's state is declared at rest (last checkpoint on disk);
* a restarted worker that heartbeats again is added back (``EV_NODES``), which triggers a
  reschedule that can grow jobs onto it.
"""
from __future__ import annotations

import logging
import threading

from ..runtime.pool import PoolBackend, worker_id
from ..runtime.rendezvous import JobRendezvous
from .base import EV_NODES

log = logging.getLogger("vodascheduler_amd.local")


class LocalBackend(PoolBackend):
    def __init__(self, store, agents, train_defaults: dict | None = None, poll_interval: float = 0.05,
                 wait_healthy: bool = True):
        locs = [(a.node, w.gpu) for a in agents for w in a.workers.values()]
        super().__init__(store, locs, train_defaults, poll_interval)
        self.agents = list(agents)
        self._health_lock = threading.Lock()
        self.healthy: set[str] = set()
        self.failures: list[dict] = []
        for a in self.agents:
            a.add_listener(self._on_worker_event)
            for w in a.workers.values():
                if w.healthy:
                    self.healthy.add(w.wid)

    # ------------------------------------------------------------------ inventory
    def nodes(self) -> dict[str, list[int]]:
        out: dict[str, list[int]] = {}
        with self._health_lock:
            for n, gpus in self.node_gpus.items():
                out[n] = sorted(g for g in gpus if worker_id((n, g)) in self.healthy)
        return out

    # ------------------------------------------------------------------ failures
    def _on_worker_event(self, event: str, wid: str) -> None:
        if event == "healthy":
            with self._health_lock:
                self.healthy.add(wid)
            self.emit(EV_NODES, self.nodes())
            return
        if event != "dead":
            return
        with self._health_lock:
            self.healthy.discard(wid)
        with self._pub_lock:
            with self._lock:
                affected = {j: list(m) for j, (_, m) in self.live.items() if wid in m}
            for job, mem in affected.items():
                survivors = [m for m in mem if m != wid]
                rdzv = JobRendezvous(self.store, job)
                self.pending.pop(job, None)  # the scheduler re-places the job after EV_NODES
                e = rdzv.publish(survivors, abort=True)
                if not survivors:
                    rdzv.set_live_epoch(-1)  # nobody holds the state: resume from the last checkpoint
                with self._lock:
                    self.live[job] = (e, survivors)
                    self.members[job] = survivors
                self.failures.append({"job": job, "worker": wid, "epoch": e, "survivors": len(survivors)})
                log.warning("worker %s died: job %s continues on %d worker(s) (abort epoch %d)", wid, job,
                            len(survivors), e)
        self.emit(EV_NODES, self.nodes())

    def shutdown(self) -> None:
        super().shutdown()
        for a in self.agents:
            a.shutdown()
