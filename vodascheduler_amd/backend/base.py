"""Execution backends: how allocation + placement decisions become running workers.

The reference scheduler drives Kubernetes: create the MPIJob (start), update
``Worker.replicas`` (scale in/out), delete the MPIJob (halt), delete pods (migration) and
learns completion from MPIJob conditions (pkg/scheduler/scheduler/scheduler.go:483-627,
pkg/placement/placement_manager.go:622-633).  Here that surface is the :class:`Backend`
interface with three implementations:

* ``backend.local.LocalBackend`` -- node agent with warm per-GPU worker processes on the
  local MI355X node (the MI355X-native path);
* ``backend.sim.SimBackend`` -- discrete-event cluster model (policy evaluation without GPUs);
* ``backend.k8s.K8sBackend`` -- emits the reference's MPIJob/Pod operations for a real
  Kubernetes + MPI-Operator cluster.
"""
from __future__ import annotations

from abc import ABC, abstractmethod
from dataclasses import dataclass, field
from typing import Callable

from ..common.trainingjob import TrainingJob

Loc = tuple[str, int]

HALT, SCALE_IN, START, SCALE_OUT, MIGRATE = "halt", "scale_in", "start", "scale_out", "migrate"
ACTION_ORDER = (HALT, SCALE_IN, START, SCALE_OUT, MIGRATE)  # reference order (scheduler.go:434-445)


@dataclass
class JobAction:
    kind: str
    job: TrainingJob
    num_workers: int
    workers: list[Loc] | None = None  # full worker list after the change (None: backend picks)
    prev_workers: list[Loc] = field(default_factory=list)


# backend -> scheduler events
EV_FINISHED = "finished"          # (EV_FINISHED, job_name, succeeded: bool)
EV_NODES = "nodes"                # (EV_NODES, {node: [gpu, ...]})
EV_PROGRESS = "progress"          # (EV_PROGRESS, job_name, info dict)  (optional)

EventSink = Callable[..., None]


class Backend(ABC):
    def __init__(self):
        self._sink: EventSink | None = None

    def set_event_sink(self, sink: EventSink) -> None:
        self._sink = sink

    def emit(self, *ev) -> None:
        if self._sink is not None:
            self._sink(*ev)

    @abstractmethod
    def apply(self, actions: list[JobAction]) -> None:
        """Execute actions in order (halts, scale-ins, starts, scale-outs, migrations)."""

    @abstractmethod
    def delete_job(self, job_name: str) -> None:
        """Tear down every worker of a job (user delete)."""

    @abstractmethod
    def nodes(self) -> dict[str, list[int]]:
        """Schedulable GPUs per node."""

    def list_running(self) -> dict[str, list[Loc]]:
        """Worker locations of jobs currently running (for scheduler resume)."""
        return {}

    def shutdown(self) -> None:
        pass


class NullBackend(Backend):
    """Records actions; used by state-machine tests."""

    def __init__(self, nodes: dict[str, list[int]] | None = None):
        super().__init__()
        self._nodes = nodes or {"node0": list(range(8))}
        self.log: list[JobAction] = []
        self.deleted: list[str] = []
        self.running: dict[str, list[Loc]] = {}

    def apply(self, actions):
        for a in actions:
            self.log.append(a)
            if a.kind == HALT:
                self.running.pop(a.job.name, None)
            else:
                self.running[a.job.name] = list(a.workers or [])

    def delete_job(self, job_name):
        self.deleted.append(job_name)
        self.running.pop(job_name, None)

    def nodes(self):
        return {k: list(v) for k, v in self._nodes.items()}

    def list_running(self):
        return {k: list(v) for k, v in self.running.items()}
