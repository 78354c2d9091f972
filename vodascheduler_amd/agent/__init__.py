"""Node agent: warm per-GPU worker processes on one MI355X node (replaces the reference's
MPI-Operator pods + kubelet + ``horovodrun`` host discovery)."""
from .node_agent import NodeAgent, WorkerProc

__all__ = ["NodeAgent", "WorkerProc"]
