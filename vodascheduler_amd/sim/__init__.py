"""Discrete-event simulation of the full control plane (policy evaluation without GPUs)."""
from .simulator import SimResult, simulate
from .trace import PROFILES, ModelProfile, TraceJob, make_spec, philly_trace, scale_trace, workload_of

__all__ = ["SimResult", "simulate", "PROFILES", "ModelProfile", "TraceJob", "make_spec", "philly_trace",
           "scale_trace", "workload_of"]
