"""Scheduling policies (reference pkg/algorithm) and the factory ``new_algorithm``."""
from __future__ import annotations

from .afsl import AFSL
from .base import AllocationError, SchedulerAlgorithm, validate_result
from .ffdl import FfDLOptimizer
from .fifo import FIFO, ElasticFIFO
from .srjf import SRJF, ElasticSRJF
from .tiresias import (ELASTIC_TIRESIAS_COMPACTION_THRESHOLD, TIRESIAS_PROMOTE_KNOB, TIRESIAS_QUEUE_NUM,
                       TIRESIAS_THRESHOLDS_SEC, ElasticTiresias, Tiresias, demote_priority, promote_priority)

ALGORITHMS: dict[str, type[SchedulerAlgorithm]] = {
    "FIFO": FIFO,
    "ElasticFIFO": ElasticFIFO,
    "SRJF": SRJF,
    "ElasticSRJF": ElasticSRJF,
    "Tiresias": Tiresias,
    "ElasticTiresias": ElasticTiresias,
    "FfDLOptimizer": FfDLOptimizer,
    "AFS-L": AFSL,
}

DEFAULT_ALGORITHM = "ElasticFIFO"


def new_algorithm(name: str, scheduler_id: str = "") -> SchedulerAlgorithm:
    """``NewAlgorithmFactory`` (types.go:26-47); raises KeyError("Not found") for unknown names."""
    try:
        return ALGORITHMS[name](scheduler_id)
    except KeyError:
        raise KeyError(f"Not found: algorithm {name!r}; known: {sorted(ALGORITHMS)}") from None


__all__ = [
    "AFSL", "AllocationError", "SchedulerAlgorithm", "validate_result", "FfDLOptimizer", "FIFO", "ElasticFIFO",
    "SRJF", "ElasticSRJF", "Tiresias", "ElasticTiresias", "ALGORITHMS", "DEFAULT_ALGORITHM", "new_algorithm",
    "TIRESIAS_QUEUE_NUM", "TIRESIAS_THRESHOLDS_SEC", "TIRESIAS_PROMOTE_KNOB", "ELASTIC_TIRESIAS_COMPACTION_THRESHOLD",
    "demote_priority", "promote_priority",
]
