"""Training-job data model (reference pkg/common/trainingjob/trainingjob.go:17-187,
pkg/common/mongo/mongo.go:22-95).

Documents keep the reference's bson/json field names so stored records and REST payloads
stay shape-compatible.  Times are float epoch seconds and durations float seconds (the Go
code used time.Time / time.Duration).
"""
from __future__ import annotations

import copy
import time
from dataclasses import asdict, dataclass, field
from typing import Any

from .types import DEFAULT_GPU_TYPE, GPU_NAME_LABEL, MAX_NUM_GPU, MAX_TIME, JobConfigEnv, JobKind, JobStatus


def linear_speedup(max_gpu: int = MAX_NUM_GPU) -> dict[str, float]:
    """Default speedup table {"0": 0, "1": 1, ..., "33": 33} (trainingjob.go:168-187)."""
    sp = {"0": 0.0}
    for i in range(1, max_gpu + 2):
        sp[str(i)] = float(i)
    return sp


def linear_efficiency(max_gpu: int = MAX_NUM_GPU) -> dict[str, float]:
    ef = {"0": 0.0}
    for i in range(1, max_gpu + 2):
        ef[str(i)] = 1.0
    return ef


@dataclass
class JobConfig:
    num_proc: int = 1
    min_num_proc: int = 1
    max_num_proc: int = 1
    epochs: int = 1

    def validate(self) -> None:
        if self.min_num_proc < 1:
            raise ValueError("MIN_NUM_PROC must be >= 1")
        if self.max_num_proc < self.min_num_proc:
            raise ValueError("MAX_NUM_PROC must be >= MIN_NUM_PROC")
        if not self.min_num_proc <= self.num_proc <= self.max_num_proc:
            raise ValueError("NUM_PROC must lie in [MIN_NUM_PROC, MAX_NUM_PROC]")
        if self.epochs < 0:
            raise ValueError("EPOCHS must be >= 0")


@dataclass
class JobMetrics:
    """Time metrics (trainingjob.go:44-56), seconds."""

    running_time: float = 0.0
    waiting_time: float = 0.0
    gpu_time: float = 0.0
    total_time: float = 0.0
    last_running_time: float = 0.0
    last_waiting_time: float = 0.0
    last_gpu_time: float = 0.0
    first_start_timestamp: float = MAX_TIME
    last_update_timestamp: float = field(default_factory=time.time)


@dataclass
class JobInfo:
    """Per-job performance info used by info-driven policies (trainingjob.go:58-66)."""

    job_name: str = ""
    job_category: str = ""
    gpu_type: str = DEFAULT_GPU_TYPE
    estimate_remainning_time_seconds: float = 0.0
    speedup: dict[str, float] = field(default_factory=linear_speedup)
    efficiency: dict[str, float] = field(default_factory=linear_efficiency)

    def s(self, n: int) -> float:
        """speedup[n] with the reference's missing-key semantics (Go map zero value)."""
        return float(self.speedup.get(str(n), 0.0))


def new_base_job_info(name: str, category: str, gpu_type: str) -> JobInfo:
    return JobInfo(job_name=name, job_category=category, gpu_type=gpu_type)


@dataclass
class TrainingJob:
    job_name: str
    job_category: str
    user: str = "voda"
    kind: str = JobKind.MPIJOB.value
    spec: dict | None = None
    gpu_type: str = DEFAULT_GPU_TYPE
    priority: int = 0
    status: str = JobStatus.SUBMITTED.value
    submit_timestamp: float = field(default_factory=time.time)
    finish_timestamp: float = MAX_TIME
    config: JobConfig = field(default_factory=JobConfig)
    time_metrics: JobMetrics = field(default_factory=JobMetrics)
    info: JobInfo | None = None

    # --- convenient aliases mirroring the Go field names used by the algorithms ---
    @property
    def name(self) -> str:
        return self.job_name

    @property
    def metrics(self) -> JobMetrics:
        return self.time_metrics

    def to_dict(self) -> dict[str, Any]:
        d = asdict(self)
        if self.info is None:
            d.pop("info")  # omitempty, like the reference
        return d

    @classmethod
    def from_dict(cls, d: dict[str, Any]) -> "TrainingJob":
        d = dict(d)
        cfg = JobConfig(**d.pop("config", {}))
        tm = JobMetrics(**d.pop("time_metrics", {}))
        info = d.pop("info", None)
        job = cls(**{k: v for k, v in d.items() if k in cls.__dataclass_fields__},
                  config=cfg, time_metrics=tm)
        job.info = JobInfo(**info) if info else None
        return job

    def clone(self) -> "TrainingJob":
        return copy.deepcopy(self)


# ---------------------------------------------------------------------------------------
# TrainingJobInfo (Mongo job_info schema, mongo.go:22-35) as stored by the job store.
# ---------------------------------------------------------------------------------------
def create_base_job_info_record(job_name: str, max_gpu: int = MAX_NUM_GPU) -> dict[str, Any]:
    """``CreateBaseJobInfo`` (mongo.go:64-95): linear speedup, 1 s epoch/step time."""
    t = {"0": 0.0}
    for i in range(1, max_gpu + 2):
        t[str(i)] = 1.0
    return {
        "name": job_name,
        "gpu_time_sec": 0.0,
        "current_epoch": 0,
        "efficiency": linear_efficiency(max_gpu),
        "elasped_time_sec": 0.0,
        "epoch_time_sec": dict(t),
        "estimated_remainning_time_sec": 0.0,
        "remainning_epochs": 1,
        "running_time_sec": 0.0,
        "speedup": linear_speedup(max_gpu),
        "step_time_sec": dict(t),
        "total_epochs": 1,
        # extension: where the estimates come from (placeholder | profile | measured)
        "info_source": "placeholder",
    }


def init_job_info_record(base: dict[str, Any], job_name: str, epochs: int) -> dict[str, Any]:
    """``initJobInfo`` (handlers.go:212-223): reset progress, estimate remaining time."""
    info = copy.deepcopy(base)
    info.update(
        name=job_name,
        current_epoch=0,
        elasped_time_sec=0.0,
        estimated_remainning_time_sec=float(epochs) * float(base["epoch_time_sec"].get("1", 1.0)),
        gpu_time_sec=0.0,
        remainning_epochs=int(epochs),
        running_time_sec=0.0,
        total_epochs=int(epochs),
    )
    return info


def job_info_from_record(rec: dict[str, Any], category: str, gpu_type: str) -> JobInfo:
    """Map a job_info record to the ``JobInfo`` the algorithms consume (the allocator step
    the reference intended but never delivered)."""
    return JobInfo(job_name=rec["name"], job_category=category, gpu_type=gpu_type,
                   estimate_remainning_time_seconds=float(rec.get("estimated_remainning_time_sec", 0.0)),
                   speedup={k: float(v) for k, v in rec.get("speedup", linear_speedup()).items()},
                   efficiency={k: float(v) for k, v in rec.get("efficiency", linear_efficiency()).items()})


# ---------------------------------------------------------------------------------------
# Constructing a TrainingJob from an MPIJob-shaped spec (trainingjob.go:69-150)
# ---------------------------------------------------------------------------------------
def launcher_env(spec: dict) -> list[dict]:
    try:
        return spec["spec"]["mpiReplicaSpecs"]["Launcher"]["template"]["spec"]["containers"][0].setdefault("env", [])
    except (KeyError, IndexError, TypeError) as e:
        raise ValueError("job spec has no Launcher container") from e


def worker_template_spec(spec: dict) -> dict:
    try:
        return spec["spec"]["mpiReplicaSpecs"]["Worker"]["template"]["spec"]
    except (KeyError, TypeError) as e:
        raise ValueError("job spec has no Worker template") from e


def new_training_job(spec: dict, category: str, submit_time: float | None = None) -> TrainingJob:
    """Parse launcher env knobs + worker nodeSelector into a ``TrainingJob``."""
    name = spec.get("metadata", {}).get("name")
    if not name:
        raise ValueError("job spec has no metadata.name")
    num = mn = mx = epochs = prio = 0
    for e in launcher_env(spec):
        n, v = e.get("name"), e.get("value")
        try:
            if n in (JobConfigEnv.MIN_NUM_PROC, JobConfigEnv.MIN_NUM_PROC_DEPRECATED):
                mn = int(v)
            elif n in (JobConfigEnv.MAX_NUM_PROC, JobConfigEnv.MAX_NUM_PROC_DEPRECATED):
                mx = int(v)
            elif n in (JobConfigEnv.NUM_PROC, JobConfigEnv.NUM_PROC_DEPRECATED):
                num = int(v)
            elif n == JobConfigEnv.EPOCHS:
                epochs = int(v)
            elif n == JobConfigEnv.JOB_PRIORITY:
                prio = int(v)
            elif n == JobConfigEnv.JOB_NAME and v != name:
                raise ValueError("environment variable JOB_NAME and metadata.name mismatched")
        except (TypeError, ValueError) as ex:
            if isinstance(ex, ValueError) and "mismatched" in str(ex):
                raise
            raise ValueError(f"bad value for {n}: {v!r}") from ex
    if num == 0:
        num = mn
    cfg = JobConfig(num_proc=num, min_num_proc=mn, max_num_proc=mx, epochs=epochs)
    # the reference's one rejection of a spec without a scheduler nodeSelector (raw Horovod
    # MPIJobs such as examples/test_yaml/*.yaml) comes first, with its message
    gpu_type = (worker_template_spec(spec).get("nodeSelector") or {}).get(GPU_NAME_LABEL)
    if not gpu_type:
        raise ValueError("gpu type not specified")
    cfg.validate()  # stricter than the reference (trainingjob.go:114 TODO): knobs must be consistent
    return TrainingJob(job_name=name, job_category=category, kind=spec.get("kind", JobKind.MPIJOB.value),
                       spec=spec, gpu_type=gpu_type, priority=prio, status=JobStatus.SUBMITTED.value,
                       submit_timestamp=time.time() if submit_time is None else submit_time,
                       config=cfg, info=None)
