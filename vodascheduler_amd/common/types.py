"""Shared enums and constants (reference pkg/common/types/types.go:8-65, config/config.go:3-12)."""
from __future__ import annotations

from enum import Enum


class JobConfigEnv(str, Enum):
    """Launcher env vars that configure a job (types.go:10-28)."""

    NUM_PROC = "NUM_PROC"
    MIN_NUM_PROC = "MIN_NUM_PROC"
    MAX_NUM_PROC = "MAX_NUM_PROC"
    NUM_PROC_DEPRECATED = "NP"
    MIN_NUM_PROC_DEPRECATED = "MIN_NP"
    MAX_NUM_PROC_DEPRECATED = "MAX_NP"
    EPOCHS = "EPOCHS"
    JOB_NAME = "JOB_NAME"
    JOB_PRIORITY = "JOB_PRIORITY"
    # extension: jobs naming the same category share job-info history (the reference uses the
    # un-timestamped job name as the category, handlers.go:180-206)
    JOB_CATEGORY = "JOB_CATEGORY"


class JobStatus(str, Enum):
    """Job status FSM (types.go:33-48): Submitted -> Waiting <-> Running -> Completed|Failed, + Canceled."""

    SUBMITTED = "Submitted"
    WAITING = "Waiting"
    RUNNING = "Running"
    COMPLETED = "Completed"
    FAILED = "Failed"
    CANCELED = "Canceled"

    @property
    def done(self) -> bool:
        return self in (JobStatus.COMPLETED, JobStatus.FAILED, JobStatus.CANCELED)


class JobKind(str, Enum):
    MPIJOB = "MPIJob"
    TFJOB = "TFJob"
    PYTORCHJOB = "PyTorchJob"
    # native kind of this framework: an elastic job run by the local node agent
    ELASTICJOB = "ElasticJob"


# JobScheduleResult: job name -> number of GPUs (types.go:61)
JobScheduleResult = dict

# types.go:65 uses the max representable Go time; a JSON-safe sentinel (year 9999) here.
MAX_TIME = 253402300799.0

# ---- global config (config/config.go:3-12) ----
NAME = "vodascheduler"
VERSION = "0.2.2-amd"
PORT_TRAINING_SERVICE = 55587
PORT_SCHEDULER = 55588
PORT_ALLOCATOR = 55589
ENTRY_POINT = "/training"
TAINT_KEY = "vodascheduler/hostname"
NAMESPACE = "voda-scheduler"
GPU_NAME_LABEL = "vodascheduler/accelerator"
GPU_RESOURCE = "amd.com/gpu"  # nvidia.com/gpu in the reference (scheduler.go:903-906)
DEFAULT_GPU_TYPE = "amd-instinct-mi355x"

# ---- behaviour constants ----
RESCHED_RATE_LIMIT_SEC = 30.0        # scheduler.go:212
TIME_METRICS_TICK_SEC = 5.0          # scheduler.go:48
RESCHED_CHANNEL_SIZE = 100           # scheduler.go:47
MQ_BUFFER = 200                      # rabbitmq.go:13
MAX_NUM_GPU = 32                     # trainingjob.go:13 (speedup table size, +1)
DB_JOB_INFO = "job_info"
DB_JOB_METADATA = "job_metadata"
COLLECTION_JOB_METADATA = "v1beta1"
