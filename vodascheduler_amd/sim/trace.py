"""Synthetic Philly-style job traces (BASELINE.json: "32-job Philly-style synthetic trace").

The reference publishes no trace or numbers; this generator follows the
published shape of the Microsoft Philly workload: Poisson arrivals, mostly small jobs
(1-GPU dominated, power-of-two requests), heavy-tailed (log-normal) durations.  Each job
is an MPIJob-shaped spec with the reference's launcher env knobs (NP / MIN_NP / MAX_NP /
EPOCHS) plus a ``vodascheduler/workload`` annotation that the simulator and the GPU pool
backend read: the model, the per-epoch time on one GPU and its scaling curve.
"""
from __future__ import annotations

import json
import math
import random
from dataclasses import dataclass

from ..common.types import DEFAULT_GPU_TYPE, GPU_NAME_LABEL, GPU_RESOURCE, JobConfigEnv
from ..common.workload import (ASSUMED_BUSBW_GBS, ASSUMED_INTERNODE_BUSBW_GBS, PROFILES,  # noqa: F401
                               WORKLOAD_ANNOTATION, ModelProfile, model_profile, speedup_table,
                               workload_from_launcher, workload_of)


def make_spec(name: str, model: str, np_: int, min_np: int, max_np: int, epochs: int, steps_per_epoch: int,
              gpu_type: str = DEFAULT_GPU_TYPE, priority: int | None = None, per_gpu_batch: int | None = None,
              epoch_time_1gpu: float | None = None, category: str | None = None,
              precision: str | None = None) -> dict:
    """An MPIJob spec with the reference's launcher env knobs.  ``category``: the
    ``JOB_CATEGORY`` knob -- jobs of one category share measured job-info history (the
    reference keys history by the un-timestamped job name, handlers.go:180-206).
    ``precision`` (bf16 | fp32) is declared in the workload annotation: it prices the job
    (``common.workload.model_profile``) and selects the workers' compute precision."""
    prof = model_profile(model, precision or "bf16")
    env = [{"name": "JOB_NAME", "value": name}, {"name": "NP", "value": str(np_)},
           {"name": "MIN_NP", "value": str(min_np)}, {"name": "MAX_NP", "value": str(max_np)},
           {"name": "EPOCHS", "value": str(epochs)}]
    if priority is not None:
        env.append({"name": "JOB_PRIORITY", "value": str(priority)})
    if category is not None:
        env.append({"name": JobConfigEnv.JOB_CATEGORY.value, "value": category})
    wl = {"model": model, "steps_per_epoch": steps_per_epoch,
          "epoch_time_1gpu": epoch_time_1gpu if epoch_time_1gpu is not None else steps_per_epoch * prof.step_time_1gpu,
          "alpha": prof.alpha}
    if per_gpu_batch is not None:
        wl["per_gpu_batch"] = per_gpu_batch
    if precision is not None:
        wl["precision"] = precision
    cmd = (f"vodarun --min-np $(MIN_NP) --max-np $(MAX_NP) python -m vodascheduler_amd.workloads.train "
           f"--model {model} --epochs $(EPOCHS) --steps-per-epoch {steps_per_epoch} --name $(JOB_NAME)")
    return {
        "apiVersion": "kubeflow.org/v1",
        "kind": "MPIJob",
        "metadata": {"name": name, "annotations": {WORKLOAD_ANNOTATION: json.dumps(wl)}},
        "spec": {
            "slotsPerWorker": 1,
            "cleanPodPolicy": "Running",
            "mpiReplicaSpecs": {
                "Launcher": {"replicas": 1, "template": {"spec": {"containers": [
                    {"name": "launcher", "image": "vodascheduler-amd:latest", "env": env,
                     "command": ["/bin/bash", "-c"], "args": [cmd]}]}}},
                "Worker": {"replicas": np_, "template": {"spec": {
                    "containers": [{"name": "worker", "image": "vodascheduler-amd:latest",
                                    "resources": {"limits": {GPU_RESOURCE: 1}}}],
                    "nodeSelector": {GPU_NAME_LABEL: gpu_type}}}},
            },
        },
    }


@dataclass
class TraceJob:
    submit_time: float
    spec: dict

    @property
    def name(self) -> str:
        return self.spec["metadata"]["name"]


def philly_trace(n_jobs: int = 32, seed: int = 0, mean_interarrival_s: float = 30.0,
                 mean_duration_1gpu_s: float = 600.0, max_gpus: int = 8,
                 models: tuple[str, ...] = ("resnet50", "bert-base", "vgg16", "transformer"),
                 elastic: bool = True, duration_scale: float = 1.0, precision: str | None = None) -> list[TraceJob]:
    """Generate ``n_jobs`` jobs.  Sizes: 1 GPU 50 %, 2 GPUs 25 %, 4 GPUs 15 %, 8 GPUs 10 %
    (capped at ``max_gpus``); durations log-normal (sigma 1.0) around the mean GPU-time of the
    bf16 profile.  ``precision`` (bf16 | fp32) is declared by every job: the same steps
    (the same work) are then priced at that precision's step time, so an fp32 trace runs
    ~3x longer than the bf16 one (``common.workload.PROFILES_FP32``)."""
    rng = random.Random(seed)
    sizes, weights = [1, 2, 4, 8], [0.50, 0.25, 0.15, 0.10]
    t = 0.0
    out = []
    for i in range(n_jobs):
        if i > 0:
            t += rng.expovariate(1.0 / mean_interarrival_s)
        np_ = min(rng.choices(sizes, weights)[0], max_gpus)
        model = models[i % len(models)]
        prof = PROFILES[model]
        gpu_seconds = rng.lognormvariate(math.log(mean_duration_1gpu_s) - 0.5, 1.0) * duration_scale
        gpu_seconds = max(gpu_seconds, 20 * prof.step_time_1gpu)
        epochs = max(1, min(20, int(round(gpu_seconds / 60.0)) or 1))
        steps_per_epoch = max(1, int(round(gpu_seconds / epochs / prof.step_time_1gpu)))
        min_np = 1 if elastic else np_
        max_np = min(max_gpus, max(np_ * 2, 2)) if elastic else np_
        name = f"{model}-j{i:02d}"
        out.append(TraceJob(t, make_spec(name, model, np_, min_np, max_np, epochs, steps_per_epoch,
                                         category=model, precision=precision)))
    return out


def bench_trace(n_jobs: int = 32, mean_steps: int = 30, n_gpus: int = 1, seed: int = 0,
                mean_interarrival_s: float = 0.5, models: tuple[str, ...] = ("resnet50", "bert-base"),
                batches: dict[str, int] | None = None, epochs: int = 2, precision: str | None = None,
                step_time_s: dict[str, float] | None = None) -> list[TraceJob]:
    """The 32-job Philly-style trace run by ``bench.py`` on real MI355X GPUs.

    Weak scaling: every job's work (single-GPU steps at the per-GPU batch) is multiplied by
    ``n_gpus``, so the per-GPU work is fixed as the pool grows.  Requests follow the Philly
    size mix capped at ``n_gpus``; every job is elastic in ``[1, min(n_gpus, 2 x request)]``.
    Durations are log-normal (sigma 0.8) around ``mean_steps``; arrivals are Poisson.
    ``precision`` is declared in every job's workload; ``step_time_s`` (model -> measured
    seconds per single-GPU step on this box at that precision) prices the declared epoch
    times -- the job-info priors of the info-driven policies -- instead of the profiles.
    """
    rng = random.Random(seed)
    sizes, weights = [1, 2, 4, 8], [0.50, 0.25, 0.15, 0.10]
    batches = batches or {}
    t = 0.0
    out = []
    for i in range(n_jobs):
        if i > 0:
            t += rng.expovariate(1.0 / mean_interarrival_s)
        np_ = min(rng.choices(sizes, weights)[0], n_gpus)
        model = models[i % len(models)]
        steps = max(2 * epochs, int(round(rng.lognormvariate(math.log(mean_steps) - 0.32, 0.8) * n_gpus)))
        spe = max(1, steps // epochs)
        max_np = max(np_, min(n_gpus, 2 * np_))
        ep1 = spe * step_time_s[model] if step_time_s and step_time_s.get(model) else None
        out.append(TraceJob(t, make_spec(f"{model}-j{i:02d}", model, np_, 1, max_np, epochs, spe,
                                         per_gpu_batch=batches.get(model), category=model,
                                         epoch_time_1gpu=ep1, precision=precision)))
    return out


def scale_trace(trace: list[TraceJob], work_scale: float) -> list[TraceJob]:
    """Multiply every job's work (steps per epoch) by ``work_scale`` (weak scaling over N GPUs)."""
    out = []
    for tj in trace:
        spec = json.loads(json.dumps(tj.spec))
        wl = workload_of(spec)
        wl["steps_per_epoch"] = max(1, int(round(wl["steps_per_epoch"] * work_scale)))
        wl["epoch_time_1gpu"] = wl["epoch_time_1gpu"] * work_scale
        spec["metadata"]["annotations"][WORKLOAD_ANNOTATION] = json.dumps(wl)
        out.append(TraceJob(tj.submit_time, spec))
    return out
