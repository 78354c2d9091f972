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

from ..common.types import DEFAULT_GPU_TYPE, GPU_NAME_LABEL, GPU_RESOURCE

WORKLOAD_ANNOTATION = "vodascheduler/workload"


# Ring all-reduce bus bandwidth assumed for the speed model until the multi-GPU bench measures
# it (GB/s, fp32 gradients, one 8 x MI355X node over xGMI).  ASSUMED, not measured.
ASSUMED_BUSBW_GBS = 300.0
# Cross-node all-reduce bus bandwidth assumed for jobs whose workers span nodes (GB/s).
ASSUMED_INTERNODE_BUSBW_GBS = 40.0


@dataclass
class ModelProfile:
    """Scaling model of a workload.

    With ``grad_mb`` > 0 (the models measured on MI355X): one step on ``n`` GPUs takes
    ``t1 + exposed(n)`` with ``t1 = step_time_1gpu`` (MEASURED, single MI355X, bf16 compute,
    fp32 gradients) and the ring all-reduce ``c(n) = 2 (n-1)/n * grad_bytes / busbw`` of which
    the part not hidden behind the backward pass (``overlap`` x t1) is exposed;
    ``speedup(n) = n t1 / (t1 + exposed(n))``.  ``busbw`` is ASSUMED (``ASSUMED_BUSBW_GBS``)
    until the 8-GPU bench measures it.  Otherwise the Amdahl-like fallback
    ``n / (1 + alpha (n - 1))`` with a guessed ``alpha``."""

    name: str
    alpha: float
    step_time_1gpu: float  # seconds per step at the per-GPU batch on one GPU
    grad_mb: float = 0.0   # fp32 gradient bytes per step (MB) -- exact, from the parameter count
    overlap: float = 0.3   # fraction of t1 that hides the all-reduce (bucket overlap with backward)
    measured: bool = False

    def comm_time(self, n: int, busbw_gbs: float = ASSUMED_BUSBW_GBS) -> float:
        if n <= 1:
            return 0.0
        return 2.0 * (n - 1) / n * self.grad_mb * 1e6 / (busbw_gbs * 1e9)

    def speedup(self, n: int, busbw_gbs: float | None = None) -> float:
        if n <= 0:
            return 0.0
        if self.grad_mb > 0:
            t1 = self.step_time_1gpu
            c = self.comm_time(n, busbw_gbs or ASSUMED_BUSBW_GBS)
            exposed = max(0.0, c - self.overlap * t1)
            return n * t1 / (t1 + exposed)
        return n / (1.0 + self.alpha * (n - 1))


# step_time_1gpu: MI355X measurements of the eager step (benchmarks/model_step.py, bf16
# autocast, fp32 flat gradients; profiles/r2_*, docs/PERFORMANCE.md), end of round 2:
# ResNet-50 bs256 26.2 ms, BERT-base bs64 seq128 11.45 ms, VGG16 bs128 2.63 ms, NMT
# Transformer bs512 5.24 ms, ResNet-50-CIFAR bs128 14.3 ms, ResNet-18 bs256 10.05 ms,
# InceptionV3 bs128 13.5 ms, Keras MNIST 0.74 ms.  mnist-torch is an estimate
# (measured=False).  grad_mb = 4 bytes x parameter count; alpha is only the fallback when
# grad_mb is unknown (the speed model prices the all-reduce from grad_mb and an ASSUMED busbw).
PROFILES = {
    "resnet50": ModelProfile("resnet50", alpha=0.01, step_time_1gpu=0.0262, grad_mb=102.2, measured=True),
    "bert-base": ModelProfile("bert-base", alpha=0.05, step_time_1gpu=0.01145, grad_mb=438.0, measured=True),
    "vgg16": ModelProfile("vgg16", alpha=0.08, step_time_1gpu=0.00263, grad_mb=134.6, measured=True),
    "transformer": ModelProfile("transformer", alpha=0.10, step_time_1gpu=0.00524, grad_mb=79.8, measured=True),
    "mnist": ModelProfile("mnist", alpha=0.30, step_time_1gpu=0.00074, grad_mb=4.8, measured=True),
    "mnist-torch": ModelProfile("mnist-torch", alpha=0.40, step_time_1gpu=0.002, grad_mb=0.087),
    "resnet50-cifar": ModelProfile("resnet50-cifar", alpha=0.05, step_time_1gpu=0.0143, grad_mb=94.1, measured=True),
    "resnet18": ModelProfile("resnet18", alpha=0.04, step_time_1gpu=0.01005, grad_mb=46.8, measured=True),
    "inceptionv3": ModelProfile("inceptionv3", alpha=0.05, step_time_1gpu=0.0135, grad_mb=87.3, measured=True),
}


def speedup_table(profile: ModelProfile, max_gpu: int = 32) -> dict[str, float]:
    """Speedup keyed by the worker count as a decimal string, "0".."max_gpu+1"
    (reference trainingjob.go:168-187)."""
    return {str(i): profile.speedup(i) for i in range(0, max_gpu + 2)}


def make_spec(name: str, model: str, np_: int, min_np: int, max_np: int, epochs: int, steps_per_epoch: int,
              gpu_type: str = DEFAULT_GPU_TYPE, priority: int | None = None, per_gpu_batch: int | None = None,
              epoch_time_1gpu: float | None = None) -> dict:
    prof = PROFILES[model]
    env = [{"name": "JOB_NAME", "value": name}, {"name": "NP", "value": str(np_)},
           {"name": "MIN_NP", "value": str(min_np)}, {"name": "MAX_NP", "value": str(max_np)},
           {"name": "EPOCHS", "value": str(epochs)}]
    if priority is not None:
        env.append({"name": "JOB_PRIORITY", "value": str(priority)})
    wl = {"model": model, "steps_per_epoch": steps_per_epoch,
          "epoch_time_1gpu": epoch_time_1gpu if epoch_time_1gpu is not None else steps_per_epoch * prof.step_time_1gpu,
          "alpha": prof.alpha}
    if per_gpu_batch is not None:
        wl["per_gpu_batch"] = per_gpu_batch
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


def workload_of(spec: dict) -> dict:
    """The job's workload: the ``vodascheduler/workload`` annotation, or -- for specs written
    for the reference (no annotation) -- what the launcher command line says: the
    reference's example scripts take ``--model ResNet50|VGG16|InceptionV3 --dataset cifar10``
    (examples/yaml/tensorflow2/*.yaml), the MNIST / Transformer scripts are recognised by
    name, and ``--model <workload>`` names any workload of this framework's model zoo."""
    ann = (spec.get("metadata", {}).get("annotations") or {}).get(WORKLOAD_ANNOTATION)
    if ann:
        return json.loads(ann)
    wl = workload_from_launcher(spec)
    if wl is None:
        raise KeyError("job spec has no workload annotation and no recognisable launcher command")
    return wl


_REF_MODELS = {"resnet50": "resnet50", "vgg16": "vgg16", "inceptionv3": "inceptionv3", "resnet18": "resnet18"}
_DATASET_SAMPLES = {"cifar10": 50000, "mnist": 60000, "imagenet": 1281167}


def workload_from_launcher(spec: dict) -> dict | None:
    import shlex

    try:
        cont = spec["spec"]["mpiReplicaSpecs"]["Launcher"]["template"]["spec"]["containers"][0]
    except (KeyError, IndexError, TypeError):
        return None
    text = " ".join(str(x) for x in (cont.get("command") or []) + (cont.get("args") or []))
    try:
        toks = shlex.split(text.replace(";", " ; "))
    except ValueError:
        toks = text.split()
    opts: dict[str, str] = {}
    for i, t in enumerate(toks[:-1]):
        if t.startswith("--"):
            opts[t[2:].replace("_", "-")] = toks[i + 1]
    script = " ".join(t for t in toks if t.endswith(".py") or t.startswith("vodascheduler_amd."))
    from ..models import WORKLOADS

    model = opts.get("model", "")
    dataset = opts.get("dataset", "").lower()
    key = model.lower().replace("_", "").replace("-", "")
    if model in WORKLOADS:
        name = model
    elif key in _REF_MODELS:
        name = _REF_MODELS[key]
        if name == "resnet50" and dataset.startswith("cifar"):
            name = "resnet50-cifar"
    elif "mnist" in script:
        name, dataset = ("mnist-torch" if "pytorch" in script else "mnist"), "mnist"
    elif "transformer" in script:
        name = "transformer"
    else:
        return None
    w = WORKLOADS[name]
    bs = int(opts.get("batch-size", w.per_gpu_batch))
    if "steps-per-epoch" in opts:
        spe = int(opts["steps-per-epoch"])
    else:
        spe = max(1, _DATASET_SAMPLES.get(dataset or "", 100 * bs) // bs)
    prof = PROFILES.get(name, ModelProfile(name, 0.05, 0.05))
    out = {"model": name, "steps_per_epoch": spe, "per_gpu_batch": bs, "alpha": prof.alpha,
           "epoch_time_1gpu": spe * prof.step_time_1gpu}
    if "lr" in opts:
        out["lr"] = float(opts["lr"])
    # boolean flags of the reference scripts (pytorch_mnist_elastic.py:32, cifar :145)
    if "--use-adasum" in toks:
        out["reduction"] = "adasum"
    if "--fp16-allreduce" in toks:
        out["compression"] = "fp16"
    return out


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
                 elastic: bool = True, duration_scale: float = 1.0) -> list[TraceJob]:
    """Generate ``n_jobs`` jobs.  Sizes: 1 GPU 50 %, 2 GPUs 25 %, 4 GPUs 15 %, 8 GPUs 10 %
    (capped at ``max_gpus``); durations log-normal (sigma 1.0) around the mean GPU-time."""
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
        out.append(TraceJob(t, make_spec(name, model, np_, min_np, max_np, epochs, steps_per_epoch)))
    return out


def bench_trace(n_jobs: int = 32, mean_steps: int = 30, n_gpus: int = 1, seed: int = 0,
                mean_interarrival_s: float = 0.5, models: tuple[str, ...] = ("resnet50", "bert-base"),
                batches: dict[str, int] | None = None, epochs: int = 2) -> list[TraceJob]:
    """The 32-job Philly-style trace run by ``bench.py`` on real MI355X GPUs.

    Weak scaling: every job's work (single-GPU steps at the per-GPU batch) is multiplied by
    ``n_gpus``, so the per-GPU work is fixed as the pool grows.  Requests follow the Philly
    size mix capped at ``n_gpus``; every job is elastic in ``[1, min(n_gpus, 2 x request)]``.
    Durations are log-normal (sigma 0.8) around ``mean_steps``; arrivals are Poisson.
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
        out.append(TraceJob(t, make_spec(f"{model}-j{i:02d}", model, np_, 1, max_np, epochs, spe,
                                         per_gpu_batch=batches.get(model))))
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
