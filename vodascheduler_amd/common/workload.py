"""What a job declares about its own work, and the speed model used to turn that into the
job info the info-driven policies consume.

The reference intends every job to carry per-category history (``getOrCreateBaseJobInfo``
/ ``initJobInfo``, pkg/service/service/handlers.go:180-223) that the metrics collector
keeps current (python/metrics_collector/metrics_collector.py:58-129) and the allocator reads
(pkg/allocator/allocator/resource_allocator.go:115-136).  A category with no history gets
the placeholder of ``CreateBaseJobInfo`` (pkg/common/mongo/mongo.go:64-95): a 1 s epoch and
linear speedup, so an unstarted job looks ``epochs`` seconds long whatever it really is.
SRJF / AFS-L ordered by that placeholder are worse than FIFO (Weak #1).

This module supplies the prior used instead when a category has no measured history: the
workload the job declares (the ``vodascheduler/workload`` annotation, or the model / dataset
/ batch flags of the reference's launcher command line) priced with the MI355X-measured
single-GPU step time of that model and its all-reduce scaling curve
(:class:`ModelProfile`).  Measurements always win over the prior (collector/collector.py).
"""
from __future__ import annotations

import json
import math
import os
import shlex
import dataclasses
from dataclasses import dataclass

from .types import MAX_NUM_GPU

WORKLOAD_ANNOTATION = "vodascheduler/workload"

# Ring all-reduce bus bandwidth (GB/s, fp32 gradients, one 8 x MI355X node over xGMI) used by
# the speed model when no measurement is loaded.  ASSUMED, not measured: ``load_busbw``
# replaces it with the per-world busbw a multi-GPU ``bench.py`` run prints.
ASSUMED_BUSBW_GBS = 300.0
# Cross-node all-reduce bus bandwidth assumed for jobs whose workers span nodes (GB/s).
ASSUMED_INTERNODE_BUSBW_GBS = 40.0

# world size -> measured intra-node busbw (GB/s) at the gradient-bucket size; empty = assumed
_MEASURED_BUSBW: dict[int, float] = {}


def set_measured_busbw(table: dict[int, float] | None) -> None:
    """Install measured per-world bus bandwidths (GB/s); ``None``/empty reverts to the
    assumed constant."""
    _MEASURED_BUSBW.clear()
    for k, v in (table or {}).items():
        if v and float(v) > 0:
            _MEASURED_BUSBW[int(k)] = float(v)


def busbw_source() -> str:
    return "measured" if _MEASURED_BUSBW else "assumed"


def intra_node_busbw(n: int) -> float:
    """Bus bandwidth of an ``n``-GPU ring inside one node: the measured value for that world
    size, else the nearest measured world, else the assumed constant."""
    if not _MEASURED_BUSBW:
        return ASSUMED_BUSBW_GBS
    if n in _MEASURED_BUSBW:
        return _MEASURED_BUSBW[n]
    k = min(_MEASURED_BUSBW, key=lambda w: (abs(w - n), -w))
    return _MEASURED_BUSBW[k]


def load_busbw(path: str, bucket_mb: int = 64) -> dict[int, float]:
    """Read ``allreduce_busbw_gbs`` from bench JSON files (a single ``bench.py --out`` file,
    a driver ``SCALE_rNN.json``, or a JSON list of bench lines) and install it.  Uses the
    ``bucket_mb`` entry (the gradient bucket size) of every world size found."""
    with open(path) as f:
        doc = json.load(f)
    lines: list[dict] = []

    def walk(x):
        if isinstance(x, dict):
            if "allreduce_busbw_gbs" in x and "n_gpus" in x:
                lines.append(x)
            for v in x.values():
                walk(v)
        elif isinstance(x, list):
            for v in x:
                walk(v)
        elif isinstance(x, str) and "allreduce_busbw_gbs" in x:
            for ln in x.splitlines():
                ln = ln.strip()
                if ln.startswith("{") and "allreduce_busbw_gbs" in ln:
                    try:
                        walk(json.loads(ln))
                    except json.JSONDecodeError:
                        pass

    walk(doc)
    table: dict[int, float] = {}
    for ln in lines:
        bw = ln["allreduce_busbw_gbs"] or {}
        v = bw.get(str(bucket_mb)) or bw.get(bucket_mb)
        if v:
            table[int(ln["n_gpus"])] = float(v)
    set_measured_busbw(table)
    return table


# (model, precision) -> {world size: measured seconds per training step} from a bench run's
# online profiling (``step_ms_by_world``); overrides the speed model of the profile of THAT
# precision at the measured world sizes (a mixed bf16 / fp32 trace prices each job with its
# own precision's measurements)
_MEASURED_STEP: dict[tuple[str, str], dict[int, float]] = {}


def _prec(precision: str | None) -> str:
    """bench / workload precision names -> profile precision (``bf16-amp`` is bf16)."""
    return "fp32" if precision == "fp32" else "bf16"


def set_measured_step_times(table: dict[str, dict] | None, precision: str = "bf16", clear: bool = True) -> None:
    """Install measured per-world step times ({model: {world: ms}}) of one compute
    ``precision``; None clears them (all precisions)."""
    if clear or table is None:
        _MEASURED_STEP.clear()
    for model, per in (table or {}).items():
        d = {int(w): float(ms) / 1e3 for w, ms in (per or {}).items() if ms and float(ms) > 0}
        if d:
            _MEASURED_STEP[(model, _prec(precision))] = d


def load_bench_json(path: str, bucket_mb: int = 64) -> dict:
    """Measured busbw (``load_busbw``) AND per-model per-world step times from bench JSON(s):
    the simulator then prices jobs with the hardware's own numbers."""
    bw = load_busbw(path, bucket_mb)
    with open(path) as f:
        doc = json.load(f)
    steps: dict[str, dict[str, dict[str, float]]] = {}  # precision -> model -> {world: ms}

    def walk(x):
        if isinstance(x, dict):
            if isinstance(x.get("step_ms_by_world"), dict):
                by = steps.setdefault(_prec(x.get("precision")), {})
                for m, per in x["step_ms_by_world"].items():
                    by.setdefault(m, {}).update(per)
            for v in x.values():
                walk(v)
        elif isinstance(x, list):
            for v in x:
                walk(v)
        elif isinstance(x, str) and "step_ms_by_world" in x:
            for ln in x.splitlines():
                ln = ln.strip()
                if ln.startswith("{") and "step_ms_by_world" in ln:
                    try:
                        walk(json.loads(ln))
                    except json.JSONDecodeError:
                        pass

    walk(doc)
    set_measured_step_times(None)
    for prec, table in steps.items():
        set_measured_step_times(table, prec, clear=False)
    flat = {m: per for table in steps.values() for m, per in table.items()}
    return {"busbw_gbs": bw, "step_ms_by_world": flat, "step_ms_by_precision": steps}


@dataclass
class ModelProfile:
    """Scaling model of a workload.

    With ``grad_mb`` > 0 (the models measured on MI355X): one step on ``n`` GPUs takes
    ``t1 + exposed(n)`` with ``t1 = step_time_1gpu`` (MEASURED, single MI355X, bf16 compute,
    fp32 gradients) and the ring all-reduce ``c(n) = 2 (n-1)/n * grad_bytes / busbw`` of which
    the part not hidden behind the backward pass (``overlap`` x t1) is exposed;
    ``speedup(n) = n t1 / (t1 + exposed(n))``.  ``busbw`` is the measured per-world value
    when one is loaded (``load_busbw``), else ``ASSUMED_BUSBW_GBS``.  Otherwise the
    Amdahl-like fallback ``n / (1 + alpha (n - 1))`` with a guessed ``alpha``."""

    name: str
    alpha: float
    step_time_1gpu: float  # seconds per step at the per-GPU batch on one GPU
    grad_mb: float = 0.0   # fp32 gradient bytes per step (MB) -- exact, from the parameter count
    overlap: float = 0.3   # fraction of t1 that hides the all-reduce (bucket overlap with backward)
    measured: bool = False
    precision: str = "bf16"  # compute precision the step time is for ("bf16" autocast or "fp32")

    def comm_time(self, n: int, busbw_gbs: float | None = None) -> float:
        if n <= 1:
            return 0.0
        bw = busbw_gbs if busbw_gbs is not None else intra_node_busbw(n)
        return 2.0 * (n - 1) / n * self.grad_mb * 1e6 / (bw * 1e9)

    def t1(self) -> float:
        """Seconds per single-GPU step: this box's measurement when one is installed
        (``set_measured_step_times``: the bench warm-up at the run's precision), else the
        profile's."""
        meas = _MEASURED_STEP.get((self.name, self.precision))
        return meas.get(1, self.step_time_1gpu) if meas else self.step_time_1gpu

    def speedup(self, n: int, busbw_gbs: float | None = None) -> float:
        if n <= 0:
            return 0.0
        meas = _MEASURED_STEP.get((self.name, self.precision))
        if meas and n in meas and busbw_gbs is None:
            # measured: n workers each process one per-GPU batch per step of meas[n] seconds
            return n * self.t1() / meas[n]
        if self.grad_mb > 0:
            t1 = self.t1()
            c = self.comm_time(n, busbw_gbs)
            exposed = max(0.0, c - self.overlap * t1)
            return n * t1 / (t1 + exposed)
        return n / (1.0 + self.alpha * (n - 1))


# step_time_1gpu: MI355X measurements (bf16 autocast compute, fp32 flat gradients): ResNet-50
# bs256 23.15 ms (end of round 3, profiles/r3/resnet50_steps.md) and BERT-base bs64 seq128
# 10.2 ms (kernel time per step: 10.21 ms in profiles/r3/rocprof_bert_bf16_final.md, 10.18 ms
# with the fused attention in profiles/r3/rocprof_bert_bf16_session2_final.md; the bench
# workers' graph replays run 9.9-10.5 ms by box); VGG16 bs128 2.63 ms, NMT
# Transformer bs512 5.24 ms, ResNet-50-CIFAR bs128 14.3 ms, ResNet-18 bs256 10.05 ms,
# InceptionV3 bs128 13.5 ms, Keras MNIST 0.74 ms (benchmarks/model_step.py).  mnist-torch is
# an estimate (measured=False).  grad_mb = 4 bytes x parameter count.
PROFILES = {
    "resnet50": ModelProfile("resnet50", alpha=0.01, step_time_1gpu=0.02315, grad_mb=102.2, measured=True),
    "bert-base": ModelProfile("bert-base", alpha=0.05, step_time_1gpu=0.0102, grad_mb=438.0, measured=True),
    "vgg16": ModelProfile("vgg16", alpha=0.08, step_time_1gpu=0.00263, grad_mb=134.6, measured=True),
    "transformer": ModelProfile("transformer", alpha=0.10, step_time_1gpu=0.00524, grad_mb=79.8, measured=True),
    "mnist": ModelProfile("mnist", alpha=0.30, step_time_1gpu=0.00074, grad_mb=4.8, measured=True),
    "mnist-torch": ModelProfile("mnist-torch", alpha=0.40, step_time_1gpu=0.002, grad_mb=0.087),
    "resnet50-cifar": ModelProfile("resnet50-cifar", alpha=0.05, step_time_1gpu=0.0143, grad_mb=94.1, measured=True),
    "resnet18": ModelProfile("resnet18", alpha=0.04, step_time_1gpu=0.01005, grad_mb=46.8, measured=True),
    "inceptionv3": ModelProfile("inceptionv3", alpha=0.05, step_time_1gpu=0.0135, grad_mb=87.3, measured=True),
}


# fp32 compute (the reference's precision: tensorflow2_keras_cifar_elastic.py:147-166 builds
# the Keras model with no mixed-precision policy; pytorch_mnist_elastic.py is plain fp32):
# MI355X single-GPU step times, same batches.  ResNet-50 58.16 ms / BERT-base 31.68 ms at the end of
# round 6 (bench.py warm-up, ``warmup_single_gpu_step_ms`` of profiles/r6/bench_n1_fp32_r6z.json;
# 58.75 / 33.53 before the variant-8 split GEMM, r6i; 63.18 / 35.59 early in round 6, r6a; round 4
# ended at 69.96 / 37.1, BENCH_r04); the other models' fp32 step times are unmeasured, so they fall
# back to the bf16 profile.
PROFILES_FP32 = {
    "resnet50": ModelProfile("resnet50", alpha=0.01, step_time_1gpu=0.05816, grad_mb=102.2, measured=True,
                             precision="fp32"),
    "bert-base": ModelProfile("bert-base", alpha=0.05, step_time_1gpu=0.03168, grad_mb=438.0, measured=True,
                              precision="fp32"),
}
PRECISIONS = ("bf16", "fp32")


def model_profile(model: str, precision: str = "bf16") -> ModelProfile | None:
    """The MI355X profile of ``model`` at a compute precision (``bf16`` = bf16 autocast with
    fp32 master weights / gradients, ``fp32`` = the reference's precision)."""
    if precision == "fp32" and model in PROFILES_FP32:
        return PROFILES_FP32[model]
    prof = PROFILES.get(model)
    if prof is not None and precision == "fp32":
        # no fp32 profile: the bf16 numbers stand in, but labelled fp32 so that step times
        # measured at fp32 (set_measured_step_times(..., "fp32")) apply to this job
        prof = dataclasses.replace(prof, precision="fp32")
    return prof


def profile_of(wl: dict) -> ModelProfile:
    """The speed model of a declared workload: the model's MI355X profile at the workload's
    declared ``precision`` (default bf16); a model without one gets the Amdahl fallback with
    the workload's own ``alpha`` and a step time derived from its declared epoch time."""
    prof = model_profile(wl.get("model", ""), wl.get("precision", "bf16"))
    if prof is not None:
        return prof
    spe = max(1, int(wl.get("steps_per_epoch", 1)))
    t1 = float(wl["epoch_time_1gpu"]) / spe if wl.get("epoch_time_1gpu") else 0.05
    return ModelProfile(wl.get("model", "?"), float(wl.get("alpha", 0.05)), t1)


def speedup_table(profile: ModelProfile, max_gpu: int = MAX_NUM_GPU) -> dict[str, float]:
    """Speedup keyed by the worker count as a decimal string, "0".."max_gpu+1"
    (reference trainingjob.go:168-187)."""
    return {str(i): profile.speedup(i) for i in range(0, max_gpu + 2)}


def workload_of(spec: dict) -> dict:
    """The job's workload: the ``vodascheduler/workload`` annotation, or -- for specs written
    for the reference (no annotation) -- what the launcher command line says: the
    reference's example scripts take ``--model ResNet50|VGG16|InceptionV3 --dataset cifar10``
    (examples/yaml/tensorflow2/*.yaml), the MNIST / Transformer scripts are recognised by
    name, and ``--model <workload>`` names any workload of this framework's model zoo."""
    wl = declared_workload(spec)
    if wl is None:
        raise KeyError("job spec has no workload annotation and no recognisable launcher command")
    return wl


def declared_workload(spec: dict | None) -> dict | None:
    """``workload_of`` that returns None instead of raising."""
    if not spec:
        return None
    ann = (spec.get("metadata", {}).get("annotations") or {}).get(WORKLOAD_ANNOTATION)
    if ann:
        return json.loads(ann)
    return workload_from_launcher(spec)


_REF_MODELS = {"resnet50": "resnet50", "vgg16": "vgg16", "inceptionv3": "inceptionv3", "resnet18": "resnet18"}
_DATASET_SAMPLES = {"cifar10": 50000, "mnist": 60000, "imagenet": 1281167}


def workload_from_launcher(spec: dict) -> dict | None:
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
    try:
        bs = int(opts.get("batch-size", WORKLOADS[name].per_gpu_batch))
    except ValueError:
        bs = WORKLOADS[name].per_gpu_batch
    if "steps-per-epoch" in opts and opts["steps-per-epoch"].isdigit():
        spe = int(opts["steps-per-epoch"])
    else:
        spe = max(1, _DATASET_SAMPLES.get(dataset or "", 100 * bs) // bs)
    prof = PROFILES.get(name, ModelProfile(name, 0.05, 0.05))
    out = {"model": name, "steps_per_epoch": spe, "per_gpu_batch": bs, "alpha": prof.alpha,
           "epoch_time_1gpu": spe * prof.step_time_1gpu}
    if "lr" in opts:
        try:
            out["lr"] = float(opts["lr"])
        except ValueError:
            pass
    # boolean flags of the reference scripts (pytorch_mnist_elastic.py:32, cifar :145)
    if "--use-adasum" in toks:
        out["reduction"] = "adasum"
    if "--fp16-allreduce" in toks:
        out["compression"] = "fp16"
    return out


# ---------------------------------------------------------------------------------------
# job_info priors
# ---------------------------------------------------------------------------------------
INFO_PLACEHOLDER = "placeholder"   # reference CreateBaseJobInfo: 1 s epochs, linear speedup
INFO_PROFILE = "profile"           # declared workload x MI355X speed model
INFO_MEASURED = "measured"         # collector measurements (this job or its category)


def declared_steps_1gpu(wl: dict, epochs: int) -> float:
    """Total single-GPU steps of a declared workload (``epochs x steps_per_epoch``)."""
    return float(max(1, epochs)) * float(max(1, int(wl.get("steps_per_epoch", 1))))


def prior_fields(wl: dict, epochs: int, max_gpu: int = MAX_NUM_GPU) -> dict:
    """job_info fields (mongo.go:22-35 schema) estimated from a declared workload: remaining
    time = ``epochs x epoch_time_1gpu`` one-GPU seconds, speedup / efficiency from the
    model's scaling curve, per-worker-count step / epoch time consistent with both."""
    prof = profile_of(wl)
    spe = max(1, int(wl.get("steps_per_epoch", 1)))
    ep1 = float(wl["epoch_time_1gpu"]) if wl.get("epoch_time_1gpu") else spe * prof.step_time_1gpu
    t1 = ep1 / spe
    sp = speedup_table(prof, max_gpu)
    step_t = {"0": 0.0}
    epoch_t = {"0": 0.0}
    for k in range(1, max_gpu + 2):
        s = sp[str(k)]
        # k workers split the epoch's samples: spe / k steps of k x t1 / s(k) seconds
        step_t[str(k)] = k * t1 / s if s > 0 else t1
        epoch_t[str(k)] = ep1 / s if s > 0 else ep1
    return {
        "info_source": INFO_PROFILE,
        "speedup": sp,
        "efficiency": {k: (v / int(k) if int(k) else 0.0) for k, v in sp.items()},
        "step_time_sec": step_t,
        "epoch_time_sec": epoch_t,
        "estimated_remainning_time_sec": float(max(1, epochs)) * ep1,
    }


def remaining_from_history(base: dict, wl: dict | None, epochs: int) -> float:
    """Remaining one-GPU seconds of a new job from its category's measured history: the
    measured 1-GPU step time x the job's own declared step count when it declares one (jobs
    of a category may differ in length), else the reference's ``epochs x epoch_time(1)``."""
    st1 = float((base.get("step_time_sec") or {}).get("1", 0.0) or 0.0)
    if wl is not None and st1 > 0 and "steps_per_epoch" in wl:
        return declared_steps_1gpu(wl, epochs) * st1
    return float(epochs) * float((base.get("epoch_time_sec") or {}).get("1", 1.0))


def finite(x: float, default: float = 0.0) -> float:
    return x if isinstance(x, (int, float)) and math.isfinite(x) else default


def busbw_from_env() -> None:
    """``VODA_BUSBW_JSON=<bench json>`` installs measured busbw at import time of the
    services that price all-reduces (simulator, experiments)."""
    p = os.environ.get("VODA_BUSBW_JSON")
    if p and os.path.exists(p):
        load_busbw(p)
