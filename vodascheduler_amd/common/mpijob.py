"""MPIJob-shaped job specs: parse, mutate and query (kubeflow.org/v1 MPIJob CRD shape).

Reference: service-side parsing/renaming (pkg/service/service/handlers.go:60-171), the
scheduler's spec mutations (pkg/scheduler/scheduler/scheduler.go:519-524,891-914) and
MPIJob status helpers (pkg/scheduler/scheduler/status.go:9-29).  Specs are plain dicts
(no kubernetes client in this image); every mutation keeps the CRD shape so the same YAML
can be fed to a real MPI-Operator via ``backend/k8s.py``.
"""
from __future__ import annotations

import copy
import re
import shlex
import time
from datetime import datetime

import yaml

from .types import GPU_NAME_LABEL, GPU_RESOURCE, NAMESPACE, JobConfigEnv
from .trainingjob import launcher_env, worker_template_spec

TIMESTAMP_RE = re.compile(r"-\d{8}-\d{6}$")


def load_spec(data: bytes | str) -> dict:
    """YAML/JSON bytes -> MPIJob dict (``bytesToMPIJob``, handlers.go:142-156)."""
    if isinstance(data, bytes):
        data = data.decode()
    spec = yaml.safe_load(data)
    if not isinstance(spec, dict):
        raise ValueError("job spec must be a YAML/JSON mapping")
    if spec.get("kind") not in ("MPIJob", "ElasticJob", None):
        raise ValueError(f"unsupported job kind {spec.get('kind')!r}")
    if "metadata" not in spec or "name" not in spec["metadata"]:
        raise ValueError("job spec has no metadata.name")
    launcher_env(spec)  # validates Launcher container presence
    worker_template_spec(spec)
    return spec


def timestamped_name(name: str, now: float | None = None) -> str:
    """``name-YYYYMMDD-hhmmss``.  The reference formats with Go layout ``20060102-030405``,
    i.e. a 12-hour clock (handlers.go:86); we use a 24-hour clock so names stay unique
    and sortable (documented deviation)."""
    ts = datetime.fromtimestamp(time.time() if now is None else now)
    return f"{name}-{ts.strftime('%Y%m%d-%H%M%S')}"


def category_of(job_name: str) -> str:
    """Strip the timestamp suffix (metrics_collector.py:73-79)."""
    return TIMESTAMP_RE.sub("", job_name)


def set_name(spec: dict, name: str) -> None:
    spec["metadata"]["name"] = name
    set_env_job_name(spec, name)


def set_env_job_name(spec: dict, name: str) -> None:
    """Set or ADD the launcher JOB_NAME env var.  The reference appends to a local slice
    copy so the added variable is lost; fixed here."""
    env = launcher_env(spec)
    for e in env:
        if e.get("name") == JobConfigEnv.JOB_NAME:
            e["value"] = name
            return
    env.append({"name": JobConfigEnv.JOB_NAME.value, "value": name})


def get_env(spec: dict, key: str, default: str | None = None) -> str | None:
    for e in launcher_env(spec):
        if e.get("name") == key:
            return e.get("value")
    return default


def set_worker_replicas(spec: dict, n: int) -> None:
    """``setMPIJobWorkerReplicas`` (scheduler.go:521-524)."""
    spec["spec"]["mpiReplicaSpecs"]["Worker"]["replicas"] = int(n)


def worker_replicas(spec: dict) -> int:
    return int(spec["spec"]["mpiReplicaSpecs"]["Worker"].get("replicas", 0))


def preprocess(spec: dict, gpu_type: str) -> None:
    """Force 1 GPU per worker and inject the accelerator label into the job, launcher and
    worker templates (``preprocessTrainingJob``, scheduler.go:891-914)."""
    ws = worker_template_spec(spec)
    c = ws["containers"][0]
    limits = c.setdefault("resources", {}).setdefault("limits", {})
    limits.pop("nvidia.com/gpu", None)
    limits[GPU_RESOURCE] = 1
    spec.setdefault("metadata", {}).setdefault("labels", {})[GPU_NAME_LABEL] = gpu_type
    spec["metadata"].setdefault("namespace", NAMESPACE)
    for role in ("Launcher", "Worker"):
        tmpl = spec["spec"]["mpiReplicaSpecs"][role]["template"]
        tmpl.setdefault("metadata", {}).setdefault("labels", {})[GPU_NAME_LABEL] = gpu_type


def _expand_env(tok: str, env: dict[str, str]) -> str:
    return re.sub(r"\$\((\w+)\)", lambda m: env.get(m.group(1), m.group(0)), tok)


_LAUNCHER_BINARIES = ("horovodrun", "vodarun", "mpirun", "torchrun")
_LAUNCHER_OPTS_WITH_ARG = {"--num-proc", "-np", "--min-num-proc", "--max-num-proc", "--host-discovery-script",
                           "--network-interface", "--slots-per-host", "--nproc-per-node", "--nnodes",
                           "-H", "--hosts", "--start-timeout", "--reset-limit"}


def worker_command(spec: dict) -> list[str]:
    """Extract the per-worker training command from the launcher container.

    The reference launcher runs ``horovodrun <opts> python train.py <args>`` through
    ``/bin/bash -c`` (examples/yaml/tensorflow2/*.yaml); the local backend runs one
    ``python train.py <args>`` per GPU itself, so everything up to the script is dropped
    and ``$(VAR)`` references are expanded from the launcher env.
    """
    c = spec["spec"]["mpiReplicaSpecs"]["Launcher"]["template"]["spec"]["containers"][0]
    env = {e["name"]: str(e.get("value", "")) for e in c.get("env", [])}
    parts: list[str] = []
    for p in list(c.get("command", [])) + list(c.get("args", [])):
        parts.append(p)
    text = " ".join(parts)
    # keep only the segment containing the launcher / python invocation
    segs = [s.strip() for s in re.split(r"[;&]{1,2}|\n", text) if s.strip()]
    seg = next((s for s in segs if any(b in s for b in _LAUNCHER_BINARIES) or "python" in s), None)
    if seg is None:
        raise ValueError("cannot find the training command in the launcher container")
    toks = [_expand_env(t, env) for t in shlex.split(seg)]
    if toks and toks[0] in ("/bin/bash", "bash", "sh", "/bin/sh"):
        toks = toks[2:] if len(toks) > 1 and toks[1] == "-c" else toks[1:]
    if toks and toks[0] in _LAUNCHER_BINARIES:
        i = 1
        while i < len(toks) and toks[i].startswith("-"):
            opt = toks[i]
            if opt == "--blacklist-cooldown-range":
                i += 3
            elif opt in _LAUNCHER_OPTS_WITH_ARG or ("=" not in opt and i + 1 < len(toks)
                                                     and not toks[i + 1].startswith("-")
                                                     and not toks[i + 1].startswith("python")):
                i += 2
            else:
                i += 1
        toks = toks[i:]
    if not toks:
        raise ValueError("empty training command")
    return toks


# ---- MPIJob status conditions (status.go:9-29) ----
def _has_condition(status: dict | None, ctype: str) -> bool:
    for c in (status or {}).get("conditions", []) or []:
        if c.get("type") == ctype and str(c.get("status")) == "True":
            return True
    return False


def is_succeeded(status: dict | None) -> bool:
    return _has_condition(status, "Succeeded")


def is_failed(status: dict | None) -> bool:
    return _has_condition(status, "Failed")


def is_finished(status: dict | None) -> bool:
    return is_succeeded(status) or is_failed(status)


def clone(spec: dict) -> dict:
    return copy.deepcopy(spec)
