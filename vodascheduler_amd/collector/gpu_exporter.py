"""GPU telemetry exporter (the external nvidia_smi_exporter of the reference, README.md:94,
re-done for AMD Instinct): utilisation, power, temperature, HBM used/total per GPU via
``rocm-smi --json`` (or ``amd-smi``), exported as Prometheus gauges
``voda_scheduler_gpu_{utilization_percent,power_watts,temperature_celsius,memory_used_bytes,
memory_total_bytes}{gpu="N"}``; also the schedulable-GPU discovery for the local backend.
"""
from __future__ import annotations

import json
import logging
import re
import shutil
import subprocess

from prometheus_client import CollectorRegistry, Gauge, generate_latest

log = logging.getLogger("vodascheduler_amd.gpu_exporter")


def _num(v) -> float | None:
    if v is None:
        return None
    m = re.search(r"[-+]?\d+(\.\d+)?", str(v))
    return float(m.group(0)) if m else None


def parse_rocm_smi_json(text: str) -> dict[int, dict[str, float]]:
    """Parse ``rocm-smi --showuse --showpower --showtemp --showmeminfo vram --json``."""
    data = json.loads(text)
    out: dict[int, dict[str, float]] = {}
    for card, d in data.items():
        m = re.match(r"card(\d+)", card)
        if not m or not isinstance(d, dict):
            continue
        g: dict[str, float] = {}
        for k, v in d.items():
            kl = k.lower()
            if "gpu use" in kl:
                g["utilization_percent"] = _num(v)
            elif "power" in kl and ("average" in kl or "current socket" in kl or "socket graphics" in kl):
                g["power_watts"] = _num(v)
            elif "temperature" in kl and ("junction" in kl or "hotspot" in kl or "edge" in kl):
                g.setdefault("temperature_celsius", _num(v))
            elif "vram total used" in kl:
                g["memory_used_bytes"] = _num(v)
            elif "vram total memory" in kl:
                g["memory_total_bytes"] = _num(v)
        out[int(m.group(1))] = {k: v for k, v in g.items() if v is not None}
    return out


def query_gpus(timeout: float = 10.0) -> dict[int, dict[str, float]]:
    exe = shutil.which("rocm-smi") or "/opt/rocm/bin/rocm-smi"
    try:
        r = subprocess.run([exe, "--showuse", "--showpower", "--showtemp", "--showmeminfo", "vram", "--json"],
                           capture_output=True, text=True, timeout=timeout)
    except (OSError, subprocess.TimeoutExpired) as e:
        log.warning("rocm-smi unavailable: %s", e)
        return {}
    if r.returncode != 0 or not r.stdout.strip().startswith("{"):
        return {}
    try:
        return parse_rocm_smi_json(r.stdout)
    except (ValueError, json.JSONDecodeError):
        return {}


def discover_gpus() -> list[int]:
    """Schedulable GPU indices on this node (HIP_VISIBLE_DEVICES honoured)."""
    import os

    vis = os.environ.get("HIP_VISIBLE_DEVICES") or os.environ.get("ROCR_VISIBLE_DEVICES")
    if vis:
        return [int(x) for x in vis.split(",") if x.strip() != ""]
    try:
        import torch

        return list(range(torch.cuda.device_count()))
    except Exception:
        return sorted(query_gpus())


class GpuExporter:
    FIELDS = ("utilization_percent", "power_watts", "temperature_celsius", "memory_used_bytes", "memory_total_bytes")

    def __init__(self, query=query_gpus):
        self.registry = CollectorRegistry()
        self.query = query
        self.gauges = {f: Gauge(f"voda_scheduler_gpu_{f}", f"AMD GPU {f.replace('_', ' ')}", ["gpu"],
                                registry=self.registry) for f in self.FIELDS}

    def refresh(self) -> dict[int, dict[str, float]]:
        data = self.query()
        for gpu, vals in data.items():
            for f, v in vals.items():
                if f in self.gauges:
                    self.gauges[f].labels(str(gpu)).set(v)
        return data

    def exposition(self) -> bytes:
        self.refresh()
        return generate_latest(self.registry)


def main(argv=None) -> int:
    """Serve ``GET /metrics`` with rocm-smi telemetry (the reference relies on an external
    nvidia_smi_exporter, README.md:94)."""
    import argparse
    import logging

    from ..utils.http import HttpServer, Router

    ap = argparse.ArgumentParser("vodascheduler-gpu-exporter")
    ap.add_argument("--port", type=int, default=9400)
    a = ap.parse_args(argv)
    logging.basicConfig(level=logging.INFO)
    exp = GpuExporter()
    r = Router()
    r.add("GET", "/metrics", lambda b, q: (200, "text/plain; version=0.0.4", exp.exposition()))
    srv = HttpServer(r, port=a.port, name="gpu-exporter")
    logging.info("rocm-smi exporter on :%d", srv.port)
    srv.serve_forever()
    return 0


if __name__ == "__main__":
    raise SystemExit(main())
