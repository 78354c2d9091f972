"""GPU telemetry exporter (the external nvidia_smi_exporter of the reference, README.md:94,
re-done for AMD Instinct): utilisation, power, temperature, HBM used/total per GPU via
``rocm-smi --json``, exported as Prometheus gauges
``voda_scheduler_gpu_{utilization_percent,power_watts,temperature_celsius,memory_used_bytes,
memory_total_bytes}{gpu="N"}``; the xGMI fabric via ``amd-smi xgmi --json``:
``voda_scheduler_gpu_xgmi_{bit_rate_gbps,max_bandwidth_gbps}{gpu}``,
``voda_scheduler_gpu_xgmi_link_up{gpu,port}`` and, where the driver reports them,
``voda_scheduler_gpu_xgmi_{read,write}_bytes{gpu,peer}`` (cumulative per-peer link traffic --
the data-parallel all-reduce traffic of the jobs placed on the node); also the
schedulable-GPU discovery for the local backend.
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


_UNIT_BYTES = {"b": 1, "kb": 1e3, "mb": 1e6, "gb": 1e9, "tb": 1e12, "kib": 1024, "mib": 2 ** 20, "gib": 2 ** 30}


def _bytes(v) -> float | None:
    """amd-smi link counters: ``{"value": N, "unit": "KB"}``, a bare number, or "N/A"."""
    if isinstance(v, dict):
        n = _num(v.get("value"))
        if n is None:
            return None
        return n * _UNIT_BYTES.get(str(v.get("unit", "B")).strip().lower(), 1)
    return _num(v) if not (isinstance(v, str) and "n/a" in v.lower()) else None


def parse_amdsmi_xgmi_json(text: str) -> dict[int, dict]:
    """Parse ``amd-smi xgmi --json`` (tests/fixtures/mi355x_amdsmi_xgmi_1gpu_box.json, captured
    on an MI355X box: 8 xGMI ports per GPU, bit rate 38 Gb/s, 608 Gb/s max bandwidth).

    Returns {gpu: {"bit_rate_gbps", "max_bandwidth_gbps", "ports": {port: up}, "read_bytes":
    {peer: B}, "write_bytes": {peer: B}}}.  Per-peer read/write counters read "N/A" inside a
    one-GPU container; their numeric form (value + unit) is handled but not pinned by a
    captured fixture."""
    data = json.loads(text)
    out: dict[int, dict] = {}
    metrics = data.get("xgmi_metric", [])
    for group in metrics:
        for ent in group if isinstance(group, list) else [group]:
            g = out.setdefault(int(ent.get("gpu", 0)), {"ports": {}, "read_bytes": {}, "write_bytes": {}})
            lm = ent.get("link_metrics", {})
            br, mb = lm.get("bit_rate", {}), lm.get("max_bandwidth", {})
            if _num(br.get("value") if isinstance(br, dict) else br) is not None:
                g["bit_rate_gbps"] = _num(br.get("value") if isinstance(br, dict) else br)
            if _num(mb.get("value") if isinstance(mb, dict) else mb) is not None:
                g["max_bandwidth_gbps"] = _num(mb.get("value") if isinstance(mb, dict) else mb)
            for ln in lm.get("links", []) or []:
                peer = int(ln.get("gpu", -1))
                for key, dst in (("read", "read_bytes"), ("write", "write_bytes")):
                    b = _bytes(ln.get(key))
                    if b is not None:
                        g[dst][peer] = b
    for ent in data.get("link_port_status", []) or []:
        g = out.setdefault(int(ent.get("gpu", 0)), {"ports": {}, "read_bytes": {}, "write_bytes": {}})
        for port, st in enumerate(ent.get("link_status", []) or []):
            st = str(st).upper()
            if st in ("U", "UP"):
                g["ports"][port] = 1
            elif st in ("D", "DOWN"):
                g["ports"][port] = 0  # "X" = the port facing this GPU itself: not a link
    return out


def query_xgmi(timeout: float = 10.0) -> dict[int, dict]:
    exe = shutil.which("amd-smi") or "/opt/rocm/bin/amd-smi"
    try:
        r = subprocess.run([exe, "xgmi", "--json"], capture_output=True, text=True, timeout=timeout)
    except (OSError, subprocess.TimeoutExpired) as e:
        log.warning("amd-smi unavailable: %s", e)
        return {}
    txt = r.stdout[r.stdout.find("{"):] if "{" in r.stdout else ""
    if r.returncode != 0 or not txt:
        return {}
    try:
        return parse_amdsmi_xgmi_json(txt)
    except (ValueError, json.JSONDecodeError, TypeError, AttributeError):
        return {}


def query_gpus(timeout: float = 10.0) -> dict[int, dict[str, float]]:
    exe = shutil.which("rocm-smi") or "/opt/rocm/bin/rocm-smi"
    try:
        r = subprocess.run([exe, "--showuse", "--showpower", "--showtemp", "--showmeminfo", "vram", "--json"],
                           capture_output=True, text=True, timeout=timeout)
    except (OSError, subprocess.TimeoutExpired) as e:
        log.warning("rocm-smi unavailable: %s", e)
        return {}
    # rocm-smi may print a warning line before the JSON (e.g. "... low-power state ...")
    txt = r.stdout[r.stdout.find("{"):] if "{" in r.stdout else ""
    if r.returncode != 0 or not txt:
        return {}
    try:
        return parse_rocm_smi_json(txt)
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
    XGMI_FIELDS = ("bit_rate_gbps", "max_bandwidth_gbps")

    def __init__(self, query=query_gpus, query_xgmi=query_xgmi):
        self.registry = CollectorRegistry()
        self.query = query
        self.query_xgmi = query_xgmi
        self.gauges = {f: Gauge(f"voda_scheduler_gpu_{f}", f"AMD GPU {f.replace('_', ' ')}", ["gpu"],
                                registry=self.registry) for f in self.FIELDS}
        self.xgmi = {f: Gauge(f"voda_scheduler_gpu_xgmi_{f}", f"xGMI {f.replace('_', ' ')}", ["gpu"],
                              registry=self.registry) for f in self.XGMI_FIELDS}
        self.xgmi_up = Gauge("voda_scheduler_gpu_xgmi_link_up", "xGMI port up (1) / down (0)", ["gpu", "port"],
                             registry=self.registry)
        self.xgmi_bytes = {d: Gauge(f"voda_scheduler_gpu_xgmi_{d}_bytes", f"xGMI bytes {d} per peer (cumulative)",
                                    ["gpu", "peer"], registry=self.registry) for d in ("read", "write")}

    def refresh(self) -> dict[int, dict[str, float]]:
        data = self.query()
        for gpu, vals in data.items():
            for f, v in vals.items():
                if f in self.gauges:
                    self.gauges[f].labels(str(gpu)).set(v)
        if self.query_xgmi is not None:
            for gpu, x in self.query_xgmi().items():
                for f in self.XGMI_FIELDS:
                    if f in x:
                        self.xgmi[f].labels(str(gpu)).set(x[f])
                for port, up in x.get("ports", {}).items():
                    self.xgmi_up.labels(str(gpu), str(port)).set(up)
                for d in ("read", "write"):
                    for peer, b in x.get(f"{d}_bytes", {}).items():
                        self.xgmi_bytes[d].labels(str(gpu), str(peer)).set(b)
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
