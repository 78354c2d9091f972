"""Metrics collector (CSV -> job_info speedup / remaining-time estimates) and the AMD GPU
telemetry exporter."""
from .collector import MetricsCollector, category_of, fit_amdahl, speedup_table
from .gpu_exporter import GpuExporter, discover_gpus, parse_rocm_smi_json, query_gpus

__all__ = ["MetricsCollector", "category_of", "fit_amdahl", "speedup_table", "GpuExporter", "discover_gpus",
           "parse_rocm_smi_json", "query_gpus"]
