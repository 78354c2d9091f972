"""vodascheduler_amd — MI355X-native elastic deep-learning scheduler and training runtime.

Capabilities of heyfey/vodascheduler (v0.2.2), re-designed for AMD Instinct MI355X:
scheduling policies (pkg/algorithm), Munkres placement (pkg/placement), the resource
allocator / scheduler / training services (pkg/allocator, pkg/scheduler, pkg/service),
the metrics collector (python/metrics_collector) and — what the reference delegated to
Horovod/NCCL inside user containers — an elastic data-parallel runtime on PyTorch-ROCm with
RCCL over xGMI and hand-written CDNA4 HIP kernels.
"""
__version__ = "0.3.0"
NAME = "vodascheduler_amd"

from .utils.miopen_db import configure as _configure_miopen  # noqa: E402

# before any process of ours runs a convolution: share MIOpen's find-db / kernel cache
if __import__("os").environ.get("VODA_MIOPEN_DIR", "") != "off":
    _configure_miopen()
