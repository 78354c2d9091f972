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
