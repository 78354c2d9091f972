"""benchmarks/experiments.py prices the BASELINE configs at the precision the driver's bench
trains at (VERDICT r4 Next #6): with ``--precision fp32`` every job declares fp32 and the
simulator prices it with the measured fp32 profile (common/workload.PROFILES_FP32)."""
import os
import sys

import pytest

from vodascheduler_amd.common.workload import PROFILES, PROFILES_FP32, profile_of
from vodascheduler_amd.sim.trace import philly_trace, workload_of

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "benchmarks"))


def test_philly_trace_declares_precision_and_keeps_step_counts():
    bf = philly_trace(8, seed=1, models=("resnet50", "bert-base"))
    fp = philly_trace(8, seed=1, models=("resnet50", "bert-base"), precision="fp32")
    for a, b in zip(bf, fp):
        wa, wb = workload_of(a.spec), workload_of(b.spec)
        assert wb["precision"] == "fp32" and wa.get("precision", "bf16") == "bf16"
        assert wa["steps_per_epoch"] == wb["steps_per_epoch"]       # same work ...
        assert profile_of(wb) is PROFILES_FP32[wb["model"]]          # ... priced at fp32
        assert profile_of(wa) is PROFILES[wa["model"]]


def test_experiments_fp32_uses_fp32_profile():
    import experiments

    old = experiments.PREC
    try:
        experiments.PREC = "bf16"
        bf = {r.algorithm: r.avg_jct for r in experiments.exp2()}
        experiments.PREC = "fp32"
        fp = {r.algorithm: r.avg_jct for r in experiments.exp2()}
    finally:
        experiments.PREC = old
    ratio = PROFILES_FP32["resnet50"].step_time_1gpu / PROFILES["resnet50"].step_time_1gpu
    assert ratio > 2.5
    for a in bf:  # the same 8 ResNet-50 jobs take ~ratio x longer at fp32
        assert fp[a] > 2.0 * bf[a], (a, fp[a], bf[a])
