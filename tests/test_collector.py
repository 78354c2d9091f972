"""Metrics collector (CSV rows -> job_info, reference python/metrics_collector/
metrics_collector.py:15-184) and the rocm-smi GPU exporter (the reference's external
nvidia_smi_exporter, README.md:94).  The CSVs are written by the workloads' own
MetricsCSVLogger, so the producer/consumer contract is tested end to end; the rocm-smi JSON
is a synthetic document in the rocm-smi 3.x key format (no GPU needed)."""
import json
import os
import time

import pytest

from vodascheduler_amd.collector.collector import MetricsCollector, category_of, fit_amdahl, speedup_table
from vodascheduler_amd.collector.gpu_exporter import GpuExporter, parse_rocm_smi_json
from vodascheduler_amd.common.store import MemoryStore
from vodascheduler_amd.common.trainingjob import create_base_job_info_record, init_job_info_record
from vodascheduler_amd.workloads.metrics_logger import MetricsCSVLogger


def test_category_strips_timestamp_suffix():
    assert category_of("resnet50-20261016-031502") == "resnet50"
    assert category_of("bert-base-j03-20261016-100751") == "bert-base-j03"
    assert category_of("plain") == "plain"


def test_speedup_table_measured_points_and_amdahl_fill():
    # measured 1, 2, 4 workers with serial fraction 0.1: s(k) = k / (1 + 0.1 (k - 1))
    amdahl = lambda k: k / (1 + 0.1 * (k - 1))  # noqa: E731
    t = {k: 100.0 / amdahl(k) for k in (1, 2, 4)}
    assert fit_amdahl({k: amdahl(k) for k in (2, 4)}) == pytest.approx(0.1)
    sp = speedup_table(t, max_gpu=8)
    assert sp["0"] == 0.0 and sp["1"] == pytest.approx(1.0)
    assert sp["4"] == pytest.approx(amdahl(4))
    assert sp["8"] == pytest.approx(amdahl(8))          # unmeasured: interpolated
    assert len(sp) == 10                                  # 0 .. max_gpu + 1
    vals = [sp[str(k)] for k in range(1, 10)]
    assert vals == sorted(vals)                           # monotone, saturating


def test_speedup_table_without_single_worker_measurement():
    # only 2 and 4 workers measured: t(1) inferred linearly below 2 (no 1-second placeholder)
    sp = speedup_table({2: 50.0, 4: 30.0}, max_gpu=4)
    assert sp["2"] == pytest.approx(2.0)
    assert sp["4"] == pytest.approx(100.0 / 30.0)


def _job(store, job, epochs):
    cat = category_of(job)
    try:
        base = store.find_job_info(cat, cat)
    except KeyError:
        base = create_base_job_info_record(cat)
        store.insert_job_info(cat, base)
    store.insert_job_info(cat, init_job_info_record(base, job, epochs))
    return cat


def test_collector_updates_job_and_category_history(tmp_path):
    store = MemoryStore()
    job = "resnet50-20261016-031502"
    cat = _job(store, job, epochs=10)
    lg = MetricsCSVLogger(str(tmp_path), job, total_epochs=10, local_batch_size=128)
    t0 = time.time()
    # epochs 0-1 on 1 worker (20 s), 2-3 on 2 workers (11 s), 4 on 4 workers (6.5 s); an epoch
    # is split over the workers (steps_per_epoch // size, tensorflow2_keras_cifar_elastic.py:223)
    for e, (w, et) in enumerate([(1, 20.0), (1, 20.0), (2, 11.0), (2, 11.0), (4, 6.5)]):
        lg.log_epoch(e, t0 + 30 * e, et, steps=100 // w, loss=1.0 / (e + 1), workers=w)
    assert lg.restored_epoch() == 5                       # a preempted job resumes at epoch 5
    c = MetricsCollector(store, str(tmp_path))
    assert c.jobs() == [job]
    assert c.update_info_all() == 1
    info = store.find_job_info(cat, job)
    assert info["current_epoch"] == 4 and info["remainning_epochs"] == 5
    assert info["speedup"]["2"] == pytest.approx(20.0 / 11.0)
    assert info["speedup"]["4"] == pytest.approx(20.0 / 6.5)
    assert info["efficiency"]["4"] == pytest.approx(20.0 / 6.5 / 4)
    assert info["step_time_sec"]["1"] == pytest.approx(0.2)
    assert info["estimated_remainning_time_sec"] == pytest.approx(20.0 * 5)
    assert info["gpu_time_sec"] == pytest.approx(2 * 20 + 2 * 2 * 11 + 4 * 6.5)
    assert info["running_time_sec"] == pytest.approx(2 * 20 + 2 * 11 + 6.5)
    # the category's base record learns the measured curve, so the next
    # job of this category starts from it instead of the linear default
    base = store.find_job_info(cat, cat)
    assert base["speedup"]["4"] == pytest.approx(20.0 / 6.5)
    nxt = "resnet50-20261016-041000"
    _job(store, nxt, epochs=3)
    assert store.find_job_info(cat, nxt)["estimated_remainning_time_sec"] == pytest.approx(3 * 20.0)
    # unchanged CSV: nothing to do
    assert c.update_info_all([job]) == 0


def test_collector_skips_unknown_and_empty(tmp_path):
    store = MemoryStore()
    (tmp_path / "ghost-20261016-031502.csv").write_text("")
    c = MetricsCollector(store, str(tmp_path))
    assert c.update_info_all() == 0
    assert MetricsCollector(store, str(tmp_path / "missing")).jobs() == []


ROCM_SMI = {
    "card0": {"GPU use (%)": "87", "Current Socket Graphics Package Power (W)": "912.0",
              "Temperature (Sensor junction) (C)": "71.0", "Temperature (Sensor edge) (C)": "50.0",
              "VRAM Total Memory (B)": "309220868096", "VRAM Total Used Memory (B)": "103079215104"},
    "card1": {"GPU use (%)": "0", "Average Graphics Package Power (W)": "140.0",
              "Temperature (Sensor junction) (C)": "40.0",
              "VRAM Total Memory (B)": "309220868096", "VRAM Total Used Memory (B)": "283115520"},
    "system": {"Driver version": "6.12"},
}


def test_parse_rocm_smi_json():
    g = parse_rocm_smi_json(json.dumps(ROCM_SMI))
    assert sorted(g) == [0, 1]
    assert g[0] == {"utilization_percent": 87.0, "power_watts": 912.0, "temperature_celsius": 71.0,
                    "memory_total_bytes": 309220868096.0, "memory_used_bytes": 103079215104.0}
    assert g[1]["power_watts"] == 140.0 and g[1]["utilization_percent"] == 0.0


def test_gpu_exporter_exposition_names():
    exp = GpuExporter(query=lambda: parse_rocm_smi_json(json.dumps(ROCM_SMI)), query_xgmi=None)
    text = exp.exposition().decode()
    for f in GpuExporter.FIELDS:
        assert f"voda_scheduler_gpu_{f}" in text
    assert 'voda_scheduler_gpu_utilization_percent{gpu="0"} 87.0' in text
    assert 'voda_scheduler_gpu_memory_total_bytes{gpu="1"} 3.09220868096e+11' in text


FIXTURES = os.path.join(os.path.dirname(__file__), "fixtures")


def test_parse_rocm_smi_json_captured_on_mi355x():
    with open(os.path.join(FIXTURES, "mi355x_rocm_smi_1gpu_box.json")) as f:
        g = parse_rocm_smi_json(f.read())
    assert g[0]["memory_total_bytes"] == 309220868096.0  # 288 GiB HBM3E
    assert g[0]["power_watts"] == 268.0 and g[0]["temperature_celsius"] == 48.0


def test_parse_amdsmi_xgmi_captured_on_mi355x():
    from vodascheduler_amd.collector.gpu_exporter import parse_amdsmi_xgmi_json

    with open(os.path.join(FIXTURES, "mi355x_amdsmi_xgmi_1gpu_box.json")) as f:
        x = parse_amdsmi_xgmi_json(f.read())
    assert x[0]["bit_rate_gbps"] == 38.0 and x[0]["max_bandwidth_gbps"] == 608.0
    # 8 ports: the one facing the GPU itself ("X") is not a link, the other 7 are up
    assert x[0]["ports"] == {p: 1 for p in range(1, 8)}
    assert x[0]["read_bytes"] == {} and x[0]["write_bytes"] == {}  # "N/A" in a 1-GPU container


def test_xgmi_numeric_link_counters_and_gauges():
    from vodascheduler_amd.collector.gpu_exporter import parse_amdsmi_xgmi_json

    doc = {"xgmi_metric": [[{"gpu": 1, "link_metrics": {
        "bit_rate": {"value": 38, "unit": "Gb/s"}, "max_bandwidth": {"value": 608, "unit": "Gb/s"},
        "links": [{"gpu": 0, "read": {"value": 12, "unit": "KB"}, "write": {"value": 3, "unit": "MB"}},
                  {"gpu": 2, "read": 7, "write": "N/A"}]}}]],
        "link_port_status": [{"gpu": 1, "link_status": ["U", "X", "D"]}]}
    x = parse_amdsmi_xgmi_json(json.dumps(doc))
    assert x[1]["read_bytes"] == {0: 12e3, 2: 7.0} and x[1]["write_bytes"] == {0: 3e6}
    assert x[1]["ports"] == {0: 1, 2: 0}
    exp = GpuExporter(query=lambda: {}, query_xgmi=lambda: x)
    text = exp.exposition().decode()
    assert 'voda_scheduler_gpu_xgmi_max_bandwidth_gbps{gpu="1"} 608.0' in text
    assert 'voda_scheduler_gpu_xgmi_link_up{gpu="1",port="2"} 0.0' in text
    assert 'voda_scheduler_gpu_xgmi_read_bytes{gpu="1",peer="0"} 12000.0' in text


def test_prior_gives_curve_shape_not_absolute_time():
    """a job measured only at world 2 whose prior is for another precision
    (bf16 t1 23 ms vs an fp32 step of ~77 ms) must not get speedup(2) = 2 x 23 / 80 < 1 --
    the prior's curve supplies s(2), the measurement the absolute time."""
    from vodascheduler_amd.collector.collector import estimate_tables
    from vodascheduler_amd.common.workload import PROFILES, prior_fields

    prior = prior_fields({"model": "resnet50", "steps_per_epoch": 100}, 1)   # bf16 prior: t1 = 23 ms
    t2 = 0.080                                                                 # fp32, measured at world 2
    sp, st = estimate_tables({2: t2}, prior)
    s2_prior = PROFILES["resnet50"].speedup(2)
    assert sp["2"] == pytest.approx(2 * (t2 * s2_prior / 2) / t2)            # = the prior's s(2)
    assert st["1"] == pytest.approx(t2 * s2_prior / 2)                         # fp32-scale t1, ~77-80 ms
    assert 0.07 < st["1"] < 0.09 and all(sp[str(k)] >= 1.0 for k in range(1, 9))
    # without any prior: linear below the smallest measured count (unchanged)
    sp0, st0 = estimate_tables({2: t2}, None)
    assert sp0["2"] == pytest.approx(2.0) and st0["1"] == pytest.approx(t2)
