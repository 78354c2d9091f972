"""The committed driver-timeline prediction is priced at the measured step times (VERDICT r5
Next #4): the step times in profiles/r6/driver_timeline_prediction.md are the warm-up step
times of the bench JSON line it names, the simulator's fp32 profiles agree with them, and the
predicted N = 8 driver command ends before bench.py's 540 s deadline."""
import ast
import json
import os
import re

from vodascheduler_amd.common.workload import PROFILES_FP32

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PRED = os.path.join(ROOT, "profiles", "r6", "driver_timeline_prediction.md")


def _prediction():
    text = open(PRED).read()
    source = re.search(r"Step times source: `([^`]+)`", text).group(1)
    step_ms = ast.literal_eval(re.search(r"fp32 step times (\{[^}]*\}) ms", text).group(1))
    rows = {}
    for line in text.splitlines():
        cells = [c.strip() for c in line.strip().strip("|").split("|")]
        if cells and cells[0].isdigit():
            rows[int(cells[0])] = cells
    return source, step_ms, rows


def test_timeline_step_times_match_bench_warmup():
    source, step_ms, _ = _prediction()
    bench = json.load(open(os.path.join(ROOT, source)))
    bench = bench.get("line", bench)  # bench.py --out detail file
    assert bench["precision"] == "fp32" and bench["status"] == "ok"
    assert step_ms == bench["warmup_single_gpu_step_ms"]


def test_fp32_profiles_match_bench_warmup():
    """The simulator's default fp32 pricing (sim experiments, the bench's own control
    prediction before warm-up) is within 3 % of the same measured step times."""
    source, step_ms, _ = _prediction()
    for model, ms in step_ms.items():
        assert abs(PROFILES_FP32[model].step_time_1gpu * 1e3 - ms) / ms < 0.03, (model, ms)


def test_predicted_eight_gpu_command_ends_before_deadline():
    _, _, rows = _prediction()
    assert set(rows) == {1, 2, 4, 8}
    end_s = float(rows[8][9])
    assert end_s < 540.0, rows[8]
