"""Predicted timeline of the driver's ``bench.py --gpus N --steps 20 --warmup 5`` at N = 1, 2,
4, 8 against the 540 s deadline: warm-up, RCCL busbw sweep, timed main trace (FfDL) and the
FIFO control -- SIMULATED with the same simulator bench.py uses to decide whether the control
fits (sim/simulator.py), priced with measured fp32 single-GPU step times and an ASSUMED
all-reduce bus bandwidth (no multi-GPU box is available to this build).

    python benchmarks/predict_driver_timeline.py --step-ms resnet50=69.88,bert-base=37.12 \
        --out profiles/r5/driver_timeline_prediction.md
    python benchmarks/predict_driver_timeline.py --bench-json profiles/r6/bench_n1_fp32_r6a.json \
        --out profiles/r6/driver_timeline_prediction.md

``--bench-json`` takes the step times from a measured N = 1 bench line
(``warmup_single_gpu_step_ms``) and names that file in the output, so a CPU test
(tests/test_timeline_prediction_cpu.py) can check the prediction is priced at the measured times.
"""
from __future__ import annotations

import argparse
import copy
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import bench  # noqa: E402
from vodascheduler_amd.common.mpijob import set_name  # noqa: E402
from vodascheduler_amd.common.workload import set_measured_step_times  # noqa: E402
from vodascheduler_amd.sim.trace import ASSUMED_BUSBW_GBS  # noqa: E402


def timeline(n: int, step_ms: dict, steps: int, warmup_s: float, deadline: float, comm_init_s: float) -> dict:
    set_measured_step_times({m: {1: v} for m, v in step_ms.items()}, "fp32")
    trace = bench.bench_trace(32, steps * bench.STEP_SCALE["fp32"], n, 0, 2.0, bench.MODELS, bench.BATCH,
                              precision="fp32", step_time_s={m: v / 1e3 for m, v in step_ms.items()})
    ctl = []
    for tj in trace:
        spec = copy.deepcopy(tj.spec)
        set_name(spec, "ctl-" + spec["metadata"]["name"])
        ctl.append(type(tj)(tj.submit_time, spec))
    main_wall, main_jct = bench.predict(trace, "FfDLOptimizer", n, bench.RATE_LIMIT_S)
    ctl_wall, ctl_jct = bench.predict(ctl, "FIFO", n, bench.RATE_LIMIT_S)
    # busbw sweep: one communicator build per power-of-two sub-world + 3 sizes x 7 all-reduces
    ks = [k for k in (2, 4, 8) if k <= n]
    sweep = sum(comm_init_s + 7 * (16 + 64 + 256) * 2**20 * 4 / 4 / (ASSUMED_BUSBW_GBS * 1e9) for _ in ks)
    t_main_end = warmup_s + sweep + main_wall
    left = deadline - t_main_end
    need = ctl_wall * 1.15 + 20  # bench.py's skip rule with calibration 1
    return {"n": n, "warmup_s": warmup_s, "busbw_sweep_s": round(sweep, 1), "main_wall_s": round(main_wall, 1),
            "main_avg_jct_s": round(main_jct, 2), "main_end_s": round(t_main_end, 1),
            "control_wall_s": round(ctl_wall, 1), "control_avg_jct_s": round(ctl_jct, 2),
            "control_runs": left >= need, "end_s": round(t_main_end + (ctl_wall if left >= need else 0), 1),
            "predicted_vs_baseline": round(ctl_jct / main_jct, 3)}


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("--step-ms", default="resnet50=69.88,bert-base=37.12",
                    help="measured fp32 single-GPU step ms (default: BENCH_r04 warm-up)")
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup-s", type=float, default=45.0,
                    help="warm-up wall before the timed trace (BENCH_r05: 296.3 s command - 127.0 main - 127.0 "
                         "control = 42.3 s, rounded up)")
    ap.add_argument("--comm-init-s", type=float, default=3.0, help="ASSUMED RCCL communicator build time")
    ap.add_argument("--deadline", type=float, default=540.0)
    ap.add_argument("--out", default=None)
    ap.add_argument("--bench-json", default=None,
                    help="measured bench.py JSON line: its warmup_single_gpu_step_ms replace --step-ms")
    a = ap.parse_args()
    step_ms = {k: float(v) for k, v in (kv.split("=") for kv in a.step_ms.split(","))}
    source = "--step-ms"
    if a.bench_json:
        with open(a.bench_json) as f:
            d = json.load(f)
        d = d.get("line", d)  # bench.py --out detail file: the printed line is under "line"
        step_ms = {k: float(v) for k, v in d["warmup_single_gpu_step_ms"].items()}
        source = a.bench_json
    rows = [timeline(n, step_ms, a.steps, a.warmup_s, a.deadline, a.comm_init_s) for n in (1, 2, 4, 8)]
    lines = [
        "# Predicted driver timeline (`bench.py --gpus N --steps 20 --warmup 5`, fp32)",
        "",
        f"Step times source: `{source}`",
        "",
        f"SIMULATED (sim/simulator.py, the predictor bench.py itself uses), priced with fp32 step times {step_ms} ms "
        f"and an ASSUMED {ASSUMED_BUSBW_GBS:g} GB/s all-reduce busbw; warm-up {a.warmup_s:g} s and "
        f"{a.comm_init_s:g} s per RCCL communicator build are ASSUMED.  Deadline {a.deadline:g} s.  When the "
        "control does not fit, bench.py skips it and reports `control.predicted_avg_jct_s` (labelled simulated).",
        "",
        "| N | warm-up s | busbw sweep s | main wall s | main ends at s | main avg JCT s | FIFO control wall s "
        "| control avg JCT s | control runs? | command ends at s | predicted vs_baseline |",
        "|---:|---:|---:|---:|---:|---:|---:|---:|---|---:|---:|",
    ]
    for r in rows:
        lines.append(f"| {r['n']} | {r['warmup_s']:g} | {r['busbw_sweep_s']} | {r['main_wall_s']} | {r['main_end_s']} "
                     f"| {r['main_avg_jct_s']} | {r['control_wall_s']} | {r['control_avg_jct_s']} "
                     f"| {'yes' if r['control_runs'] else 'no (skipped: predicted in JSON)'} | {r['end_s']} "
                     f"| {r['predicted_vs_baseline']} |")
    text = "\n".join(lines) + "\n"
    print(text)
    if a.out:
        os.makedirs(os.path.dirname(a.out), exist_ok=True)
        with open(a.out, "w") as f:
            f.write(text)


if __name__ == "__main__":
    main()
