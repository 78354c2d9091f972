"""The BASELINE.json experiment configs, run in the discrete-event simulator (the real
scheduler + allocator + placement code in virtual time).  Job speed
curves come from the MI355X-calibrated ``sim.trace.PROFILES``.

  1. Elastic-FIFO, 2 toy MNIST jobs, 2 slots   -> real CPU/gloo run: tests/test_elastic_cpu.py
  2. Elastic-Tiresias, 8 ResNet-50 ImageNet-shape jobs on 8 GPUs (vs Tiresias)
  3. AFS-L, mixed ResNet-50 + BERT-base trace on 8 GPUs (vs FIFO / ElasticFIFO)
  4. Munkres placement + worker migration under GPU drain (2 nodes x 8 GPUs)
  5. FfDL Optimizer, 32-job Philly-style trace, 1/2/4/8 GPUs (all 8 policies side by side),
     and with autoscale: capacity ramping 1 -> 2 -> 4 -> 8 GPUs during the trace

python benchmarks/experiments.py [--precision fp32] [--out profiles/r6_sim_experiments.md] [--bench-json SCALE.json]

``--precision`` (default fp32, the reference's and the driver bench's precision) is declared by
every job of every trace: the same steps are priced at that precision's measured step time
(``common.workload.PROFILES_FP32``; models without an fp32 measurement keep the bf16 one).

Job info (what SRJF / E-Tiresias / FfDL / AFS-L see) follows the real pipeline by default
(``info_mode="online"``): the training service seeds every job from the workload it declares
(common/workload.py), the collector refreshes running jobs every 60 s (the reference cron).
The ablation table re-runs the info-driven policies with the reference's placeholder info
(1 s epochs, linear speedup) and with an oracle.
"""
from __future__ import annotations

import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from vodascheduler_amd.algorithm import ALGORITHMS  # noqa: E402
from vodascheduler_amd.sim.simulator import simulate  # noqa: E402
from vodascheduler_amd.common.workload import (busbw_source, intra_node_busbw, load_bench_json,  # noqa: E402
                                               model_profile)
from vodascheduler_amd.sim.trace import (ASSUMED_BUSBW_GBS, ASSUMED_INTERNODE_BUSBW_GBS, TraceJob,  # noqa: E402
                                         make_spec, philly_trace)

ORDER = ["FIFO", "ElasticFIFO", "SRJF", "ElasticSRJF", "Tiresias", "ElasticTiresias", "FfDLOptimizer", "AFS-L"]


def row(r) -> str:
    return (f"| {r.algorithm} | {r.gpus} | {r.avg_jct:.0f} | {r.median_jct:.0f} | {r.p95_jct:.0f} | {r.makespan:.0f} "
            f"| {r.avg_wait:.0f} | {100 * r.utilization:.0f} % | {r.resizes} | {r.migrations} |")


HEADER = ("| policy | GPUs | avg JCT (s) | median JCT | p95 JCT | makespan (s) | avg wait | utilization | resizes "
          "| migrations |\n|---|---:|---:|---:|---:|---:|---:|---:|---:|---:|")


PREC = "fp32"  # compute precision every job declares (main: --precision)


def exp2():
    tr = [TraceJob(60.0 * i, make_spec(f"resnet50-{i}", "resnet50", 4, 1, 8, 10, 2000, category="resnet50",
                                       precision=PREC))
          for i in range(8)]
    return [simulate(tr, a, gpus=8) for a in ("Tiresias", "ElasticTiresias")]


def exp3():
    tr = philly_trace(32, seed=3, models=("resnet50", "bert-base"), precision=PREC)
    return [simulate(tr, a, gpus=8) for a in ("FIFO", "ElasticFIFO", "AFS-L")]


def exp4():
    tr = philly_trace(24, seed=4, mean_interarrival_s=20.0, precision=PREC)
    nodes = {"node0": list(range(8)), "node1": list(range(8))}
    drains = [(300.0, "node0", 2), (600.0, "node1", 5), (900.0, "node0", 6)]
    out = []
    for name, kw in (("Munkres + best-fit", {}), ("best-fit, migration-naive binding", {"naive_placement": True})):
        r = simulate(tr, "ElasticFIFO", nodes=nodes, drain=drains, **kw)
        out.append((name, r))
    return out


def exp5():
    out = []
    for g in (1, 2, 4, 8):
        # requests capped at the cluster size (a non-elastic 8-GPU job can never start on 4 GPUs)
        tr32 = philly_trace(32, seed=0, max_gpus=g, precision=PREC)
        for a in ORDER:
            out.append(simulate(tr32, a, gpus=g))
    return out


RAMP_T = 600.0  # seconds between capacity doublings of the autoscale ramp


def exp_autoscale():
    """BASELINE config 5's "autoscale 1->8": the config-5 trace while the cluster grows 1 -> 2 ->
    4 -> 8 GPUs (one doubling every RAMP_T s -- an autoscaler adding nodes), next to a fixed
    8-GPU cluster.  Node addition: reference scheduler.go:689-747, placement_manager.go:239-304."""
    tr = philly_trace(32, seed=0, max_gpus=8, precision=PREC)
    ramp = [(0.0, {"node0": [0]}), (RAMP_T, {"node0": [0, 1]}), (2 * RAMP_T, {"node0": list(range(4))}),
            (3 * RAMP_T, {"node0": list(range(8))})]
    out = []
    for a in ORDER:
        out.append((a, simulate(tr, a, gpus=8, capacity=ramp), simulate(tr, a, gpus=8)))
    return out


INFO_ALGOS = ["SRJF", "ElasticSRJF", "ElasticTiresias", "FfDLOptimizer", "AFS-L"]


def exp_info():
    """Info-source ablation on config 5's trace at 1 and 8 GPUs: the reference's placeholder
    info, the real pipeline (default), an oracle."""
    out = []
    for g in (1, 8):
        tr = philly_trace(32, seed=0, max_gpus=g, precision=PREC)
        fifo = simulate(tr, "FIFO", gpus=g).avg_jct
        for a in INFO_ALGOS:
            row = {"gpus": g, "algorithm": a, "fifo": fifo}
            for mode in ("mixed", "placeholder", "online", "oracle"):
                row[mode] = simulate(tr, a, gpus=g, info_mode=mode).avg_jct
            out.append(row)
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--out", default="profiles/r6_sim_experiments.md")
    ap.add_argument("--precision", default="fp32", choices=["fp32", "bf16"],
                    help="compute precision every job declares (prices its steps)")
    ap.add_argument("--bench-json", default=None,
                    help="bench.py --out / driver SCALE json with allreduce_busbw_gbs: measured busbw")
    a = ap.parse_args()
    global PREC
    PREC = a.precision
    assert set(ORDER) == set(ALGORITHMS)
    if a.bench_json:
        print("measured (busbw GB/s by world, step ms by model/world):", load_bench_json(a.bench_json))
    bw = (f"MEASURED per world ({', '.join(f'{k}: {intra_node_busbw(k):.0f}' for k in (2, 4, 8))} GB/s)"
          if busbw_source() == "measured" else f"ASSUMED ({ASSUMED_BUSBW_GBS:.0f} GB/s intra-node)")
    rn, bb = model_profile("resnet50", PREC), model_profile("bert-base", PREC)
    what = ("fp32 compute, the reference's precision and the driver bench's" if PREC == "fp32"
            else "bf16 autocast compute, fp32 gradients")
    lines = [f"# BASELINE.json configs in the discrete-event simulator (round 6, {PREC})", "",
             "Real training service / scheduler / allocator / placement code driven in virtual time "
             f"(`benchmarks/experiments.py --precision {PREC}`). Job speed model (`vodascheduler_amd/common/"
             f"workload.py`): single-GPU step times MEASURED on MI355X ({what}; "
             f"ResNet-50 {rn.step_time_1gpu * 1e3:.2f} ms, "
             f"BERT-base {bb.step_time_1gpu * 1e3:.2f} ms"
             + ("; VGG16 / Transformer have no fp32 measurement and keep their bf16 step times" if PREC == "fp32"
                else "") + "); "
             "fp32 gradient bytes exact; ring all-reduce bus bandwidth **" + bw + "** on every row, "
             f"{ASSUMED_INTERNODE_BUSBW_GBS:.0f} GB/s across nodes (ASSUMED); 30 % of a step hides the all-reduce.  "
             "Every job declares its precision and keeps the step count of the bf16 trace, so the fp32 "
             "tables carry ~3x the GPU-seconds of round 4's bf16 tables.  Resize pause 5 s, "
             "restart-from-checkpoint pause 15 s, rate limit 30 s (reference default).", "",
             "Job info (round 3): every job is seeded at submission from the workload it declares (remaining = "
             "epochs x epoch time on one GPU, speedup = the model's curve), jobs of one model share a category "
             "(JOB_CATEGORY), and the collector refreshes running jobs every 60 s -- the round-2 tables ran the "
             "info-driven policies on the reference's placeholder (1 s epochs, linear speedup) for unstarted jobs.",
             ""]
    lines += ["## Config 2: Elastic-Tiresias vs Tiresias, 8 ResNet-50 jobs, 8 GPUs", "", HEADER]
    lines += [row(r) for r in exp2()]
    lines += ["", "## Config 3: AFS-L on a mixed ResNet-50 + BERT-base trace, 8 GPUs", "", HEADER]
    lines += [row(r) for r in exp3()]
    lines += ["", "## Config 4: GPU drain on 2 x 8 GPUs, Elastic-FIFO: Munkres vs migration-naive binding", "",
              "Both use the same best-fit packing; the naive binding maps virtual nodes and GPU slots in index "
              "order, ignoring where workers run (reference bindNodes, placement_manager.go:492-522, is what "
              "the Munkres binding reproduces).  A job split across nodes all-reduces at inter-node bandwidth.",
              "",
              "| placement | avg JCT (s) | makespan (s) | resizes | worker migrations |", "|---|---:|---:|---:|---:|"]
    for name, r in exp4():
        lines.append(f"| {name} | {r.avg_jct:.0f} | {r.makespan:.0f} | {r.resizes} | {r.migrations} |")
    lines += ["", "## Config 5: 32-job Philly-style trace, all 8 policies, 1/2/4/8 GPUs", "", HEADER]
    res5 = exp5()
    lines += [row(r) for r in res5]
    lines += ["", f"## Config 5 with autoscale: capacity 1 -> 2 -> 4 -> 8 GPUs (doubling every {RAMP_T:.0f} s)", "",
              "The same 32-job trace (requests capped at 8) while GPUs ARRIVE: the scheduler learns of each "
              "addition through a node event and re-plans at once (work-conserving); elastic jobs grow onto "
              "the new GPUs, Munkres keeps running workers in place; a fixed 8-GPU cluster is the bound. "
              "Utilization is measured against the GPUs present at each moment (a fixed 1-GPU cluster cannot "
              "run this trace's non-elastic 8-GPU requests at all).", "",
              "| policy | avg JCT ramp 1->8 (s) | avg JCT fixed 8 (s) | makespan ramp / fixed 8 (s) "
              "| ramp utilization | ramp resizes | ramp migrations |", "|---|---:|---:|---|---:|---:|---:|"]
    for pol, rr, r8 in exp_autoscale():
        lines.append(f"| {pol} | {rr.avg_jct:.0f} | {r8.avg_jct:.0f} | {rr.makespan:.0f} / {r8.makespan:.0f} "
                     f"| {100 * rr.utilization:.0f} % | {rr.resizes} | {rr.migrations} |")
    lines += ["", "## Info-source ablation (config 5 trace): avg JCT (s) of the info-driven policies", "",
              "round-2 = what round 2 ran: exact info for started jobs, the reference placeholder for unstarted "
              "ones (units mixed: started jobs look long next to '1 s/epoch' arrivals); placeholder = the "
              "reference's CreateBaseJobInfo info for every job (1 s epochs, linear speedup -- on this trace the "
              "epoch count happens to track the length); online = the real round-3 pipeline (seeded from the "
              "declared workload, collector every 60 s; the default of every table above); oracle = exact "
              "remaining time and speed curve of every submitted job.", "",
              "| GPUs | policy | FIFO | round-2 | placeholder | online | oracle |",
              "|---:|---|---:|---:|---:|---:|---:|"]
    for r in exp_info():
        lines.append(f"| {r['gpus']} | {r['algorithm']} | {r['fifo']:.0f} | {r['mixed']:.0f} | "
                     f"{r['placeholder']:.0f} | {r['online']:.0f} | {r['oracle']:.0f} |")
    text = "\n".join(lines) + "\n"
    print(text)
    os.makedirs(os.path.dirname(a.out), exist_ok=True)
    with open(a.out, "w") as f:
        f.write(text)
    with open(a.out.replace(".md", ".json"), "w") as f:
        json.dump([r.summary() for r in res5], f, indent=1)


if __name__ == "__main__":
    main()
