"""The BASELINE.json experiment configs, run in the discrete-event simulator (the real
scheduler + allocator + placement code in virtual time).  Job speed
curves come from the MI355X-calibrated ``sim.trace.PROFILES``.

  1. Elastic-FIFO, 2 toy MNIST jobs, 2 slots   -> real CPU/gloo run: tests/test_elastic_cpu.py
  2. Elastic-Tiresias, 8 ResNet-50 ImageNet-shape jobs on 8 GPUs (vs Tiresias)
  3. AFS-L, mixed ResNet-50 + BERT-base trace on 8 GPUs (vs FIFO / ElasticFIFO)
  4. Munkres placement + worker migration under GPU drain (2 nodes x 8 GPUs)
  5. FfDL Optimizer, 32-job Philly-style trace, 1/2/4/8 GPUs (all 8 policies side by side)

python benchmarks/experiments.py [--out profiles/r1_sim_experiments.md]
"""
from __future__ import annotations

import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from vodascheduler_amd.algorithm import ALGORITHMS  # noqa: E402
from vodascheduler_amd.sim.simulator import simulate  # noqa: E402
from vodascheduler_amd.sim.trace import (ASSUMED_BUSBW_GBS, ASSUMED_INTERNODE_BUSBW_GBS, TraceJob,  # noqa: E402
                                         make_spec, philly_trace)

ORDER = ["FIFO", "ElasticFIFO", "SRJF", "ElasticSRJF", "Tiresias", "ElasticTiresias", "FfDLOptimizer", "AFS-L"]


def row(r) -> str:
    return (f"| {r.algorithm} | {r.gpus} | {r.avg_jct:.0f} | {r.median_jct:.0f} | {r.p95_jct:.0f} | {r.makespan:.0f} "
            f"| {r.avg_wait:.0f} | {100 * r.utilization:.0f} % | {r.resizes} | {r.migrations} |")


HEADER = ("| policy | GPUs | avg JCT (s) | median JCT | p95 JCT | makespan (s) | avg wait | utilization | resizes "
          "| migrations |\n|---|---:|---:|---:|---:|---:|---:|---:|---:|---:|")


def exp2():
    tr = [TraceJob(60.0 * i, make_spec(f"resnet50-{i}", "resnet50", 4, 1, 8, 10, 2000)) for i in range(8)]
    return [simulate(tr, a, gpus=8) for a in ("Tiresias", "ElasticTiresias")]


def exp3():
    tr = philly_trace(32, seed=3, models=("resnet50", "bert-base"))
    return [simulate(tr, a, gpus=8) for a in ("FIFO", "ElasticFIFO", "AFS-L")]


def exp4():
    tr = philly_trace(24, seed=4, mean_interarrival_s=20.0)
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
        tr32 = philly_trace(32, seed=0, max_gpus=g)
        for a in ORDER:
            out.append(simulate(tr32, a, gpus=g))
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--out", default="profiles/r2_sim_experiments.md")
    a = ap.parse_args()
    assert set(ORDER) == set(ALGORITHMS)
    lines = ["# BASELINE.json configs in the discrete-event simulator (round 2)", "",
             "Real scheduler / allocator / placement code driven in virtual time (`benchmarks/experiments.py`). "
             "Job speed model (`vodascheduler_amd/sim/trace.py`): single-GPU step times MEASURED on MI355X for "
             "every workload but the PyTorch MNIST net (`benchmarks/model_step.py`, fp32 gradients, eager step); "
             "fp32 gradient bytes exact; ring all-reduce bus bandwidth ASSUMED "
             f"({ASSUMED_BUSBW_GBS:.0f} GB/s intra-node, {ASSUMED_INTERNODE_BUSBW_GBS:.0f} GB/s across nodes) until "
             "the 8-GPU bench measures it; 30 % of a step hides the all-reduce.  Resize pause 5 s, "
             "restart-from-checkpoint pause 15 s, rate limit 30 s (reference default).", ""]
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
    text = "\n".join(lines) + "\n"
    print(text)
    os.makedirs(os.path.dirname(a.out), exist_ok=True)
    with open(a.out, "w") as f:
        f.write(text)
    with open(a.out.replace(".md", ".json"), "w") as f:
        json.dump([r.summary() for r in res5], f, indent=1)


if __name__ == "__main__":
    main()
