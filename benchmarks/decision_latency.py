"""Allocation + placement decision latency (BASELINE.md row "Allocation + placement decision
latency, all 8 policies, 32 jobs"): one reschedule's allocator call (policy) and Munkres
placement, timed on the host for 32 ready jobs on 1, 2, 4 and 8 GPUs (and a 16 x 8 GPU
cluster).  CPU only.

python benchmarks/decision_latency.py [--out profiles/r1_decision_latency.json]
"""
from __future__ import annotations

import argparse
import json
import os
import statistics
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from vodascheduler_amd.algorithm import ALGORITHMS  # noqa: E402
from vodascheduler_amd.allocator.allocator import AllocationRequest, ResourceAllocator  # noqa: E402
from vodascheduler_amd.common.mq import InProcQueue  # noqa: E402
from vodascheduler_amd.common.store import MemoryStore  # noqa: E402
from vodascheduler_amd.common.trainingjob import TrainingJob  # noqa: E402
from vodascheduler_amd.common.types import DEFAULT_GPU_TYPE  # noqa: E402
from vodascheduler_amd.placement.manager import PlacementManager  # noqa: E402
from vodascheduler_amd.service.service import TrainingService  # noqa: E402
from vodascheduler_amd.sim.trace import philly_trace  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--jobs", type=int, default=32)
    ap.add_argument("--reps", type=int, default=50)
    ap.add_argument("--out", default=None)
    a = ap.parse_args()
    store = MemoryStore()
    svc = TrainingService(store, InProcQueue(maxsize=10 ** 6))
    names = [svc.create_training_job(json.dumps(tj.spec)) for tj in philly_trace(a.jobs, seed=0)]
    jobs = [TrainingJob.from_dict(store.find_metadata(n, DEFAULT_GPU_TYPE)) for n in names]
    alloc = ResourceAllocator(store)
    out = []
    for nodes, gpus in ((1, 1), (1, 2), (1, 4), (1, 8), (16, 8)):
        topo = {f"node{i}": list(range(gpus)) for i in range(nodes)}
        total = nodes * gpus
        for algo in sorted(ALGORITHMS):
            ta, tp = [], []
            for _ in range(a.reps):
                req = AllocationRequest(DEFAULT_GPU_TYPE, total, algo, [j.clone() for j in jobs])
                t0 = time.perf_counter()
                res = alloc.allocate(req)
                t1 = time.perf_counter()
                pm = PlacementManager(DEFAULT_GPU_TYPE, topo)
                pm.place({j: n for j, n in res.items() if n > 0})
                t2 = time.perf_counter()
                ta.append((t1 - t0) * 1e3)
                tp.append((t2 - t1) * 1e3)
            rec = {"gpus": total, "nodes": nodes, "algorithm": algo, "jobs": len(jobs),
                   "allocation_ms_p50": round(statistics.median(ta), 3),
                   "placement_ms_p50": round(statistics.median(tp), 3),
                   "total_ms_p95": round(sorted(x + y for x, y in zip(ta, tp))[int(0.95 * len(ta)) - 1], 3)}
            print(json.dumps(rec), flush=True)
            out.append(rec)
    if a.out:
        with open(a.out, "w") as f:
            json.dump(out, f, indent=1)


if __name__ == "__main__":
    main()
