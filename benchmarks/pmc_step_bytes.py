"""HBM traffic per training step from a rocprofv3 ``--pmc TCC_EA0_RDREQ_sum TCC_EA0_WRREQ_sum``
run of ``benchmarks/model_step.py``: the dispatches of the last ``--steps`` steps (a step ends
at the optimizer kernel named by ``--marker``) are grouped by kernel, and the request counts
are priced at 64 B each (gfx950 tallies 128-B streaming reads as 64 B, MI355X_MICROARCH.md).

python benchmarks/pmc_step_bytes.py run_counter_collection.csv [--steps 3] [--marker sgd_kernel]
    [--label A] [--top 25] > table.md
"""
from __future__ import annotations

import argparse
import csv
import re
from collections import defaultdict


def short_name(name: str) -> str:
    s = name.replace("(anonymous namespace)::", "").replace("voda::", "")
    return re.sub(r"\(.*", "", s)[:80]


def step_bytes(path: str, steps: int, marker: str) -> tuple[dict[str, list[float]], int]:
    """{kernel: [read bytes, write bytes, dispatches]} summed over the last ``steps`` steps."""
    disp: dict[int, dict] = {}
    with open(path) as f:
        for r in csv.DictReader(f):
            d = disp.setdefault(int(r["Dispatch_Id"]), {"name": r["Kernel_Name"]})
            d[r["Counter_Name"]] = d.get(r["Counter_Name"], 0.0) + float(r["Counter_Value"])
    order = sorted(disp)
    ends = [i for i, k in enumerate(order) if marker in disp[k]["name"]]
    # a step may run the marker more than once (one optimizer launch per dtype group): keep
    # the last marker launch of each group of consecutive marker launches
    step_ends = [e for j, e in enumerate(ends) if j + 1 == len(ends) or ends[j + 1] != e + 1]
    if len(step_ends) < steps + 1:
        raise SystemExit(f"{path}: found {len(step_ends)} steps, need {steps + 1}")
    lo, hi = step_ends[-steps - 1] + 1, step_ends[-1] + 1
    out: dict[str, list[float]] = defaultdict(lambda: [0.0, 0.0, 0])
    for k in order[lo:hi]:
        d = disp[k]
        e = out[short_name(d["name"])]
        e[0] += 64.0 * d.get("TCC_EA0_RDREQ_sum", 0.0) / steps
        e[1] += 64.0 * d.get("TCC_EA0_WRREQ_sum", 0.0) / steps
        e[2] += 1
    return out, hi - lo


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("csv", nargs="+")
    ap.add_argument("--label", nargs="*", default=None)
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("--marker", default="sgd_kernel")
    ap.add_argument("--top", type=int, default=25)
    a = ap.parse_args()
    labels = a.label or [f"run{i}" for i in range(len(a.csv))]
    runs = [step_bytes(p, a.steps, a.marker)[0] for p in a.csv]
    print("| run | HBM read GB/step | HBM write GB/step | total GB/step |")
    print("|---|---:|---:|---:|")
    for lab, r in zip(labels, runs):
        rd = sum(v[0] for v in r.values()) / 1e9
        wr = sum(v[1] for v in r.values()) / 1e9
        print(f"| {lab} | {rd:.3f} | {wr:.3f} | {rd + wr:.3f} |")
    print()
    names = sorted({k for r in runs for k in r}, key=lambda k: -max(r.get(k, [0, 0])[0] + r.get(k, [0, 0])[1]
                                                                     for r in runs))
    print("| kernel | " + " | ".join(f"{lab} rd+wr MB (calls)" for lab in labels) + " |")
    print("|---|" + "---:|" * len(labels))
    for k in names[:a.top]:
        cells = []
        for r in runs:
            v = r.get(k)
            cells.append(f"{(v[0] + v[1]) / 1e6:.1f} ({v[2] // a.steps})" if v else "")
        print(f"| `{k}` | " + " | ".join(cells) + " |")


if __name__ == "__main__":
    main()
