"""Per-kernel stats of the steady-state window of a rocprofv3 kernel trace.

``benchmarks/model_step.py --profile-marker`` launches ``torch.cuda._sleep`` (a kernel named
``*spin*``) right before its timed steps; this script keeps only the kernels dispatched
after the LAST such marker (so MIOpen's find/benchmark kernels of the warm-up steps do not
pollute the numbers) and writes a ``*_kernel_stats.csv``-compatible summary.

python benchmarks/trace_window_stats.py TRACE.csv OUT_STATS.csv
"""
from __future__ import annotations

import csv
import sys
from collections import defaultdict


def main(trace: str, out: str) -> None:
    rows = list(csv.DictReader(open(trace)))
    name_k = "Kernel_Name" if "Kernel_Name" in rows[0] else "Name"
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    last = -1
    for i, r in enumerate(rows):
        if "spin" in r[name_k].lower():
            last = i
    window = rows[last + 1:]
    agg: dict[str, list[int]] = defaultdict(list)
    for r in window:
        agg[r[name_k]].append(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]))
    tot = sum(sum(v) for v in agg.values()) or 1
    with open(out, "w", newline="") as f:
        w = csv.writer(f, quoting=csv.QUOTE_NONNUMERIC)
        w.writerow(["Name", "Calls", "TotalDurationNs", "AverageNs", "Percentage", "MinNs", "MaxNs", "StdDev"])
        for n, v in sorted(agg.items(), key=lambda kv: -sum(kv[1])):
            s = sum(v)
            w.writerow([n, len(v), s, s / len(v), round(100 * s / tot, 2), min(v), max(v), 0.0])
    span = int(window[-1]["End_Timestamp"]) - int(window[0]["Start_Timestamp"]) if window else 0
    print(f"window: {len(window)} kernels after marker #{last}, busy {tot / 1e6:.2f} ms over {span / 1e6:.2f} ms")


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2])
