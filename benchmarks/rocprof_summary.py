"""Turn a rocprofv3 ``*_kernel_stats.csv`` into a markdown table (for profiles/).

python benchmarks/rocprof_summary.py gpurun_out/prof_bert/x_kernel_stats.csv "title" [top_n] [steps]
"""
from __future__ import annotations

import csv
import sys


def summarize(path: str, title: str, top: int = 40, steps: int = 0) -> str:
    rows = list(csv.DictReader(open(path)))
    tot = sum(float(r["TotalDurationNs"]) for r in rows)
    out = [f"# {title}", "", f"Total GPU kernel time: {tot / 1e6:.1f} ms over {len(rows)} kernel names"
           + (f" ({tot / 1e6 / steps:.2f} ms per step over {steps} steps)." if steps else "."), "",
           "| % time | calls | avg us | total ms | kernel |", "|---:|---:|---:|---:|---|"]
    rows.sort(key=lambda r: -float(r["TotalDurationNs"]))
    for r in rows[:top]:
        name = r["Name"].replace("|", "/")
        if len(name) > 110:
            name = name[:107] + "..."
        out.append(f"| {100 * float(r['TotalDurationNs']) / tot:.1f} | {r['Calls']} | "
                   f"{float(r['AverageNs']) / 1e3:.1f} | {float(r['TotalDurationNs']) / 1e6:.2f} | `{name}` |")
    return "\n".join(out) + "\n"


if __name__ == "__main__":
    top = int(sys.argv[3]) if len(sys.argv) > 3 else 40
    steps = int(sys.argv[4]) if len(sys.argv) > 4 else 0
    print(summarize(sys.argv[1], sys.argv[2], top, steps))
