"""Per-dispatch rows (name, grid, duration) of the steady-state window of a rocprofv3 kernel
trace for kernels whose name contains any of the given substrings (see trace_window_stats.py
for the window).  Used to attribute a templated kernel's time to the layer shapes by grid.

python benchmarks/trace_dispatches.py TRACE.csv OUT.csv SUBSTR [SUBSTR ...]
"""
from __future__ import annotations

import csv
import sys


def main(trace: str, out: str, pats: list[str]) -> None:
    rows = list(csv.DictReader(open(trace)))
    name_k = "Kernel_Name" if "Kernel_Name" in rows[0] else "Name"
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    last = max([i for i, r in enumerate(rows) if "spin" in r[name_k].lower()], default=-1)
    grid_cols = [c for c in rows[0] if c.lower().startswith(("grid", "workgroup"))]
    with open(out, "w", newline="") as f:
        w = csv.writer(f)
        w.writerow(["Name", *grid_cols, "DurationNs"])
        for r in rows[last + 1:]:
            n = r[name_k]
            if any(p in n for p in pats):
                w.writerow([n[:90], *[r[c] for c in grid_cols], int(r["End_Timestamp"]) - int(r["Start_Timestamp"])])


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2], sys.argv[3:])
