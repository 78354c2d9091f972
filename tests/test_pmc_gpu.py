"""Hardware-counter check of the hand-written kernels ("rocprofv3
counter checks"): one ``rocprofv3 --kernel-trace --pmc`` pass over a fixed workload
(benchmarks/pmc_target.py) must show the matrix cores busy in every own GEMM / attention
kernel -- the MFMA path, not a VALU fallback, is what runs."""
import csv
import glob
import os
import shutil
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
COUNTERS = ["SQ_VALU_MFMA_BUSY_CYCLES", "SQ_INSTS_VALU", "SQ_INSTS_LDS"]  # one pass, SQ block only
KERNELS = ["gemm_f32_stats_kernel", "gemm_bnstats_kernel", "attn_f32_fwd"]


@pytest.mark.skipif(shutil.which("rocprofv3") is None, reason="rocprofv3 not on PATH")
def test_own_kernels_run_on_the_matrix_cores(tmp_path):
    out = tmp_path / "pmc"
    env = dict(os.environ, TMPDIR="/tmp", PYTHONPATH=ROOT + os.pathsep + os.environ.get("PYTHONPATH", ""))
    cmd = ["timeout", "-s", "KILL", "90", "rocprofv3", "--kernel-trace", "--pmc", *COUNTERS, "-d", str(out),
           "-o", "run", "--output-format", "csv", "--", sys.executable, os.path.join(ROOT, "benchmarks", "pmc_target.py")]
    r = subprocess.run(cmd, cwd="/tmp", env=env, capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, (r.returncode, r.stdout[-2000:], r.stderr[-2000:])
    files = glob.glob(str(out / "**" / "*counter_collection.csv"), recursive=True)
    assert files, f"no counter file under {out}: {r.stdout[-1000:]}"
    busy: dict[str, list[float]] = {}
    with open(files[0]) as f:
        for row in csv.DictReader(f):
            name = row.get("Kernel_Name", "")
            for k in KERNELS:
                if k in name and row.get("Counter_Name") == "SQ_VALU_MFMA_BUSY_CYCLES":
                    busy.setdefault(k, []).append(float(row["Counter_Value"]))
    for k in KERNELS:
        assert busy.get(k), f"{k}: no SQ_VALU_MFMA_BUSY_CYCLES record ({sorted(busy)})"
        assert min(busy[k]) > 0, f"{k}: matrix cores idle ({busy[k]})"
