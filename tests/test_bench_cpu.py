"""Multi-rank rehearsal of bench.py on CPU/gloo (the driver runs the real thing with one rank
per MI355X under torch.distributed.run): pool workers as torchrun ranks, rank 0 running the
control plane, elastic resizes across ranks, the JSON line contract."""
import json
import os
import subprocess
import sys

from vodascheduler_amd.runtime.cluster import free_port

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_bench_two_ranks_cpu_rehearsal():
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2", "--master-addr",
           "127.0.0.1", "--master-port", str(free_port()), os.path.join(ROOT, "bench.py"), "--gpus", "2", "--steps",
           "1", "--warmup", "2", "--jobs", "6", "--device", "cpu", "--rate-limit", "0.5", "--interarrival", "0.3"]
    env = dict(os.environ, VODA_STACKDUMP_S="100")
    r = subprocess.run(cmd, cwd="/tmp", env=env, capture_output=True, text=True, timeout=150)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [l for l in r.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, r.stdout  # rank 0 prints exactly one JSON line
    d = json.loads(lines[0])
    for k in ("metric", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step", "higher_is_better", "scaling",
              "vs_baseline", "dtype", "data", "config"):
        assert k in d
    assert d["n_gpus"] == 2 and d["higher_is_better"] is False and d["scaling"] == "weak"
    assert d["value"] > 0 and d["makespan_s"] >= d["value"]
    assert d["membership_changes"] >= 6  # every job started; some were resized across the two ranks
    assert d["grad_dtype"] == "fp32" and d["allreduce_dtype"] == "fp32"


import pytest  # noqa: E402


@pytest.mark.parametrize("n", [2, 4])
def test_bench_self_launches_ranks(n):
    """``python bench.py --gpus N`` with no WORLD_SIZE starts its own N ranks (a child
    torch.distributed.run launched before any GPU call) and prints one JSON line."""
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    cmd = [sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", str(n), "--steps", "1", "--warmup", "1",
           "--jobs", str(2 * n), "--device", "cpu", "--rate-limit", "0.5",
           "--interarrival", "0.2"]
    r = subprocess.run(cmd, cwd="/tmp", env=env, capture_output=True, text=True, timeout=240)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [l for l in r.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, r.stdout
    d = json.loads(lines[0])
    assert d["n_gpus"] == n and d["config"]["jobs"] == 2 * n
    assert d["value"] > 0
