"""Fused attention forward + backward on one shape (default: BERT-base seq 128), timed with
CUDA events; run under ``rocprofv3 --pmc`` for counters.

python benchmarks/bench_attention.py [--B 64 --H 12 --T 128 --D 64 --iters 20]
"""
from __future__ import annotations

import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from vodascheduler_amd.ops import _native  # noqa: E402
from vodascheduler_amd.ops.attention import attention_qkvpacked  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--B", type=int, default=64)
    ap.add_argument("--H", type=int, default=12)
    ap.add_argument("--T", type=int, default=128)
    ap.add_argument("--D", type=int, default=64)
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--fwd-only", action="store_true")
    ap.add_argument("--dtype", default="bf16", choices=["bf16", "fp32"])
    a = ap.parse_args()
    _native.hip()
    dev = "cuda"
    dt = torch.bfloat16 if a.dtype == "bf16" else torch.float32
    qkv = torch.randn(a.B, a.T, 3, a.H, a.D, device=dev).to(dt).requires_grad_()
    km = torch.ones(a.B, a.T, dtype=torch.bool, device=dev)
    do = torch.randn(a.B, a.T, a.H, a.D, device=dev).to(dt)

    def step():
        if a.fwd_only:
            with torch.no_grad():
                attention_qkvpacked(qkv, km, False)
            return
        o = attention_qkvpacked(qkv, km, False)
        o.backward(do)

    for _ in range(3):
        step()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(a.iters):
        step()
    e1.record()
    torch.cuda.synchronize()
    us = e0.elapsed_time(e1) / a.iters * 1e3
    flops = 4 * a.B * a.H * a.T * a.T * a.D * (1.0 if a.fwd_only else 3.5)  # fwd 2 GEMMs + bwd 5 GEMMs
    print(json.dumps({"B": a.B, "H": a.H, "T": a.T, "D": a.D, "dtype": a.dtype, "fwd_only": a.fwd_only,
                      "env_resident": os.environ.get("VODA_ATTN_RESIDENT", "1"),
                      "us": round(us, 1), "tflops": round(flops / (us * 1e-6) / 1e12, 1)}))


if __name__ == "__main__":
    main()
