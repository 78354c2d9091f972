"""Fused Adam / AdamW step (csrc/hip/optim.hip) on a BERT-base-sized flat buffer (110 M fp32
params, fp32 gradients, bf16 model copy): HBM throughput, with and without the bf16 copy.  Bytes
per element: p g m v read (16) + p m v written (12) + bf16 copy (2).

python benchmarks/bench_adam.py [--n 110000000]
"""
from __future__ import annotations

import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from vodascheduler_amd.ops import _native as N  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=110_000_000)
    ap.add_argument("--iters", type=int, default=20)
    a = ap.parse_args()
    h = N.hip()
    n = a.n
    p = torch.randn(n, device="cuda")
    g = torch.randn(n, device="cuda")
    m = torch.zeros(n, device="cuda")
    v = torch.zeros(n, device="cuda")
    lp = torch.empty(n, device="cuda", dtype=torch.bfloat16)
    s = torch.cuda.current_stream().cuda_stream
    # reference: a device copy of the same element count (read 4 B + write 4 B per element)
    for _ in range(3):
        m.copy_(p)
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(a.iters):
        m.copy_(p)
    e1.record()
    torch.cuda.synchronize()
    us = e0.elapsed_time(e1) / a.iters * 1e3
    print(json.dumps({"n": n, "copy_us": round(us, 1), "copy_TBps": round(8 * n / us / 1e6, 2)}), flush=True)
    m.zero_()
    for lowp in (True, False):
        def step(k):
            h.adam_step(p.data_ptr(), g.data_ptr(), N.dtype_code(g.dtype), m.data_ptr(), v.data_ptr(),
                        lp.data_ptr() if lowp else 0, N.dtype_code(lp.dtype) if lowp else -1, n, 1e-4, 0.9,
                        0.999, 1e-8, 1e-2, True, k, 1.0, 0, s)
        for k in range(3):
            step(k + 1)
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for k in range(a.iters):
            step(k + 4)
        e1.record()
        torch.cuda.synchronize()
        us = e0.elapsed_time(e1) / a.iters * 1e3
        nbytes = n * (28 + (2 if lowp else 0))
        print(json.dumps({"n": n, "bf16_copy": lowp, "us": round(us, 1),
                          "TBps": round(nbytes / us / 1e6, 2)}), flush=True)


if __name__ == "__main__":
    main()
