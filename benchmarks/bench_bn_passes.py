"""Fused BatchNorm(+add)(+ReLU) forward/backward over every ResNet-50 (bs 256, 224x224) BN shape,
timed per layer shape with the achieved HBM bandwidth of the whole fwd / bwd (bytes that must
move: fwd = x read twice (stats + apply) + residual + y + mask bit; bwd = dy, x, mask twice +
dx (+ dres)).  Run under ``rocprofv3 --kernel-trace --stats`` for the per-pass split.

python benchmarks/bench_bn_passes.py [--batch 256]
"""
from __future__ import annotations

import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from vodascheduler_amd.ops.batchnorm import FusedBatchNorm2d  # noqa: E402

# (C, H, residual, relu, count per step) of the ResNet-50 v1.5 BN layers at 224x224
ITERS = [20]
SHAPES = [(64, 112, False, True, 1), (64, 56, False, True, 6), (256, 56, True, True, 3), (256, 56, False, False, 1),
          (128, 56, False, True, 1), (128, 28, False, True, 7), (512, 28, True, True, 4), (512, 28, False, False, 1),
          (256, 28, False, True, 1), (256, 14, False, True, 11), (1024, 14, True, True, 6),
          (1024, 14, False, False, 1), (512, 14, False, True, 1), (512, 7, False, True, 5), (2048, 7, True, True, 3),
          (2048, 7, False, False, 1)]


def timeit(fn, iters=20, warmup=3):
    iters = ITERS[0]
    for _ in range(warmup):
        fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(iters):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / iters * 1e3  # us


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=256)
    ap.add_argument("--tuning", default="", help="deep,blocks,sweep for the reduction passes (A/B)")
    ap.add_argument("--shapes", default="", help="comma-separated indices into SHAPES (PMC runs)")
    ap.add_argument("--iters", type=int, default=20)
    a = ap.parse_args()
    ITERS[0] = a.iters
    if a.tuning:
        from vodascheduler_amd.ops import _native

        _native.hip().bn_set_tuning(*[int(v) for v in a.tuning.split(",")])
    dev = "cuda"
    cl = torch.channels_last
    rows, tot_f, tot_b = [], 0.0, 0.0
    big = torch.empty(1 << 28, dtype=torch.bfloat16, device=dev)
    copy_us = timeit(lambda: big.clone())
    copy_tbs = 2 * big.numel() * 2 / (copy_us * 1e-6) / 1e12
    shapes = [SHAPES[int(i)] for i in a.shapes.split(",")] if a.shapes else SHAPES
    for C, H, res, relu, cnt in shapes:
        bn = FusedBatchNorm2d(C, relu=relu).to(dev)
        x = torch.randn(a.batch, C, H, H, device=dev).to(torch.bfloat16).to(memory_format=cl).requires_grad_()
        r = torch.randn_like(x).requires_grad_() if res else None
        y = bn(x, r)
        g = torch.randn_like(y)
        n = x.numel()
        fwd = timeit(lambda: bn(x, r))
        y = bn(x, r)
        bwd = timeit(lambda: torch.autograd.grad(y, [x] + ([r] if res else []), g, retain_graph=True))
        fb = 2 * n * 2 + (2 * n if res else 0) + 2 * n + (n / 8 if relu else 0)
        bb = 2 * (2 * n * 2 + (n / 8 if relu else 0)) + 2 * n + (2 * n if res else 0)
        rows.append({"C": C, "H": H, "res": res, "relu": relu, "count": cnt, "fwd_us": round(fwd, 1),
                     "bwd_us": round(bwd, 1), "fwd_TBs": round(fb / (fwd * 1e-6) / 1e12, 2),
                     "bwd_TBs": round(bb / (bwd * 1e-6) / 1e12, 2)})
        tot_f += cnt * fwd
        tot_b += cnt * bwd
    print(json.dumps({"batch": a.batch, "tuning": a.tuning, "copy_TBs": round(copy_tbs, 2), "per_step_fwd_ms": round(tot_f / 1e3, 3),
                      "per_step_bwd_ms": round(tot_b / 1e3, 3), "shapes": rows}, indent=1))


if __name__ == "__main__":
    main()
