"""Microbenchmarks for the ResNet-50 (bs 256, 224x224, channels_last bf16) op mix:

1. fused HIP BN(+add)(+ReLU) fwd+bwd vs MIOpen BatchNorm + separate add / ReLU kernels;
2. 1x1 convolutions: MIOpen conv vs the same product as a hipBLASLt GEMM on the NHWC
   [M, Cin] x [Cin, Cout] view (fwd + both backward products).

python benchmarks/bench_resnet_ops.py [--batch 256]
"""
from __future__ import annotations

import argparse
import json
import os
import sys

import torch
import torch.nn.functional as F

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from vodascheduler_amd.ops.batchnorm import batch_norm_act  # noqa: E402

# (C, H) of ResNet-50 BN layers at 224x224 (count in parentheses in comments)
BN_SHAPES = [(64, 112), (64, 56), (256, 56), (128, 56), (128, 28), (512, 28), (256, 28), (256, 14), (1024, 14),
             (512, 14), (512, 7), (2048, 7)]
CONV1x1 = [(64, 256, 56), (256, 64, 56), (256, 128, 56), (128, 512, 28), (512, 128, 28), (512, 256, 28),
           (256, 1024, 14), (1024, 256, 14), (1024, 512, 14), (512, 2048, 7), (2048, 512, 7)]


def timeit(fn, iters=20, warmup=3):
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


def bench_bn(batch):
    out = []
    for C, H in BN_SHAPES:
        for res in (False, True):
            x = torch.randn(batch, C, H, H, device="cuda", dtype=torch.bfloat16).to(
                memory_format=torch.channels_last).requires_grad_()
            r = torch.randn_like(x).requires_grad_() if res else None
            w = torch.ones(C, device="cuda", requires_grad=True)
            b = torch.zeros(C, device="cuda", requires_grad=True)
            rm, rv = torch.zeros(C, device="cuda"), torch.ones(C, device="cuda")
            dy = torch.randn_like(x)

            def fused():
                y = batch_norm_act(x, w, b, rm, rv, True, 0.1, 1e-5, r, True)
                y.backward(dy)

            def ref():
                y = F.batch_norm(x, rm, rv, w, b, True, 0.1, 1e-5)
                if r is not None:
                    y = y + r
                F.relu(y).backward(dy)

            tf, tr = timeit(fused), timeit(ref)
            nbytes = x.numel() * 2 * (3 + 5 + (2 if res else 0))  # min traffic of the fused schedule
            out.append({"op": "bn_relu" + ("_add" if res else ""), "C": C, "H": H, "fused_us": round(tf, 1),
                        "miopen_us": round(tr, 1), "speedup": round(tr / tf, 2),
                        "fused_TBps": round(nbytes / tf / 1e6, 2)})
            print(json.dumps(out[-1]), flush=True)
    return out


def bench_conv1x1(batch):
    out = []
    for cin, cout, H in CONV1x1:
        x = torch.randn(batch, cin, H, H, device="cuda", dtype=torch.bfloat16).to(
            memory_format=torch.channels_last).requires_grad_()
        w = (torch.randn(cout, cin, 1, 1, device="cuda", dtype=torch.bfloat16) * 0.05).to(
            memory_format=torch.channels_last).requires_grad_()
        dy = torch.randn(batch, cout, H, H, device="cuda", dtype=torch.bfloat16).to(memory_format=torch.channels_last)

        def conv():
            y = F.conv2d(x, w)
            y.backward(dy)

        def gemm():
            M = batch * H * H
            x2 = x.permute(0, 2, 3, 1).reshape(M, cin)
            y2 = x2 @ w.view(cout, cin).t()
            y = y2.view(batch, H, H, cout).permute(0, 3, 1, 2)
            y.backward(dy)

        tc, tg = timeit(conv), timeit(gemm)
        flops = 3 * 2 * batch * H * H * cin * cout
        out.append({"op": "conv1x1", "cin": cin, "cout": cout, "H": H, "miopen_us": round(tc, 1),
                    "gemm_us": round(tg, 1), "speedup": round(tc / tg, 2),
                    "miopen_TF": round(flops / tc / 1e6, 1), "gemm_TF": round(flops / tg / 1e6, 1)})
        print(json.dumps(out[-1]), flush=True)
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=256)
    ap.add_argument("--out", default="gpurun_out/bench_resnet_ops.json")
    a = ap.parse_args()
    res = {"bn": bench_bn(a.batch), "conv1x1": bench_conv1x1(a.batch)}
    os.makedirs(os.path.dirname(a.out), exist_ok=True)
    with open(a.out, "w") as f:
        json.dump(res, f, indent=1)


if __name__ == "__main__":
    main()
