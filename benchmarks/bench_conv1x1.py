"""1x1 convolutions of ResNet-50 (batch 256, channels_last, bf16) on MI355X: MIOpen (torch
conv2d forward + backward) vs the GEMM formulation -- forward and input gradient as
hipBLASLt GEMMs on the [N*H*W, C] views, weight gradient on the split-K MFMA kernel
(csrc/hip/wgrad.hip) accumulating into a bf16 gradient buffer.

python benchmarks/bench_conv1x1.py
"""
from __future__ import annotations

import json
import os
import sys

import torch
import torch.nn.functional as F

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from vodascheduler_amd.ops import wgrad as W  # noqa: E402

# (H=W of the conv input, Cin, Cout, stride, count per ResNet-50 step)
SHAPES = [(56, 64, 64, 1, 1), (56, 256, 64, 1, 2), (56, 64, 256, 1, 4), (56, 256, 128, 1, 1), (56, 256, 512, 2, 1),
          (28, 128, 512, 1, 4), (28, 512, 128, 1, 3), (28, 512, 256, 1, 1), (28, 512, 1024, 2, 1),
          (14, 256, 1024, 1, 6), (14, 1024, 256, 1, 5), (14, 1024, 512, 1, 1), (14, 1024, 2048, 2, 1),
          (7, 512, 2048, 1, 3), (7, 2048, 512, 1, 2)]
B = 256


def timeit(fn, iters=20, warm=3) -> float:
    for _ in range(warm):
        fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(iters):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / iters * 1e3


def main():
    torch.backends.cudnn.benchmark = True
    dev = torch.device("cuda", 0)
    tot = {"miopen": 0.0, "gemm": 0.0}
    for H, cin, cout, stride, count in SHAPES:
        x = torch.randn(B, cin, H, H, device=dev).bfloat16().to(memory_format=torch.channels_last)
        w = (torch.randn(cout, cin, 1, 1, device=dev) * 0.05).bfloat16().to(memory_format=torch.channels_last)
        Ho = H // stride
        dy = torch.randn(B, cout, Ho, Ho, device=dev).bfloat16().to(memory_format=torch.channels_last)
        xr = x.detach().requires_grad_(True)
        wr = w.detach().requires_grad_(True)

        def miopen():
            y = F.conv2d(xr, wr, stride=stride)
            y.backward(dy)

        gw = torch.zeros(cout, cin, device=dev, dtype=torch.bfloat16)
        w2 = w.view(cout, cin)
        dy2 = dy.permute(0, 2, 3, 1).reshape(-1, cout)

        def gemm():
            xs = x if stride == 1 else x[:, :, ::stride, ::stride]
            x2 = xs.permute(0, 2, 3, 1).reshape(-1, cin)       # copy only when strided
            y2 = x2 @ w2.t()                                   # forward
            dx2 = dy2 @ w2                                     # input gradient (stride 1; stride 2 scatters)
            W.wgrad_accumulate_(dy2, x2, gw)                   # weight gradient
            return y2, dx2

        # numerics of the GEMM path against MIOpen
        y_ref = F.conv2d(x.float(), w.float(), stride=stride)
        y2, _ = gemm()
        err = float((y2.float() - y_ref.permute(0, 2, 3, 1).reshape(-1, cout)).norm() / y_ref.norm())
        t_m = timeit(miopen)
        t_g = timeit(gemm)
        tot["miopen"] += t_m * count
        tot["gemm"] += t_g * count
        print(json.dumps({"H": H, "cin": cin, "cout": cout, "stride": stride, "count": count, "miopen_us": round(t_m, 1),
                          "gemm_us": round(t_g, 1), "speedup": round(t_m / t_g, 2), "fwd_rel_err": round(err, 5),
                          "splits": W.default_splits(B * Ho * Ho, cout, cin)}), flush=True)
    print(json.dumps({"resnet50_1x1_convs_per_step_ms": {k: round(v / 1e3, 3) for k, v in tot.items()}}), flush=True)


if __name__ == "__main__":
    main()
