"""ResNet-50 stem (7x7 stride-2 convolution, 3 -> 64 channels, bs 256, 224x224, channels_last
bf16): MIOpen forward + weight gradient with the input channels zero-padded to 3 / 4 / 8.

A 3-channel NHWC image gives MIOpen's implicit-GEMM solvers a 147-long reduction made of
6-byte pixel rows; the round-2 profile has the stem at ~360 us forward + ~350 us weight
gradient per step (~85 TFLOP/s).  Padding the channels (zeros; the padded weight rows get zero
gradients) changes the solver choice.  The timing of the padded variants INCLUDES building the
padded input (one extra pass over the image) and slicing the weight gradient back.

python benchmarks/bench_stem.py
"""
from __future__ import annotations

import json

import torch
import torch.nn.functional as F

torch.backends.cudnn.benchmark = True
B = 256


def t_us(fn, it=10):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(it):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / it * 1e3


def main():
    torch.manual_seed(0)
    x3 = torch.randn(B, 3, 224, 224, device="cuda", dtype=torch.bfloat16).to(memory_format=torch.channels_last)
    w3 = (torch.randn(64, 3, 7, 7, device="cuda", dtype=torch.bfloat16) * 0.05).to(memory_format=torch.channels_last)
    dy = None
    ref = None
    for cin in (3, 4, 8):
        w = w3.detach().clone().requires_grad_()

        def step():
            if cin == 3:
                xp, wp = x3, w
            else:
                xp = F.pad(x3, (0, 0, 0, 0, 0, cin - 3)).contiguous(memory_format=torch.channels_last)
                wp = F.pad(w, (0, 0, 0, 0, 0, cin - 3)).contiguous(memory_format=torch.channels_last)
            y = F.conv2d(xp, wp, stride=2, padding=3)
            return y

        y = step()
        if dy is None:
            dy = torch.randn_like(y)

        def fwd():
            with torch.no_grad():
                step()

        def fwd_bwd():
            w.grad = None
            step().backward(dy)

        fwd_bwd()
        g = w.grad.float().clone()
        if ref is None:
            ref = g
        err = ((g - ref).norm() / ref.norm()).item()
        tf = t_us(fwd)
        tfb = t_us(fwd_bwd)
        flop = 2.0 * B * 112 * 112 * 64 * 147
        print(json.dumps({"cin": cin, "fwd_us": round(tf, 1), "fwd_wgrad_us": round(tfb, 1),
                          "wgrad_us": round(tfb - tf, 1), "fwd_tflops": round(flop / tf / 1e6, 1),
                          "wgrad_rel_err_vs_cin3": err}), flush=True)


def bn_pool():
    """Stem BN + ReLU + 3x3/2 max pool, bs 256 x 64 x 112 x 112 bf16: fused kernels vs the
    fused BN(+ReLU) followed by the HIP max pool (forward + backward, flat-free gradients)."""
    import sys
    import os

    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    from vodascheduler_amd.ops.batchnorm import FusedBatchNorm2d, FusedBNReLUMaxPool2d
    from vodascheduler_amd.ops.pool import max_pool2d

    torch.manual_seed(0)
    x = torch.randn(B, 64, 112, 112, device="cuda", dtype=torch.bfloat16).to(memory_format=torch.channels_last)
    fused = FusedBNReLUMaxPool2d(64).cuda()
    bn = FusedBatchNorm2d(64, relu=True).cuda()
    dy = torch.randn(B, 64, 56, 56, device="cuda", dtype=torch.bfloat16).to(memory_format=torch.channels_last)
    xi = x.clone().requires_grad_()

    def run_fused():
        xi.grad = None
        fused(xi).backward(dy)

    def run_split():
        xi.grad = None
        max_pool2d(bn(xi), 3, 2, 1).backward(dy)

    for name, fn in (("split", run_split), ("fused", run_fused), ("split", run_split), ("fused", run_fused)):
        print(json.dumps({"stem_bn_relu_pool": name, "fwd_bwd_us": round(t_us(fn), 1)}), flush=True)


if __name__ == "__main__":
    import sys as _sys

    if "--only-bn-pool" not in _sys.argv:
        main()
    bn_pool()
