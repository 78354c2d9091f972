"""Every convolution of a ResNet-50 bs256 step at fp32 (the reference's precision), channels_last,
on MI355X: forward / input-gradient / weight-gradient times of MIOpen (aten convolution) and, for
the 1x1 layers, of the GEMM formulation on hipBLASLt (the [N*H*W, C] views), with TFLOP/s
against the 157 TF fp32 MFMA peak.  Tells where the fp32 step's convolution time goes.

python benchmarks/bench_resnet_fp32_convs.py [--out file.jsonl]
"""
from __future__ import annotations

import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import vodascheduler_amd  # noqa: F401,E402 -- shared MIOpen find-db (var/miopen)

B = 256
# (H_in, Cin, Cout, k, stride, count per step) -- ResNet-50 v1.5 (stride on the 3x3)
SHAPES = [
    (224, 3, 64, 7, 2, 1),
    (56, 64, 64, 1, 1, 1), (56, 64, 64, 3, 1, 3), (56, 64, 256, 1, 1, 4), (56, 256, 64, 1, 1, 2),
    (56, 256, 128, 1, 1, 1), (56, 128, 128, 3, 2, 1), (56, 256, 512, 1, 2, 1),
    (28, 128, 128, 3, 1, 3), (28, 128, 512, 1, 1, 4), (28, 512, 128, 1, 1, 3),
    (28, 512, 256, 1, 1, 1), (28, 256, 256, 3, 2, 1), (28, 512, 1024, 1, 2, 1),
    (14, 256, 256, 3, 1, 5), (14, 256, 1024, 1, 1, 6), (14, 1024, 256, 1, 1, 5),
    (14, 1024, 512, 1, 1, 1), (14, 512, 512, 3, 2, 1), (14, 1024, 2048, 1, 2, 1),
    (7, 512, 512, 3, 1, 2), (7, 512, 2048, 1, 1, 3), (7, 2048, 512, 1, 1, 2),
]


def timeit(fn, iters=10, warm=3) -> float:
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
    ap = argparse.ArgumentParser()
    ap.add_argument("--out", default=None)
    ap.add_argument("--only-1x1", action="store_true")
    a = ap.parse_args()
    torch.backends.cudnn.benchmark = True
    dev = torch.device("cuda", 0)
    out = open(a.out, "w") if a.out else None
    tot: dict[str, float] = {}
    for H, cin, cout, k, stride, count in SHAPES:
        pad = k // 2
        Ho = (H + 2 * pad - k) // stride + 1
        x = torch.randn(B, cin, H, H, device=dev).to(memory_format=torch.channels_last)
        w = (torch.randn(cout, cin, k, k, device=dev) * 0.05).to(memory_format=torch.channels_last)
        dy = torch.randn(B, cout, Ho, Ho, device=dev).to(memory_format=torch.channels_last)
        flop = 2.0 * B * Ho * Ho * cout * cin * k * k
        conv = torch.ops.aten.convolution
        bwd = torch.ops.aten.convolution_backward
        args = ([stride, stride], [pad, pad], [1, 1], False, [0, 0], 1)
        rec = {"H": H, "cin": cin, "cout": cout, "k": k, "stride": stride, "count": count, "gflop": round(flop / 1e9, 2)}
        if a.only_1x1 and k != 1:
            continue
        rec["miopen_fwd_us"] = timeit(lambda: conv(x, w, None, *args))
        if cin > 3:
            rec["miopen_dgrad_us"] = timeit(lambda: bwd(dy, x, w, None, *args, [True, False, False]))
        rec["miopen_wgrad_us"] = timeit(lambda: bwd(dy, x, w, None, *args, [False, True, False]))
        if k == 1:
            xs = x if stride == 1 else x[:, :, ::stride, ::stride].contiguous(memory_format=torch.channels_last)
            x2 = xs.permute(0, 2, 3, 1).reshape(-1, cin)
            w2 = w.view(cout, cin)
            dy2 = dy.permute(0, 2, 3, 1).reshape(-1, cout)
            rec["blas_fwd_us"] = timeit(lambda: x2 @ w2.t())
            rec["blas_dgrad_us"] = timeit(lambda: dy2 @ w2)
            rec["blas_wgrad_us"] = timeit(lambda: dy2.t() @ x2)
            # own f32-MFMA kernels (csrc/hip/conv1x1_f32.hip)
            from vodascheduler_amd.ops.conv1x1 import StatsHolder, gemm_f32_2d

            x2c = x2.contiguous()
            if gemm_f32_2d(x2c, w2, StatsHolder()) is not None:
                rec["own_fwd_us"] = timeit(lambda: gemm_f32_2d(x2c, w2, StatsHolder()))
            wt = w2.t().contiguous()
            if gemm_f32_2d(dy2, wt) is not None:
                rec["own_dgrad_us"] = timeit(lambda: gemm_f32_2d(dy2, wt))
        if a.only_1x1 and k != 1:
            continue
        for key in [k_ for k_ in rec if k_.endswith("_us")]:
            rec[key] = round(rec[key], 1)
            rec[key.replace("_us", "_tf")] = round(flop / (rec[key] * 1e-6) / 1e12, 1)
            tot[key] = tot.get(key, 0.0) + rec[key] * count
        line = json.dumps(rec)
        print(line, flush=True)
        if out:
            out.write(line + "\n")
        del x, w, dy
    summary = {"per_step_ms": {k: round(v / 1e3, 2) for k, v in tot.items()}}
    print(json.dumps(summary), flush=True)
    if out:
        out.write(json.dumps(summary) + "\n")


if __name__ == "__main__":
    main()
