"""fp32 3x3 stride-1 forward convolution of ResNet-50's bottlenecks at batch 256: the own
Winograd F(2x2, 3x3) kernel (filter transform included) vs MIOpen through F.conv2d (channels_last,
the models' layout).  One JSON line per shape: us, effective TF of the direct convolution's
FLOPs, relative error vs fp64 on a slice.

python benchmarks/bench_winograd.py [--batch 256]
"""
from __future__ import annotations

import argparse
import json
import os
import sys

import torch
import torch.nn.functional as F

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from vodascheduler_amd.ops import winograd as Wg  # noqa: E402


def timeit(fn, reps=20):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) * 1e3 / reps


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=256)
    a = ap.parse_args()
    torch.backends.cudnn.benchmark = False
    for c, h in ((64, 56), (128, 28), (256, 14), (512, 7)):
        n = a.batch
        x = torch.randn(n, c, h, h, device="cuda").contiguous(memory_format=torch.channels_last)
        w = (torch.randn(c, c, 3, 3, device="cuda") / (3 * c ** 0.5)).contiguous(memory_format=torch.channels_last)
        gf = 2.0 * n * h * h * c * c * 9 / 1e9
        row = {"C": c, "H": h, "N": n, "gflop_direct": round(gf, 1)}
        ref = F.conv2d(x[:2].double(), w.double(), None, 1, 1)
        # f32 MFMA / split-bf16 tile GEMMs at 32 (sx) and 64 (sx2) output channels per workgroup
        for tag, sx, wide, onepos in (("", False, False, True), ("_sx", True, False, False), ("_sx1p", True, False, True),
                                      ("_sx2", True, True, True)):
            Wg.USE_WIDE = wide
            Wg.ONEPOS = onepos
            u = Wg.filter_transform(w, sx=sx)
            y = Wg.conv3x3_wino(x, w, u)
            row["relerr_vs_fp64" + tag] = float(((y[:2].double() - ref).norm() / ref.norm()).item())
            row["wino_us" + tag] = round(timeit(lambda: Wg.conv3x3_wino(x, w, u)), 1)
            row["wino_filter_us" + tag] = round(timeit(lambda: Wg.filter_transform(w, sx=sx)), 1)
            row["wino_eff_tf" + tag] = round(gf / row["wino_us" + tag] * 1e3, 1)
        row["miopen_us"] = round(timeit(lambda: F.conv2d(x, w, None, 1, 1)), 1)
        row["miopen_tf"] = round(gf / row["miopen_us"] * 1e3, 1)
        print(json.dumps(row), flush=True)


if __name__ == "__main__":
    main()
