"""Split-K count sweep of ResNet-50 bs256 fp32 weight gradients on the split-bf16 kernel: the 1x1
layers (dW = dY^T X over the pixels, tiles as ops/conv1x1 picks them) and the 3x3 implicit-GEMM
ones (C >= 128), at 0.25 / 0.375 / 0.5 / 0.75 / 1 x (or --factors) the shipped split count, in the
shipped kernel forms (variant 8 / conv mode 3 on 128 x 128 tiles).  us per (shape, splits).

    python benchmarks/probe_resnet_wgrad_splits.py [--out gpurun_out/rwsplits.jsonl]
"""
from __future__ import annotations

import argparse
import json
import os
import statistics
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(__file__), ".."))
from benchmarks.bench_splitgemm import timeit  # noqa: E402
from vodascheduler_amd.ops import conv1x1 as C1  # noqa: E402
from vodascheduler_amd.ops import splitgemm as SG  # noqa: E402

FACTORS = (0.25, 0.375, 0.5, 0.75, 1.0)

ONE = [(64, 256, 802816), (256, 64, 802816), (128, 256, 802816), (512, 128, 200704), (128, 512, 200704),
       (1024, 256, 50176), (256, 1024, 50176), (2048, 512, 12544), (512, 2048, 12544)]
THREE = [(128, 28, 1, 28), (256, 14, 1, 14), (512, 7, 1, 7), (128, 28, 2, 56), (256, 14, 2, 28),
         (512, 7, 2, 14)]  # (C, Ho, stride, H)


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("--out", default="")
    ap.add_argument("--factors", default="", help="comma list of multiples of the shipped split count")
    args = ap.parse_args()
    global FACTORS
    if args.factors:
        FACTORS = tuple(float(f) for f in args.factors.split(","))
    dev = torch.device("cuda", 0)
    sink = open(args.out, "a") if args.out else None

    def emit(rec):
        print(json.dumps(rec), flush=True)
        if sink:
            sink.write(json.dumps(rec) + "\n")

    for cout, cin, m in ONE:
        dy = torch.randn(m, cout, device=dev)
        x = torch.randn(m, cin, device=dev)
        g = torch.zeros(cout, cin, device=dev)
        tile = SG.thin_tile(cout, cin)
        s0 = SG.conv_wgrad_splits(cout, cin, m, tile, C1.WGRAD_TARGET_WG)
        ss = sorted({max(1, int(s0 * f)) for f in FACTORS})
        v = 8 if C1.WGRAD_V8 and tile == 0 else None
        fns = {s: (lambda s=s: SG.matmul(dy.t(), x, out=g, accumulate=True, tile=tile, splits=s, variant=v))
               for s in ss}
        for f in fns.values():
            f()
        torch.cuda.synchronize()
        ts = {s: statistics.median([timeit(f, 5) for _ in range(3)]) for s, f in fns.items()}
        for s, us in ts.items():
            emit({"kind": "1x1", "cout": cout, "cin": cin, "M": m, "tile": tile, "splits": s, "shipped": s == s0,
                  "us": round(us, 2)})
        del dy, x, g
        torch.cuda.empty_cache()
    cl = torch.channels_last
    for c, ho, stride, h in THREE:
        x = torch.randn(256, c, h, h, device=dev).contiguous(memory_format=cl)
        dy = torch.randn(256, c, ho, ho, device=dev).contiguous(memory_format=cl)
        gw = torch.zeros(c, c, 3, 3, device=dev).contiguous(memory_format=cl)
        s0 = SG.conv_wgrad_splits(c, 9 * c, 256 * ho * ho)
        ss = sorted({max(1, int(s0 * f)) for f in FACTORS})
        fns = {s: (lambda s=s: SG.conv_wgrad_(dy, x, gw, stride, 1, splits=s)) for s in ss}
        for f in fns.values():
            f()
        torch.cuda.synchronize()
        ts = {s: statistics.median([timeit(f, 5) for _ in range(3)]) for s, f in fns.items()}
        for s, us in ts.items():
            emit({"kind": "3x3", "C": c, "Ho": ho, "stride": stride, "splits": s, "shipped": s == s0, "us": round(us, 2)})
        del x, dy, gw
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
