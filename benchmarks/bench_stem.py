"""ResNet-50 stem kernels (csrc/hip/stem.hip) at bs 256, 224 x 224: pack, conv forward with
BN statistics, weight gradient -- and MIOpen's forward / weight gradient of the same conv for
reference.  (The round-2 forward-kernel ablation masks were removed in round 5; their results
are in profiles/raw/r2_stem_micro.jsonl.)

python benchmarks/bench_stem.py
"""
from __future__ import annotations

import argparse
import json
import os
import sys

B = 256


def t_us(fn, it=20):
    import torch

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


def run() -> dict:
    import torch
    import torch.nn.functional as F

    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    from vodascheduler_amd.ops import stem as S

    torch.backends.cudnn.benchmark = True
    torch.manual_seed(0)
    x = torch.randn(B, 3, 224, 224, device="cuda").to(memory_format=torch.channels_last)
    w = (torch.randn(64, 3, 7, 7, device="cuda") * 0.05).bfloat16().to(memory_format=torch.channels_last)
    x4 = S.pack_nhwc4(x)
    dyc = torch.randn(B, 64, 112, 112, device="cuda").bfloat16().to(memory_format=torch.channels_last)
    gw = torch.zeros(64, 3, 7, 7, device="cuda").to(memory_format=torch.channels_last)
    h = S.N.hip()
    ws = torch.empty(h.stem_wgrad_workspace_floats(B, 112), dtype=torch.float32, device="cuda")
    out = {"pack_us": t_us(lambda: S.pack_nhwc4(x)),
           "conv_fwd_stats_us": t_us(lambda: S.stem_conv_stats(x4, w, 3))}
    out["wgrad_us"] = t_us(lambda: h.stem_conv_wgrad(x4.data_ptr(), dyc.data_ptr(), gw.data_ptr(), *gw.stride(), 3,
                                                     ws.data_ptr(), B, 224, 224, 112, 112, True, 0,
                                                     S.N.stream_of(x4)))
    xb = x.bfloat16()
    out["miopen_fwd_us"] = t_us(lambda: F.conv2d(xb, w, stride=2, padding=3))
    out["miopen_wgrad_us"] = t_us(lambda: torch.ops.aten.convolution_backward(
        dyc, xb, w, None, [2, 2], [3, 3], [1, 1], False, [0, 0], 1, [False, True, False]))
    return out


def main():
    argparse.ArgumentParser().parse_args()
    print(json.dumps(run()), flush=True)


if __name__ == "__main__":
    main()
