"""One wgrad kernel configuration in a loop (for rocprofv3 counter passes).

python benchmarks/wgrad_one.py --M 8192 --N 768 --K 768 --splits 1 --variant 0 --iters 20
"""
import argparse
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from vodascheduler_amd.ops import wgrad as W  # noqa: E402

ap = argparse.ArgumentParser()
for k, d in (("M", 8192), ("N", 768), ("K", 768), ("splits", 1), ("variant", 0), ("iters", 20)):
    ap.add_argument(f"--{k}", type=int, default=d)
a = ap.parse_args()
dy = torch.randn(a.M, a.N, device="cuda").bfloat16()
x = torch.randn(a.M, a.K, device="cuda").bfloat16()
gw = torch.zeros(a.N, a.K, device="cuda", dtype=torch.bfloat16)
gb = torch.zeros(a.N, device="cuda", dtype=torch.bfloat16)
for _ in range(a.iters):
    W.wgrad_accumulate_(dy, x, gw, gb, splits=a.splits, variant=a.variant)
torch.cuda.synchronize()
print("done", float(gw.float().abs().sum()))
