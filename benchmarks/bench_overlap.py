"""Does a Linear layer's weight gradient overlap with the next input-gradient GEMM?

Times, on the BERT-base fc1 shapes (8192 tokens, 768 -> 3072), the split-K MFMA weight
gradient (ops/wgrad.py) and a hipBLASLt input-gradient GEMM of the same layer alone, back to
back on one stream, and on two streams at once.  The gap between "sequential" and
"concurrent" is what moving the weight gradients to a side stream could recover in the step.

python benchmarks/bench_overlap.py [--iters 50]
"""
from __future__ import annotations

import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from vodascheduler_amd.ops import wgrad as W  # noqa: E402


def timed(fn, iters: int) -> float:
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(iters):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / iters * 1e3


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--iters", type=int, default=50)
    a = ap.parse_args()
    dev = torch.device("cuda", 0)
    M, n_out, K = 8192, 3072, 768
    dy = torch.randn(M, n_out, device=dev).bfloat16()
    x = torch.randn(M, K, device=dev).bfloat16()
    w = torch.randn(n_out, K, device=dev).bfloat16()
    gw = torch.zeros(n_out, K, device=dev)
    gb = torch.zeros(n_out, device=dev)
    side = torch.cuda.Stream(dev)
    main_s = torch.cuda.current_stream(dev)

    def dgrad():
        return dy @ w

    def wgrad():
        W.wgrad_accumulate_(dy, x, gw, gb)

    def seq():
        dgrad()
        wgrad()

    def conc():
        side.wait_stream(main_s)
        with torch.cuda.stream(side):
            wgrad()
        dgrad()
        main_s.wait_stream(side)

    res = {"shape": [M, n_out, K], "dgrad_us": timed(dgrad, a.iters), "wgrad_us": timed(wgrad, a.iters),
           "sequential_us": timed(seq, a.iters), "concurrent_us": timed(conc, a.iters)}
    res["overlap_gain"] = round(1 - res["concurrent_us"] / res["sequential_us"], 3)
    print(json.dumps({k: (round(v, 2) if isinstance(v, float) else v) for k, v in res.items()}), flush=True)


if __name__ == "__main__":
    main()
