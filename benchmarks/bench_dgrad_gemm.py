"""ResNet-50 stage-1/2 1x1-conv input-gradient GEMMs: hipBLASLt (``dy2 @ w2``, the current
backward) vs the MFMA GEMM of csrc/hip/gemm_bnstats.hip on the same [M x K] . [K x N] product
(its statistics epilogue included, as it would run), to decide whether the backward GEMMs
should move to it.

python benchmarks/bench_dgrad_gemm.py
"""
from __future__ import annotations

import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from vodascheduler_amd.ops import _native as N  # noqa: E402


def timeit(fn, iters=20):
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
    h = N.hip()
    dev = torch.device("cuda", 0)
    # (M, K in, N out): conv3 dgrad stage 1 (256 -> 64), conv1 dgrad stage 1 (64 -> 256),
    # conv1 dgrad of the stage-2 first block at 56x56 (128 -> 256), conv3 dgrad stage 2 (512 -> 128)
    for M, K, Nc in ((802816, 256, 64), (802816, 64, 256), (802816, 128, 256), (200704, 128, 512), (200704, 512, 128)):
        dy = torch.randn(M, K, device=dev).bfloat16()
        w = torch.randn(K, Nc, device=dev).bfloat16()          # dX = dY . W  ([K][N] weight view)
        wt = w.t().contiguous()                                   # [N][K] for the Y = X W^T kernel
        res = {"M": M, "K": K, "N": Nc, "hipblaslt_us": round(timeit(lambda: dy @ w), 1)}
        if h.gemm_bnstats_supported(M, Nc, K):
            G = h.gemm_bnstats_groups(M, Nc, K)
            y = torch.empty(M, Nc, dtype=torch.bfloat16, device=dev)
            ws = torch.empty(max(2 * G * Nc + 3 * Nc, h.bn_workspace_floats(M, Nc)), dtype=torch.float32, device=dev)
            res["mfma_gemm_us"] = round(timeit(lambda: h.gemm_bnstats(dy.data_ptr(), wt.data_ptr(), y.data_ptr(),
                                                                       ws.data_ptr(), M, Nc, K, G,
                                                                       N.stream_of(dy))), 1)
            ref = (dy.float() @ w.float())
            res["rel_err"] = float(((y.float() - ref).norm() / ref.norm()).item())
        print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
