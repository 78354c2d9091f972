"""Runs one split-bf16 GEMM shape (and hipBLASLt fp32 on it) a few times: the target of the
rocprofv3 counter passes in benchmarks/pmc_splitgemm.sh.

    python benchmarks/sgemm_one.py --shape 8192,2304,768 --op fwd --variants 1,4 --reps 5
"""
from __future__ import annotations

import argparse
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(__file__), ".."))
from vodascheduler_amd.ops import splitgemm as SG  # noqa: E402


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("--shape", default="8192,2304,768", help="M,N,K of the GEMM")
    ap.add_argument("--op", default="fwd", choices=["fwd", "dgrad", "wgrad"])
    ap.add_argument("--variants", default="0")
    ap.add_argument("--tile", type=int, default=-1)
    ap.add_argument("--splits", type=int, default=0)
    ap.add_argument("--reps", type=int, default=5)
    ap.add_argument("--blas", action="store_true")
    a = ap.parse_args()
    torch.backends.cuda.matmul.allow_tf32 = False
    M, Nn, K = (int(v) for v in a.shape.split(","))
    dev = torch.device("cuda", 0)
    g = torch.Generator(device=dev).manual_seed(0)
    if a.op == "fwd":      # a [M, K] K-contiguous, b = W^T (K-contiguous)
        x, w = torch.randn(M, K, device=dev, generator=g), torch.randn(Nn, K, device=dev, generator=g)
        A, B = x, w.t()
    elif a.op == "dgrad":  # b = W [K, N] row-major: K-major
        A, B = torch.randn(M, K, device=dev, generator=g), torch.randn(K, Nn, device=dev, generator=g)
    else:                  # a = dY^T (K-major), b = X (K-major)
        A = torch.randn(K, M, device=dev, generator=g).t()
        B = torch.randn(K, Nn, device=dev, generator=g)
    out = torch.empty(M, Nn, device=dev)
    kw = {}
    if a.tile >= 0:
        kw["tile"] = a.tile
    if a.splits > 0:
        kw["splits"] = a.splits
    for _ in range(a.reps):
        for v in (int(t) for t in a.variants.split(",") if t):
            SG.matmul(A, B, out=out, variant=v, **kw)
        if a.blas:
            torch.mm(A, B, out=out)
    torch.cuda.synchronize()


if __name__ == "__main__":
    main()
