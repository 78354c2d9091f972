"""The fp32 1x1-convolution GEMMs of a ResNet-50 bs256 step that still run on hipBLASLt
(forwards with K >= 512 input channels, input gradients with K = Cout >= 512) against the
split-bf16 MFMA GEMM (csrc/hip/splitgemm.hip) over a few (tile, splits, variant) choices.
One JSON line per (shape, candidate): median us over interleaved rounds.

    python benchmarks/bench_resnet_1x1_split.py [--out gpurun_out/r1x1.jsonl]
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
from vodascheduler_amd.ops import splitgemm as SG  # noqa: E402

torch.backends.cuda.matmul.allow_tf32 = False

# (op, M, K, N, calls per step): fwd Y[M, N] = X[M, K] . W[N, K]^T; dgrad dX[M, N] = dY[M, K] . W[K, N]
SHAPES = [
    ("fwd", 200704, 512, 128, 3), ("fwd", 200704, 512, 256, 1), ("fwd", 50176, 512, 1024, 1),
    ("fwd", 50176, 1024, 256, 5), ("fwd", 50176, 1024, 512, 1), ("fwd", 12544, 1024, 2048, 1),
    ("fwd", 12544, 2048, 512, 2),
    ("dgrad", 200704, 512, 128, 4), ("dgrad", 50176, 512, 256, 1), ("dgrad", 50176, 1024, 256, 6),
    ("dgrad", 50176, 1024, 512, 1), ("dgrad", 12544, 2048, 512, 3), ("dgrad", 12544, 2048, 1024, 1),
]


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("--out", default="")
    ap.add_argument("--reps", type=int, default=10)
    args = ap.parse_args()
    dev = torch.device("cuda", 0)
    sink = open(args.out, "a") if args.out else None
    for op, M, K, Nn, calls in SHAPES:
        g = torch.Generator(device=dev).manual_seed(M + K + Nn)
        a = torch.randn(M, K, device=dev, generator=g)
        if op == "fwd":
            w = torch.randn(Nn, K, device=dev, generator=g) * 0.05
            b = w.t()
        else:
            b = torch.randn(K, Nn, device=dev, generator=g) * 0.05  # W [Cout][Cin], row-major
        out = torch.empty(M, Nn, device=dev)
        t0, s0 = SG.choose(M, Nn, K)
        cands = {"hipblaslt": lambda: torch.mm(a, b, out=out)}
        for tile in (0, 1, 2):
            for s in sorted({1, 2, s0}):
                for v in ((0, 1) if tile == 0 else (0,)):
                    cands[f"t{tile}_s{s}_v{v}"] = (lambda tile=tile, s=s, v=v:
                                                   SG.matmul(a, b, out=out, tile=tile, splits=s, variant=v))
        for f in cands.values():
            f()
        torch.cuda.synchronize()
        times = {k: [] for k in cands}
        for _ in range(3):
            for k, f in cands.items():
                times[k].append(timeit(f, args.reps))
        base = statistics.median(times["hipblaslt"])
        ref = torch.mm(a.double(), b.double())
        for k, ts in times.items():
            us = statistics.median(ts)
            rec = {"op": op, "M": M, "K": K, "N": Nn, "calls": calls, "cand": k, "us": round(us, 2),
                   "tflops": round(2.0 * M * K * Nn / us / 1e6, 1), "speedup_vs_hipblaslt": round(base / us, 3)}
            if k != "hipblaslt":
                cands[k]()
                rec["max_rel_err"] = float(((out.double() - ref).abs().max() / ref.abs().max()).item())
            line = json.dumps(rec)
            print(line, flush=True)
            if sink:
                sink.write(line + "\n")
                sink.flush()
        del a, b, out, ref
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
