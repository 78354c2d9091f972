"""ResNet-50 bs256 fp32 1x1 forwards with K = 64 / 128 / 256 input channels: the own f32-MFMA
GEMM with the BN-statistics epilogue (conv1x1_f32.hip, the shipped path) against the split-bf16
GEMM (splitgemm.hip) without statistics, over tiles 0 / 5 / 6 and both math variants.  Tells
whether a statistics epilogue on the split kernel would pay.  One JSON line per (shape, cand).

    python benchmarks/bench_1x1_small_k.py [--out gpurun_out/smallk.jsonl]
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

# (M pixels, K = Cin, N = Cout, calls per step) of the stride-1 1x1 forwards on gemm_f32_stats
SHAPES = [(802816, 64, 64, 1), (802816, 64, 256, 4), (802816, 256, 64, 2), (802816, 256, 128, 1),
          (200704, 128, 512, 4), (200704, 256, 512, 1), (50176, 256, 1024, 6), (12544, 512, 2048, 0),
          (200704, 512, 128, 0)]


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("--out", default="")
    ap.add_argument("--reps", type=int, default=10)
    args = ap.parse_args()
    dev = torch.device("cuda", 0)
    sink = open(args.out, "a") if args.out else None
    for M, K, Nn, calls in SHAPES:
        g = torch.Generator(device=dev).manual_seed(M + K + Nn)
        x = torch.randn(M, K, device=dev, generator=g)
        w = torch.randn(Nn, K, device=dev, generator=g) * 0.05
        out = torch.empty(M, Nn, device=dev)
        cands = {}
        if N_ok := C1.N.hip().gemm_f32_stats_supported(M, Nn, K):
            cands["f32_stats"] = lambda: C1.gemm_f32_2d(x, w, C1.StatsHolder())
            cands["f32_nostats"] = lambda: C1.gemm_f32_2d(x, w, None)
        for tile in (0, 5, 6):
            bm, bn = SG.TILES[tile]
            if (tile == 5 and Nn % 256) or (tile == 6 and Nn != 64):
                continue
            for v in (0, 1):
                if v == 1 and tile != 0:
                    continue
                cands[f"split_t{tile}_v{v}"] = (lambda tile=tile, v=v:
                                                SG.matmul(x, w.t(), out=out, tile=tile, splits=1, variant=v))
        for f in cands.values():
            f()
        torch.cuda.synchronize()
        times = {k: [] for k in cands}
        for _ in range(3):
            for k, f in cands.items():
                times[k].append(timeit(f, args.reps))
        mb = (M * K + M * Nn) * 4 / 1e6
        for k, ts in times.items():
            us = statistics.median(ts)
            rec = {"M": M, "K": K, "N": Nn, "calls": calls, "cand": k, "us": round(us, 2),
                   "tflops": round(2.0 * M * K * Nn / us / 1e6, 1), "hbm_floor_us": round(mb / 6.0, 1),
                   "f32_supported": bool(N_ok)}
            line = json.dumps(rec)
            print(line, flush=True)
            if sink:
                sink.write(line + "\n")
                sink.flush()
        del x, w, out
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
