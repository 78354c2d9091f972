"""Split-K count sweep of the BERT-base fp32 weight-gradient GEMMs (dW = dY^T X over 8192 tokens,
both operands K-major) on the split-bf16 kernel: us per (shape, tile, splits), reduce included.

    python benchmarks/probe_wgrad_splits.py [--out gpurun_out/wsplits.jsonl]
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


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("--out", default="")
    args = ap.parse_args()
    dev = torch.device("cuda", 0)
    sink = open(args.out, "a") if args.out else None
    for n_out, k_in in ((2304, 768), (768, 768), (3072, 768), (768, 3072)):
        dy = torch.randn(8192, n_out, device=dev)
        x = torch.randn(8192, k_in, device=dev)
        a, b = dy.t(), x
        out = torch.zeros(n_out, k_in, device=dev)
        cands = {}
        for tile in (0, 7):
            if tile == 7 and k_in % 96:
                continue
            for s in (2, 3, 4, 5, 6, 7, 8, 10, 12, 16):
                cands[(tile, s)] = (lambda tile=tile, s=s: SG.matmul(a, b, out=out, accumulate=True, tile=tile, splits=s))
        for f in cands.values():
            f()
        torch.cuda.synchronize()
        times = {k: [] for k in cands}
        for _ in range(3):
            for k, f in cands.items():
                times[k].append(timeit(f, 10))
        for (tile, s), ts in times.items():
            rec = {"M": n_out, "N": k_in, "K": 8192, "tile": tile, "splits": s, "us": round(statistics.median(ts), 2),
                   "chosen": SG.choose(n_out, k_in, 8192) == (tile, s)}
            print(json.dumps(rec), flush=True)
            if sink:
                sink.write(json.dumps(rec) + "\n")
        del dy, x, out
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
