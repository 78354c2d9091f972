"""BERT-base fp32 forward GEMMs y = x W^T (+ b) on the split GEMM: the shipped K-contiguous B
(W^T as a view of the [N, K] weight) against a K-major copy of W^T ([K, N] row-major, refreshed
once per optimizer step) that lets the forward take variant 8 (three workgroups per CU, as the
input gradients do).  Prices the copy too.  One JSON line per (shape, candidate).

    python benchmarks/probe_fwd_kmajor.py [--out gpurun_out/fwd_kmajor.jsonl]
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

# (name, M tokens, K in, N out, GELU epilogue)
SHAPES = [("qkv", 8192, 768, 2304, False), ("o", 8192, 768, 768, False), ("fc1", 8192, 768, 3072, True),
          ("fc2", 8192, 3072, 768, False)]


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("--out", default="")
    ap.add_argument("--reps", type=int, default=20)
    args = ap.parse_args()
    dev = torch.device("cuda", 0)
    sink = open(args.out, "a") if args.out else None
    for name, M, K, Nn, gelu in SHAPES:
        g = torch.Generator(device=dev).manual_seed(M + K + Nn)
        x = torch.randn(M, K, device=dev, generator=g)
        w = torch.randn(Nn, K, device=dev, generator=g) * 0.05
        b = torch.randn(Nn, device=dev, generator=g)
        wt = w.t().contiguous()
        out = torch.empty(M, Nn, device=dev)
        aux = torch.empty(M, Nn, device=dev) if gelu else None
        epi = SG.EPI_GELU if gelu else SG.EPI_NONE
        ref = x.double() @ w.double().t() + b.double()
        cands = {"cur": lambda: SG.matmul(x, w.t(), out=out, bias=b, epi=epi, aux=aux),
                 "transpose_copy": lambda: wt.copy_(w.t())}
        for v in (0, 8):
            for s in (1, 2):
                cands[f"kmaj_v{v}_s{s}"] = (lambda v=v, s=s: SG.matmul(x, wt, out=out, bias=b, epi=epi, aux=aux,
                                                                      tile=0, splits=s, variant=v))
        cands["kmaj_plan"] = lambda: SG.matmul(x, wt, out=out, bias=b, epi=epi, aux=aux)
        for s in (1, 2):  # the shipped K-contiguous B on variant 8 (three workgroups per CU once the
            # K-contiguous images are 96-B pitch)
            cands[f"kc_v8_s{s}"] = (lambda s=s: SG.matmul(x, w.t(), out=out, bias=b, epi=epi, aux=aux,
                                                         tile=0, splits=s, variant=8))
        errs = {}
        for k, f in cands.items():
            f()
            if k != "transpose_copy":
                torch.cuda.synchronize()
                y = aux if gelu else out
                errs[k] = ((y.double() - ref).abs().max() / ref.abs().max()).item()
        torch.cuda.synchronize()
        times = {k: [] for k in cands}
        for _ in range(3):
            for k, f in cands.items():
                times[k].append(timeit(f, args.reps))
        for k, ts in times.items():
            rec = {"shape": name, "M": M, "K": K, "N": Nn, "gelu": gelu, "cand": k,
                   "us": round(statistics.median(ts), 2), "rel_err": errs.get(k)}
            line = json.dumps(rec)
            print(line, flush=True)
            if sink:
                sink.write(line + "\n")
                sink.flush()


if __name__ == "__main__":
    main()
