"""Probe: the exact 3-way bf16 split as ONE bf16 GEMM with the six kept cross products
concatenated along K (A' = [Al Am Ah Am Ah Ah], B' = [Bh Bh Bl Bm Bm Bh]: corrections first,
hi.hi last), fp32 output / accumulate, vs hipBLASLt fp32 and the own split kernel
(csrc/hip/splitgemm.hip) on the BERT-base projection shapes (M = 8192 tokens).

Times the GEMM alone (``torch.mm(..., out_dtype=torch.float32)``), plain bf16 at K and 6K (the
library's raw rate), and reports the error vs fp64 like bench_splitgemm.py.

    python benchmarks/probe_kconcat.py [--out gpurun_out/kconcat.jsonl]
"""
from __future__ import annotations

import argparse
import json
import os
import statistics
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(__file__), ".."))
from benchmarks.bench_splitgemm import LINEARS, M, err, operands, timeit  # noqa: E402
from vodascheduler_amd.ops import splitgemm as SG  # noqa: E402

torch.backends.cuda.matmul.allow_tf32 = False

# (plane of A, plane of B) per K segment: small corrections first, hi.hi last
ORDER = ((2, 0), (1, 0), (0, 2), (1, 1), (0, 1), (0, 0))


def planes(t: torch.Tensor) -> list[torch.Tensor]:
    return [p.to(torch.bfloat16) for p in SG.split3(t)]


def kconcat(a: torch.Tensor, b: torch.Tensor) -> tuple[torch.Tensor, torch.Tensor]:
    """a [M, K], b [K, N] fp32 -> a' [M, 6K], b' [6K, N] bf16 (any input strides)."""
    pa, pb = planes(a), planes(b)
    a2 = torch.cat([pa[i] for i, _ in ORDER], dim=1)
    b2 = torch.cat([pb[j] for _, j in ORDER], dim=0)
    return a2, b2


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=20)
    ap.add_argument("--out", default="")
    args = ap.parse_args()
    dev = torch.device("cuda", 0)
    sink = open(args.out, "a") if args.out else None

    def emit(rec):
        line = json.dumps(rec)
        print(line, flush=True)
        if sink:
            sink.write(line + "\n")
            sink.flush()

    for name, (k_in, n_out) in LINEARS.items():
        for op in ("fwd", "dgrad", "wgrad"):
            a, b = operands(op, k_in, n_out, dev, False, 1)
            Mo, Ko = a.shape
            No = b.shape[1]
            flops = 2.0 * Mo * No * Ko
            out = torch.empty(Mo, No, device=dev)
            # the concatenated operands in the orientation the op has: for the weight gradient
            # the planes stack along the token rows (K-major A / B), for fwd / dgrad along k
            a2, b2 = kconcat(a, b)
            if op == "wgrad":
                a2 = a2.t().contiguous().t()  # [M, 6K] view of a [6K, M] buffer (dY planes stacked)
                b2 = b2.contiguous()
            else:
                a2 = a2.contiguous()
                b2 = b2.t().contiguous().t() if op == "fwd" else b2.contiguous()
            ab, bb = a.to(torch.bfloat16), b.to(torch.bfloat16)
            fns = {
                "hipblaslt_fp32": lambda: torch.mm(a, b, out=out),
                "own_split": lambda: SG.matmul(a, b, out=out),
                "kconcat_bf16_f32out": lambda: torch.mm(a2, b2, out_dtype=torch.float32),
                "bf16_K": lambda: torch.mm(ab, bb),
                "bf16_K_f32out": lambda: torch.mm(ab, bb, out_dtype=torch.float32),
                "split_prepass_torch": lambda: kconcat(a, b),
            }
            for f in fns.values():
                f()
            torch.cuda.synchronize()
            times = {k: [] for k in fns}
            for _ in range(3):
                for k, f in fns.items():
                    times[k].append(timeit(f, args.reps))
            base = statistics.median(times["hipblaslt_fp32"])
            for k, ts in times.items():
                us = statistics.median(ts)
                fl = flops * (6 if k.startswith("kconcat") else 1)
                emit({"linear": name, "op": op, "M": Mo, "N": No, "K": Ko, "cand": k, "us": round(us, 2),
                      "tflops_fp32_equiv": round(flops / us / 1e6, 1), "tflops_issued": round(fl / us / 1e6, 1),
                      "speedup_vs_hipblaslt": round(base / us, 3)})
            for wide in (False, True):
                a3, b3 = operands(op, k_in, n_out, dev, wide, 2)
                x2, y2 = kconcat(a3, b3)
                res = {"hipblaslt_fp32": err(torch.mm(a3, b3), a3, b3),
                       "own_split": err(SG.matmul(a3, b3), a3, b3),
                       "kconcat": err(torch.mm(x2, y2, out_dtype=torch.float32), a3, b3)}
                for k, (comp, fro) in res.items():
                    emit({"linear": name, "op": op, "inputs": "wide2^30" if wide else "normal", "cand": k,
                          "err_comp": comp, "err_fro": fro,
                          "ratio_vs_hipblaslt": comp / max(res["hipblaslt_fp32"][0], 1e-300)})
            del a, b, a2, b2, out
            torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
