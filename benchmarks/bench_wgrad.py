"""Weight-gradient GEMM microbenchmark on MI355X: hipBLASLt (``addmm_`` with beta = 1, as
stock autograd accumulation does) + the column-sum kernel vs the split-K MFMA kernel of
csrc/hip/wgrad.hip with the fused bias gradient, on the BERT-base Linear shapes.

python benchmarks/bench_wgrad.py [--splits 1,2,4,8]
"""
from __future__ import annotations

import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from vodascheduler_amd.ops import _native  # noqa: E402
from vodascheduler_amd.ops import wgrad as W  # noqa: E402
from vodascheduler_amd.ops.dense import colsum_accumulate_  # noqa: E402

# (name, tokens M, out features N, in features K): BERT-base seq 128 x batch 64
SHAPES = [("qkv", 8192, 2304, 768), ("attn_out", 8192, 768, 768), ("fc1", 8192, 3072, 768),
          ("fc2", 8192, 768, 3072), ("mlm_dense", 1280, 768, 768)]


def timeit(fn, iters=50, warm=5) -> float:
    for _ in range(warm):
        fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(iters):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / iters * 1e3  # us


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--splits", default="1,2,3,4,6,8,12,16,28")
    ap.add_argument("--variants", default="2,4,6,7,8")
    a = ap.parse_args()
    _native.hip()
    dev = torch.device("cuda", 0)
    out = []
    for name, M, N, K in SHAPES:
        dy = torch.randn(M, N, device=dev).bfloat16()
        x = torch.randn(M, K, device=dev).bfloat16()
        gw = torch.zeros(N, K, device=dev, dtype=torch.bfloat16)
        gb = torch.zeros(N, device=dev, dtype=torch.bfloat16)
        tf = 2.0 * M * N * K / 1e12
        t_blas = timeit(lambda: gw.addmm_(dy.t(), x))
        t_blas_b = timeit(lambda: (gw.addmm_(dy.t(), x), colsum_accumulate_(dy, gb)))
        res = {"shape": name, "M": M, "N": N, "K": K, "hipblaslt_us": round(t_blas, 2),
               "hipblaslt_tflops": round(tf / (t_blas * 1e-6), 1), "hipblaslt+colsum_us": round(t_blas_b, 2),
               "default_splits": W.default_splits(M, N, K)}
        res["wide_default_splits"] = W.default_splits(M, N, K, variant=6)
        # correctness of the default configuration against fp32
        gw.normal_()
        gb.normal_()
        w_ref, b_ref = W.wgrad_ref(dy, x, gw, gb)
        W.wgrad_accumulate_(dy, x, gw, gb)
        res["max_rel_err"] = float(((gw.float() - w_ref).norm() / w_ref.norm()).item())
        for v in [int(v_) for v_ in a.variants.split(",")]:
            for s in [int(x_) for x_ in a.splits.split(",")]:
                t = timeit(lambda: W.wgrad_accumulate_(dy, x, gw, gb, splits=s, variant=v))
                res[f"hip_v{v}_s{s}_us"] = round(t, 2)
        best = min((v, k) for k, v in res.items() if k.startswith("hip_v"))
        res["hip_best"] = best[1]
        res["hip_best_tflops"] = round(tf / (best[0] * 1e-6), 1)
        res["hip_default_us"] = res.get(f"hip_v{W.VARIANT}_s{res['default_splits']}_us")
        res["speedup_vs_hipblaslt+colsum"] = round(t_blas_b / best[0], 2)
        print(json.dumps(res), flush=True)
        out.append(res)
    tot_b = sum(r["hipblaslt+colsum_us"] for r in out[:4]) * 12 + out[4]["hipblaslt+colsum_us"]
    tot_h = sum(r["hip_default_us"] or 0 for r in out[:4]) * 12 + (out[4]["hip_default_us"] or 0)
    print(json.dumps({"bert_base_step_wgrad_ms": {"hipblaslt+colsum": round(tot_b / 1e3, 3),
                                                  "hip_default": round(tot_h / 1e3, 3)}}), flush=True)


if __name__ == "__main__":
    main()
