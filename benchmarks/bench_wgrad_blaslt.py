"""bf16 Linear weight gradients into fp32 flat gradients, BERT-base bs64 x seq128 shapes:

  own      the split-K MFMA kernel with the fused bias column sum (ops/wgrad.py, the bf16 default)
  blaslt   hipBLASLt bf16 x bf16 -> fp32 with beta = 1 straight into the fp32 gradient and the
           bias gradient in the BGRADB epilogue (csrc/hip/blaslt_epi.cpp gemm_wgrad_f32acc)
           + one vector add of the bias gradient

Prints one JSON line per shape: us per call and relative errors vs fp64.
python benchmarks/bench_wgrad_blaslt.py
"""
from __future__ import annotations

import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from vodascheduler_amd.ops import _native as N  # noqa: E402
from vodascheduler_amd.ops import ffn  # noqa: E402
from vodascheduler_amd.ops import wgrad as W  # noqa: E402


def timeit(fn, reps=40):
    for _ in range(5):
        fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) * 1e3 / reps


def rel(a, b):
    return float(((a.double() - b).norm() / (b.norm() + 1e-30)).item())


def blaslt(dy, x, gw, gb, tmp):
    M, Nn = dy.shape
    K = x.shape[1]
    ws = ffn._workspace(dy.device)
    N.hip().gemm_wgrad_f32acc(dy.data_ptr(), Nn, x.data_ptr(), K, gw.data_ptr(), K, tmp.data_ptr() if gb is not None
                              else 0, M, Nn, K, N.dtype_code(dy.dtype), True, ws.data_ptr(), ws.numel(),
                              N.stream_of(dy))
    if gb is not None:
        gb.add_(tmp)


def main():
    dev = torch.device("cuda", 0)
    torch.manual_seed(0)
    for M, Nn, K, name, count in ((8192, 2304, 768, "qkv", 12), (8192, 768, 768, "attn_out", 12),
                                  (8192, 3072, 768, "fc1", 12), (8192, 768, 3072, "fc2", 12),
                                  (8192, 768, 768, "mlm_dense", 1), (1280, 30528, 768, "mlm_decoder", 1)):
        dy = torch.randn(M, Nn, device=dev).to(torch.bfloat16)
        x = torch.randn(M, K, device=dev).to(torch.bfloat16)
        base_w = torch.randn(Nn, K, device=dev)
        base_b = torch.randn(Nn, device=dev)
        ref_w = base_w.double() + dy.double().t() @ x.double()
        ref_b = base_b.double() + dy.double().sum(0)
        row = {"name": name, "M": M, "N": Nn, "K": K, "per_step": count}
        gw, gb = base_w.clone(), base_b.clone()
        W.wgrad_accumulate_(dy, x, gw, gb)
        row["own_relerr_w"], row["own_relerr_b"] = rel(gw, ref_w), rel(gb, ref_b)
        row["own_us"] = round(timeit(lambda: W.wgrad_accumulate_(dy, x, gw, gb)), 2)
        tmp = torch.empty(Nn, device=dev)
        try:
            gw = base_w.clone()
            blaslt(dy, x, gw, None, tmp)
            row["blaslt_nobias_relerr_w"] = rel(gw, ref_w)
            row["blaslt_nobias_us"] = round(timeit(lambda: blaslt(dy, x, gw, None, tmp)), 2)
        except (RuntimeError, ValueError) as e:
            row["nobias_error"] = str(e)[:200]
        try:
            gw, gb = base_w.clone(), base_b.clone()
            blaslt(dy, x, gw, gb, tmp)
            row["blaslt_relerr_w"], row["blaslt_relerr_b"] = rel(gw, ref_w), rel(gb, ref_b)
            row["blaslt_us"] = round(timeit(lambda: blaslt(dy, x, gw, gb, tmp)), 2)
        except (RuntimeError, ValueError) as e:
            row["bias_error"] = str(e)[:200]
        # reference points: torch's bf16 GEMM (bf16 out) and the fp32-out variant if available
        row["torch_bf16_mm_us"] = round(timeit(lambda: dy.t() @ x), 2)
        try:
            row["torch_mm_outf32_us"] = round(timeit(lambda: torch.mm(dy.t(), x, out_dtype=torch.float32)), 2)
        except (RuntimeError, TypeError) as e:
            row["torch_mm_outf32_error"] = str(e)[:120]
        print(json.dumps(row), flush=True)


if __name__ == "__main__":
    main()
