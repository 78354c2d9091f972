"""Bias gradients in hipBLASLt epilogues (fp32, BERT-base bs64 x seq128 shapes).

  dgelu:  gemm_dgelu + column-sum pass (today)  vs  gemm_dgelu_bgrad (DGELU_BGRAD) + vector add
  wgrad:  addmm_ into the flat gradient + column-sum pass (today)
          vs  gemm_wgrad_bgrad (BGRADB, beta = 1) + vector add

Prints one JSON line per shape (us per call, max relative error vs fp64) and the heuristic's
algorithm counts.  Run on the GPU box:  python benchmarks/bench_blaslt_bgrad.py
"""
from __future__ import annotations

import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from vodascheduler_amd.ops import _native as N  # noqa: E402
from vodascheduler_amd.ops import dense as D  # noqa: E402
from vodascheduler_amd.ops import ffn  # noqa: E402
from vodascheduler_amd.utils import tunable  # noqa: E402


def timeit(fn, reps=30):
    for _ in range(3):
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
    return ((a.double() - b).norm() / (b.norm() + 1e-30)).item()


def main():
    try:
        print(json.dumps({"tunableop": tunable.configure("fp32")}))
    except Exception as e:  # noqa: BLE001
        print(json.dumps({"tunableop": f"not enabled: {e}"}))
    h = N.hip()
    dev = torch.device("cuda", 0)
    print(json.dumps({"algos": {
        "dgelu_bgrad_f32": h.gemm_epilogue_algos(ffn.EPI_DGELU_BGRAD, 0, False, False, 3072, 8192, 768),
        "bgradb_f32_768x2304": h.gemm_epilogue_algos(ffn.EPI_BGRADB, 0, False, True, 768, 2304, 8192),
        "bgradb_f32_768x3072": h.gemm_epilogue_algos(ffn.EPI_BGRADB, 0, False, True, 768, 3072, 8192),
        "bgradb_bf16_768x3072": h.gemm_epilogue_algos(ffn.EPI_BGRADB, 1, False, True, 768, 3072, 8192),
    }}), flush=True)
    torch.manual_seed(0)
    M = 8192
    # fc1 backward: dY2 [M, 768], W2 [768, 3072], h [M, 3072]
    dy = torch.randn(M, 768, device=dev)
    w2 = torch.randn(768, 3072, device=dev) / 768 ** 0.5
    hh = torch.randn(M, 3072, device=dev)
    gb = torch.zeros(3072, device=dev)
    row = {"op": "dgelu", "M": M, "N": 768, "K": 3072}
    try:
        dh, db = ffn.gemm_dgelu_bgrad(dy, w2, hh)
        ref = (dy.double() @ w2.double()) * ffn.gelu_tanh_grad_ref(hh.double())
        row["relerr_dh"] = rel(dh, ref)
        row["relerr_db"] = rel(db, ref.sum(0))
        row["old_us"] = timeit(lambda: D.colsum_accumulate_(ffn.gemm_dgelu(dy, w2, hh), gb))
        row["new_us"] = timeit(lambda: gb.add_(ffn.gemm_dgelu_bgrad(dy, w2, hh)[1]))
        row["dgelu_only_us"] = timeit(lambda: ffn.gemm_dgelu(dy, w2, hh))
    except (RuntimeError, ValueError) as e:
        row["error"] = str(e)[:300]
    print(json.dumps(row), flush=True)
    for Mr, Nn, K, name in ((M, 2304, 768, "qkv"), (M, 3072, 768, "fc1"), (M, 768, 768, "attn_out/mlm_dense"),
                            (M, 768, 3072, "fc2"), (1280, 30528, 768, "mlm_decoder")):
        dy = torch.randn(Mr, Nn, device=dev)
        x = torch.randn(Mr, K, device=dev)
        gw = torch.zeros(Nn, K, device=dev)
        gb = torch.zeros(Nn, device=dev)
        row = {"op": "wgrad", "name": name, "M": Mr, "N": Nn, "K": K}
        try:
            base = torch.randn(Nn, K, device=dev)
            gw.copy_(base)
            db = ffn.gemm_wgrad_bgrad(dy, x, gw, True)
            ref = base.double() + dy.double().t() @ x.double()
            row["relerr_dw"] = rel(gw, ref)
            row["relerr_db"] = rel(db, dy.double().sum(0))
            row["old_us"] = timeit(lambda: (gw.addmm_(dy.t(), x), D.colsum_accumulate_(dy, gb)))
            row["addmm_only_us"] = timeit(lambda: gw.addmm_(dy.t(), x))
            row["new_us"] = timeit(lambda: gb.add_(ffn.gemm_wgrad_bgrad(dy, x, gw, True)))
        except (RuntimeError, ValueError) as e:
            row["error"] = str(e)[:300]
        print(json.dumps(row), flush=True)


if __name__ == "__main__":
    main()
