"""LayerNorm backward (csrc/hip/layernorm.hip) with 4 vs 8 waves per block on BERT-base rows
(8192 x 768, fp32 and bf16), with dgamma / dbeta (and the hand-off bias sum) as in the model.
Bytes: dy, x read + dx written.  Also times the forward with the fused residual add.

python benchmarks/bench_layernorm.py
"""
from __future__ import annotations

import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from vodascheduler_amd.ops import _native as N  # noqa: E402


def timed(fn, iters=50):
    for _ in range(5):
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
    s = torch.cuda.current_stream().cuda_stream
    for dt in (torch.float32, torch.bfloat16):
        for M, n in ((8192, 768), (10240, 256), (8192, 1024)):
            x = torch.randn(M, n, device="cuda").to(dt)
            dy = torch.randn(M, n, device="cuda").to(dt)
            g = torch.randn(n, device="cuda")
            mean = torch.randn(M, device="cuda")
            rstd = torch.rand(M, device="cuda") + 0.5
            dx = torch.empty_like(x)
            dg = torch.zeros(n, device="cuda")
            db = torch.zeros(n, device="cuda")
            dbi = torch.zeros(n, device="cuda")
            rows = h.layernorm_bwd_partial_rows(M)
            ws = torch.empty(3 * rows * n, device="cuda")
            wdt = N.dtype_code(torch.float32)
            out = {}
            ref = None
            for w in (4, 8):
                h.layernorm_set_bwd_waves(w)

                def bwd():
                    h.layernorm_bwd(dy.data_ptr(), x.data_ptr(), mean.data_ptr(), rstd.data_ptr(), g.data_ptr(),
                                    dx.data_ptr(), dg.data_ptr(), db.data_ptr(), ws.data_ptr(), M, n,
                                    N.dtype_code(dt), wdt, False, s, dbi.data_ptr())
                bwd()
                torch.cuda.synchronize()
                res = [dx.clone(), dg.clone(), db.clone(), dbi.clone()]
                if ref is None:
                    ref = res
                else:
                    out["bitwise_equal_4_vs_8"] = all(bool(torch.equal(a, b)) for a, b in zip(ref[:1], res[:1]))
                    out["max_rel_param_grads"] = max(
                        float(((a - b).norm() / (b.norm() + 1e-30)).item()) for a, b in zip(ref[1:], res[1:]))
                us = timed(bwd)
                out[f"bwd_w{w}_us"] = round(us, 2)
                out[f"bwd_w{w}_TBps"] = round(3 * x.numel() * x.element_size() / us / 1e6, 2)
            h.layernorm_set_bwd_waves(8)
            print(json.dumps({"dtype": str(dt).split(".")[-1], "M": M, "N": n, **out}), flush=True)


if __name__ == "__main__":
    main()
