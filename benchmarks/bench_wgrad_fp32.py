"""fp32-output weight gradients: the split-K MFMA kernel (csrc/hip/wgrad.hip, fp32 dW written
in place with beta = 1) vs hipBLASLt through ``aten::addmm.dtype`` (bf16 operands, fp32
accumulate and output, beta = 1) on the BERT-base Linear shapes and the ResNet-50 bs-256
1x1-convolution shapes.  Reports time, TFLOP/s and the error of each against fp32.

python benchmarks/bench_wgrad_fp32.py
"""
from __future__ import annotations

import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from vodascheduler_amd.ops import _native  # noqa: E402
from vodascheduler_amd.ops import wgrad as W  # noqa: E402

# (name, rows M, N = out features / Cout, K = in features / Cin)
SHAPES = [("bert.qkv", 8192, 2304, 768), ("bert.attn_out", 8192, 768, 768), ("bert.fc1", 8192, 3072, 768),
          ("bert.fc2", 8192, 768, 3072),
          ("r50.l1.conv1", 802816, 64, 256), ("r50.l1.conv3", 802816, 256, 64),
          ("r50.l2.conv1", 200704, 128, 512), ("r50.l2.conv3", 200704, 512, 128),
          ("r50.l3.conv1", 50176, 256, 1024), ("r50.l3.conv3", 50176, 1024, 256),
          ("r50.l4.conv1", 12544, 512, 2048), ("r50.l4.conv3", 12544, 2048, 512)]


def timeit(fn, iters=30, warm=5) -> float:
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


def blaslt_form(gw, a, b):
    """The cheapest working in-place hipBLASLt form on this PyTorch: fp32 out, beta = 1."""
    try:
        torch.addmm(gw, a, b, out_dtype=torch.float32, out=gw)
        return "addmm.dtype_out", lambda: torch.addmm(gw, a, b, out_dtype=torch.float32, out=gw)
    except Exception:
        pass
    try:
        torch.addmm(gw, a, b, out_dtype=torch.float32)
        return "addmm.dtype+copy", lambda: gw.copy_(torch.addmm(gw, a, b, out_dtype=torch.float32))
    except Exception:
        pass
    return "mm.dtype+add", lambda: gw.add_(torch.mm(a, b, out_dtype=torch.float32))


def main():
    import argparse

    ap = argparse.ArgumentParser()
    ap.add_argument("--only", default="", help="substring filter on shape names")
    ap.add_argument("--no-blaslt", action="store_true")
    ap.add_argument("--sweep", action="store_true", help="time every variant x split count (no hipBLASLt)")
    ap.add_argument("--variants", default="0,1,2,3,4,5,6,7,8", help="sweep: variants to time")
    ap.add_argument("--split-mults", default="0.25,0.5,1,2", help="sweep: multiples of the default split count")
    a = ap.parse_args()
    _native.hip()
    dev = torch.device("cuda", 0)
    for name, M, N, K in SHAPES:
        if a.only and a.only not in name:
            continue
        torch.manual_seed(0)
        dy = torch.randn(M, N, device=dev).bfloat16()
        x = torch.randn(M, K, device=dev).bfloat16()
        ref = dy.float().t() @ x.float() if M * (N + K) <= 2 ** 31 else None
        gw = torch.zeros(N, K, device=dev, dtype=torch.float32)
        tf = 2.0 * M * N * K / 1e12
        r = {"shape": name, "M": M, "N": N, "K": K}
        W.wgrad_accumulate_(dy, x, gw, accumulate=False)
        torch.cuda.synchronize()
        if ref is not None:
            r["ours_rel_err"] = float((gw - ref).norm() / ref.norm())
        t = timeit(lambda: W.wgrad_accumulate_(dy, x, gw))
        r["ours_us"], r["ours_tflops"] = round(t, 2), round(tf / (t * 1e-6), 1)
        if a.sweep:
            best = None
            for v in [int(t) for t in a.variants.split(",")]:
                base = W.default_splits(M, N, K, variant=v)
                for sp in sorted({max(1, min(256, round(base * float(f)))) for f in a.split_mults.split(",")}):
                    try:
                        t = timeit(lambda: W.wgrad_accumulate_(dy, x, gw, splits=sp, variant=v), iters=10, warm=2)
                    except Exception as e:  # a variant may reject a shape
                        r[f"v{v}_s{sp}"] = f"error: {e}"[:60]
                        continue
                    r[f"v{v}_s{sp}"] = round(t, 1)
                    if best is None or t < best[0]:
                        best = (t, v, sp)
            r["best_us"], r["best_variant"], r["best_splits"] = round(best[0], 2), best[1], best[2]
            r["best_TBs"] = round(2 * M * (N + K) / (best[0] * 1e-6) / 1e12, 2)
            print(json.dumps(r), flush=True)
            continue
        if a.no_blaslt:
            print(json.dumps(r), flush=True)
            continue
        gw.zero_()
        form, fn = blaslt_form(gw, dy.t(), x)
        torch.cuda.synchronize()
        gw.zero_()
        fn()
        torch.cuda.synchronize()
        if ref is not None:
            r["blaslt_rel_err"] = float((gw - ref).norm() / ref.norm())
        t = timeit(fn)
        r["blaslt_form"] = form
        r["blaslt_us"], r["blaslt_tflops"] = round(t, 2), round(tf / (t * 1e-6), 1)
        print(json.dumps(r), flush=True)


if __name__ == "__main__":
    main()
