"""Per-pass timing of ResNet-50's convolutions (bs 256, channels_last bf16): MIOpen (exhaustive
find) fwd / bwd-data / bwd-weight vs the same 1x1 products as hipBLASLt GEMMs, plus the HBM
roofline of each pass.  Decides which passes are worth routing away from MIOpen.

python benchmarks/bench_conv_passes.py
"""
from __future__ import annotations

import json
import os

import torch
import torch.nn.functional as F

torch.backends.cudnn.benchmark = True
B = 256
# (cin, cout, k, stride, H_in, count per step)
CONVS = [(3, 64, 7, 2, 224, 1),
         (64, 64, 1, 1, 56, 1), (64, 64, 3, 1, 56, 3), (64, 256, 1, 1, 56, 4), (256, 64, 1, 1, 56, 2),
         (256, 128, 1, 1, 56, 1), (128, 128, 3, 2, 56, 1), (256, 512, 1, 2, 56, 1), (128, 128, 3, 1, 28, 3),
         (128, 512, 1, 1, 28, 4), (512, 128, 1, 1, 28, 3),
         (512, 256, 1, 1, 28, 1), (256, 256, 3, 2, 28, 1), (512, 1024, 1, 2, 28, 1), (256, 256, 3, 1, 14, 5),
         (256, 1024, 1, 1, 14, 6), (1024, 256, 1, 1, 14, 5),
         (1024, 512, 1, 1, 14, 1), (512, 512, 3, 2, 14, 1), (1024, 2048, 1, 2, 14, 1), (512, 512, 3, 1, 7, 2),
         (512, 2048, 1, 1, 7, 3), (2048, 512, 1, 1, 7, 2)]


def t_us(fn, it=10):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(it):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / it * 1e3


def main():
    rows = []
    tot = {"fwd": 0.0, "bwd_data": 0.0, "bwd_weight": 0.0, "roof": 0.0}
    for cin, cout, k, s, H, cnt in CONVS:
        p = k // 2
        x = torch.randn(B, cin, H, H, device="cuda", dtype=torch.bfloat16).to(memory_format=torch.channels_last)
        w = (torch.randn(cout, cin, k, k, device="cuda", dtype=torch.bfloat16) * 0.05).to(
            memory_format=torch.channels_last)
        y = F.conv2d(x, w, stride=s, padding=p)
        dy = torch.randn_like(y)
        Ho = y.shape[2]
        fwd = t_us(lambda: F.conv2d(x, w, stride=s, padding=p))
        bd = t_us(lambda: torch.ops.aten.convolution_backward(dy, x, w, None, [s, s], [p, p], [1, 1], False, [0, 0],
                                                               1, [True, False, False]))
        bw = t_us(lambda: torch.ops.aten.convolution_backward(dy, x, w, None, [s, s], [p, p], [1, 1], False, [0, 0],
                                                               1, [False, True, False]))
        r = {"cin": cin, "cout": cout, "k": k, "s": s, "H": H, "count": cnt, "fwd_us": round(fwd, 1),
             "bwd_data_us": round(bd, 1), "bwd_weight_us": round(bw, 1)}
        flops = 2 * B * Ho * Ho * cout * cin * k * k
        r["fwd_TF"] = round(flops / fwd / 1e6, 1)
        bytes_fwd = (x.numel() + y.numel()) * 2
        r["roof_us_per_pass"] = round(max(bytes_fwd / 5.5e12, flops / 1.2e15) * 1e6, 1)
        if k == 1:
            M = B * Ho * Ho
            xs = x[:, :, ::s, ::s] if s > 1 else x
            x2 = xs.permute(0, 2, 3, 1).reshape(M, cin)
            w2 = w.view(cout, cin)
            dy2 = dy.permute(0, 2, 3, 1).reshape(M, cout)
            if s == 1:
                r["gemm_fwd_us"] = round(t_us(lambda: x2 @ w2.t()), 1)
            r["gemm_bwd_data_us"] = round(t_us(lambda: dy2 @ w2), 1)
            r["gemm_bwd_weight_us"] = round(t_us(lambda: dy2.t() @ x2), 1)
        rows.append(r)
        for key, v in (("fwd", fwd), ("bwd_data", bd), ("bwd_weight", bw)):
            tot[key] += v * cnt
        tot["roof"] += 3 * r["roof_us_per_pass"] * cnt
        print(json.dumps(r), flush=True)
    print(json.dumps({k: round(v / 1e3, 2) for k, v in tot.items()}), flush=True)
    os.makedirs("gpurun_out", exist_ok=True)
    json.dump({"rows": rows, "total_ms": tot}, open("gpurun_out/bench_conv_passes.json", "w"), indent=1)


if __name__ == "__main__":
    main()
