"""Single-GPU probe: ResNet-50 training-step time under several precision/layout/optimizer
choices, plus fused-optimizer HBM bandwidth.  Used to pick the flagship step recipe.

python benchmarks/probe_resnet.py --batch 256 --steps 20
"""
import argparse
import json
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from vodascheduler_amd.models.resnet import resnet50  # noqa: E402
from vodascheduler_amd.ops import FusedSGD  # noqa: E402
from vodascheduler_amd.ops import _native  # noqa: E402


def time_steps(step, steps, warmup):
    for _ in range(warmup):
        step()
    torch.cuda.synchronize()
    t = time.perf_counter()
    for _ in range(steps):
        step()
    torch.cuda.synchronize()
    return (time.perf_counter() - t) / steps


def variant(name, batch, steps, warmup, mode, fused, cl=True):
    torch.manual_seed(0)
    m = resnet50().cuda()
    if cl:
        m = m.to(memory_format=torch.channels_last)
    if mode == "bf16":
        m = m.to(torch.bfloat16)
    opt = FusedSGD(m.parameters(), lr=0.1, momentum=0.9) if fused else torch.optim.SGD(m.parameters(), lr=0.1,
                                                                                         momentum=0.9)
    dt = torch.bfloat16 if mode == "bf16" else torch.float32
    x = torch.randn(batch, 3, 224, 224, device="cuda", dtype=dt)
    if cl:
        x = x.to(memory_format=torch.channels_last)
    y = torch.randint(0, 1000, (batch,), device="cuda")
    lossf = torch.nn.CrossEntropyLoss()

    def step():
        opt.zero_grad(set_to_none=not fused)
        if mode == "amp":
            with torch.autocast("cuda", dtype=torch.bfloat16):
                loss = lossf(m(x), y)
        else:
            loss = lossf(m(x).float(), y)
        loss.backward()
        opt.step()

    s = time_steps(step, steps, warmup)
    r = dict(name=name, batch=batch, ms=s * 1e3, img_s=batch / s)
    print(json.dumps(r), flush=True)
    return r


def optim_bw(n=64 << 20):
    p = [torch.nn.Parameter(torch.randn(n, device="cuda"))]
    opt = FusedSGD(p, lr=0.1, momentum=0.9)
    opt.flat_groups[0].grad.normal_()
    s = time_steps(opt.step, 50, 5)
    gb = n * 4 * 5 / 1e9  # read p,g,buf + write p,buf
    r = dict(name="fused_sgd_bw", n=n, us=s * 1e6, GBps=gb / s)
    print(json.dumps(r), flush=True)
    return r


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=256)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--out", default="gpurun_out/probe_resnet.json")
    a = ap.parse_args()
    _native.hip()
    res = [optim_bw()]
    for name, mode, fused, cl in [("amp_cl_fused", "amp", True, True), ("amp_cl_torchsgd", "amp", False, True),
                                  ("bf16_cl_fused", "bf16", True, True), ("amp_nchw_fused", "amp", True, False)]:
        try:
            res.append(variant(name, a.batch, a.steps, a.warmup, mode, fused, cl))
        except Exception as e:  # keep probing other variants
            print(json.dumps(dict(name=name, error=repr(e))), flush=True)
    os.makedirs(os.path.dirname(a.out), exist_ok=True)
    with open(a.out, "w") as f:
        json.dump(res, f, indent=1)


if __name__ == "__main__":
    main()
