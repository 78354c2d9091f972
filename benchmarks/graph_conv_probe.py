"""Is one convolution's training step replay-safe under hipGraph capture?

For each convolution shape of ResNet-50, two identical copies (bf16 compute weight, fp32
flat gradient and master, fused SGD with momentum -- the trainer's exact setup) take the same
real-update steps on a fixed batch: one eagerly, one as a captured + replayed graph.  After
every step the tool reports whether the replayed weight gradient is finite and how far the
two weight copies have drifted apart.  ``path`` = ``miopen`` (nn.Conv2d -> MIOpen) or
``gemm`` (ops/conv1x1.py: hipBLASLt + the split-K MFMA wgrad kernel).

python benchmarks/graph_conv_probe.py --steps 6
"""
from __future__ import annotations

import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from vodascheduler_amd.ops import _native  # noqa: E402
from vodascheduler_amd.ops.conv1x1 import Conv1x1  # noqa: E402
from vodascheduler_amd.ops.optim import make_optimizer  # noqa: E402
from vodascheduler_amd.runtime.stepgraph import StepGraph  # noqa: E402
from vodascheduler_amd.utils.flat import grad_of  # noqa: E402

# name, path, batch, cin, cout, k, stride, H
CASES = [
    ("l1.conv3 64->256 1x1 @56", "miopen", 64, 64, 256, 1, 1, 56),
    ("l1.conv1 64->64 1x1 @56", "miopen", 64, 64, 64, 1, 1, 56),
    ("l1.down 64->256 1x1 @56", "miopen", 64, 64, 256, 1, 1, 56),
    ("cifar l1.conv3 64->256 1x1 @32", "miopen", 128, 64, 256, 1, 1, 32),
    ("l2.0.conv2 128->128 3x3 s2 @56", "miopen", 64, 128, 128, 3, 2, 56),
    ("stem 3->64 7x7 s2 @224", "miopen", 32, 3, 64, 7, 2, 224),
    ("l1.conv2 64->64 3x3 @56", "miopen", 64, 64, 64, 3, 1, 56),
    ("l2.conv1 256->128 1x1 @56 (gemm)", "gemm", 64, 256, 128, 1, 1, 56),
]


def make(path, cin, cout, k, stride, dev):
    torch.manual_seed(0)
    if path == "gemm":
        conv = Conv1x1(cin, cout, stride)
    else:
        conv = torch.nn.Conv2d(cin, cout, k, stride, padding=k // 2, bias=False)
    conv = conv.to(dev).to(memory_format=torch.channels_last).to(torch.bfloat16)
    opt = make_optimizer("sgd", conv.parameters(), lr=0.5, momentum=0.9)
    return conv, opt


def run_case(case, steps, dev):
    name, path, b, cin, cout, k, stride, H = case
    g = torch.Generator(device=dev).manual_seed(1)
    x = torch.randn(b, cin, H, H, device=dev, generator=g).to(torch.bfloat16).to(memory_format=torch.channels_last)
    ce, oe = make(path, cin, cout, k, stride, dev)
    cg, og = make(path, cin, cout, k, stride, dev)
    with torch.no_grad():
        t = torch.randn_like(ce(x).float())

    def step(conv, opt):
        def fn(batch):
            opt.zero_grad()
            y = conv(batch[0])
            loss = ((y.float() - t) ** 2).mean()
            loss.backward()
            opt.step()
            return loss
        return fn

    se, sg = step(ce, oe), step(cg, og)
    side = torch.cuda.Stream()
    for _ in range(3):
        se((x,))
        side.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(side):
            sg((x,))
        torch.cuda.current_stream().wait_stream(side)
    torch.cuda.synchronize()
    graph = StepGraph(sg, (x,), cg, og)
    rows = []
    for i in range(steps):
        le = float(se((x,)))
        lg = float(graph.replay((x,)))
        torch.cuda.synchronize()
        ge, gg = grad_of(ce.weight).float(), grad_of(cg.weight).float()
        we, wg = ce.weight.float(), cg.weight.float()
        rows.append({"step": i, "loss_eager": le, "loss_graph": lg, "grad_finite": bool(torch.isfinite(gg).all()),
                     "grad_rel": float((gg - ge).norm() / ge.norm().clamp_min(1e-20)),
                     "weight_rel": float((wg - we).norm() / we.norm().clamp_min(1e-20))})
    bad = [r["step"] for r in rows if not r["grad_finite"] or not r["grad_rel"] < 5e-2]
    return {"case": name, "path": path, "first_bad_step": bad[0] if bad else None, "rows": rows}


def poison_allocator(dev, gib: float = 4.0) -> None:
    """Fill a large block of the caching allocator with NaN bit patterns and free it, so the
    next step's fresh tensors (outputs a kernel must fully write) start out as NaN."""
    t = torch.empty(int(gib * 2 ** 30) // 2, dtype=torch.bfloat16, device=dev)
    t.fill_(float("nan"))
    del t
    torch.cuda.synchronize()


def poison_case(case, dev):
    """Eager steps, the last one right after poison_allocator(): does a library kernel read
    its (uninitialised) output?  Compared with an unpoisoned copy."""
    name, path, b, cin, cout, k, stride, H = case
    g = torch.Generator(device=dev).manual_seed(1)
    x = torch.randn(b, cin, H, H, device=dev, generator=g).to(torch.bfloat16).to(memory_format=torch.channels_last)
    out = {}
    for poisoned in (False, True):
        conv, opt = make(path, cin, cout, k, stride, dev)
        xi = x.clone().requires_grad_()
        for i in range(3):
            if poisoned and i == 2:
                poison_allocator(dev)
            opt.zero_grad()
            xi.grad = None
            y = conv(xi)
            (y.float() ** 2).mean().backward()
        torch.cuda.synchronize()
        out[poisoned] = (grad_of(conv.weight).float().clone(), xi.grad.float().clone())
    (gw0, gx0), (gw1, gx1) = out[False], out[True]
    return {"case": name, "path": path, "poison_wgrad_finite": bool(torch.isfinite(gw1).all()),
            "poison_dgrad_finite": bool(torch.isfinite(gx1).all()),
            "wgrad_rel": float((gw1 - gw0).norm() / gw0.norm().clamp_min(1e-20)),
            "dgrad_rel": float((gx1 - gx0).norm() / gx0.norm().clamp_min(1e-20))}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=6)
    ap.add_argument("--only", default="", help="substring filter on case names")
    ap.add_argument("--poison", action="store_true", help="eager poisoned-allocator check instead of graphs")
    ap.add_argument("--benchmark", action="store_true",
                    help="MIOpen exhaustive find (cudnn.benchmark), as prepare_model sets for the convnets")
    a = ap.parse_args()
    torch.backends.cudnn.benchmark = a.benchmark
    _native.hip()
    dev = torch.device("cuda", 0)
    for case in CASES:
        if a.only and a.only not in case[0]:
            continue
        r = poison_case(case, dev) if a.poison else run_case(case, a.steps, dev)
        r["benchmark"] = a.benchmark
        print(json.dumps(r), flush=True)


if __name__ == "__main__":
    main()
