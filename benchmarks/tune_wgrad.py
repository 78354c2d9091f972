"""Per-shape autotune of the weight-gradient kernel (csrc/hip/wgrad.hip) for the trace's models.

Enumerates every Linear / 1x1-convolution weight gradient of ResNet-50 (bs 256, 224x224) and
BERT-base (bs 64, seq 128) -- shapes taken from the real modules with forward hooks on a tiny
CPU batch, token counts scaled to the training batch -- and times candidate (variant, splits)
pairs around the current heuristic (``ops/wgrad.choose``) with CUDA events: the split-K reduce
and fp32 output of the training path included.  Writes the per-shape winners as JSON.

Round 3 result (profiles/r3/wgrad_tune.jsonl): isolated calls 2219 -> 2082 us summed over the 22
shapes, but a same-box step A/B with the table wired into ``ops/wgrad.choose`` showed no gain
(ResNet-50 23.46 vs 23.43 ms, BERT-base 10.24-10.31 either way,
profiles/r3/raw/ab_wgrad_tuned_steps.txt): the microbenchmark's operands stay hot in L2 / MALL
between calls, the step's do not.  The heuristic stays.

python benchmarks/tune_wgrad.py [--out gpurun_out/tune/wgrad_tuned.json] [--iters 20]
"""
from __future__ import annotations

import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from vodascheduler_amd.ops import wgrad as W  # noqa: E402

VARIANTS = (1, 2, 3, 4, 9, 10)


def model_shapes() -> list[tuple[str, int, int, int]]:
    """(tag, M, N, K) of every Linear / 1x1-conv weight gradient, deduplicated."""
    from vodascheduler_amd.models import get_workload

    shapes: dict[tuple[int, int, int], str] = {}
    # ResNet-50: 1x1 convolutions (stride folded into the output size), bs 256
    w = get_workload("resnet50")
    m = w.build()
    hooks = []

    def conv_hook(mod, inp, out):
        if mod.kernel_size == (1, 1):
            M = 256 * out.shape[2] * out.shape[3]
            shapes.setdefault((M, mod.out_channels, mod.in_channels), f"resnet50.{mod.out_channels}x{mod.in_channels}")

    for mod in m.modules():
        if isinstance(mod, torch.nn.Conv2d):
            hooks.append(mod.register_forward_hook(conv_hook))
    with torch.no_grad():
        m(torch.randn(1, 3, 224, 224))
    for h in hooks:
        h.remove()
    # BERT-base: every Linear at 64 x 128 tokens (the masked-LM head sees the masked positions)
    w = get_workload("bert-base")
    mb = w.build()
    tok = set()

    def lin_hook(mod, inp, out):
        tok.add((mod.out_features, mod.in_features, inp[0].numel() // inp[0].shape[-1]))

    hooks = [mod.register_forward_hook(lin_hook) for mod in mb.modules() if isinstance(mod, torch.nn.Linear)]
    ids = torch.randint(1, 1000, (2, 128))
    with torch.no_grad():
        try:
            mb(ids, torch.ones_like(ids, dtype=torch.bool))
        except TypeError:
            mb(ids)
    for h in hooks:
        h.remove()
    for n, k, rows in sorted(tok):
        M = rows * 32  # 2 sequences -> 64
        shapes.setdefault((M, n, k), f"bert.{n}x{k}")
    # the masked-LM head in training sees the masked positions only (20 % of 8192 tokens)
    shapes.setdefault((1280, 768, 768), "bert.mlm_dense")
    shapes.setdefault((1280, 30528, 768), "bert.mlm_decoder")
    return [(tag, M, N, K) for (M, N, K), tag in sorted(shapes.items())]


def timeit(fn, iters: int) -> float:
    for _ in range(3):
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
    ap = argparse.ArgumentParser()
    ap.add_argument("--out", default="gpurun_out/tune/wgrad_tuned.json")
    ap.add_argument("--iters", type=int, default=20)
    a = ap.parse_args()
    shapes = model_shapes()
    print(json.dumps({"shapes": len(shapes)}), flush=True)
    dev = torch.device("cuda", 0)
    table = {}
    for tag, M, N_, K in shapes:
        if N_ % 8 or K % 8:
            continue
        dy = torch.randn(M, N_, device=dev).bfloat16()
        x = torch.randn(M, K, device=dev).bfloat16()
        gw = torch.zeros(N_, K, device=dev)
        gb = torch.zeros(N_, device=dev) if tag.startswith("bert") else None
        hv, hs = W.choose(M, N_, K)
        res = {}
        for v in VARIANTS:
            if v >= 9 and math_tiles(N_, K, 256) < 4:
                continue
            s0 = W.default_splits(M, N_, K, variant=v)
            for s in sorted({max(1, s0 // 2), s0, min(256, 2 * s0), max(1, (3 * s0) // 4), min(256, (3 * s0) // 2)}):
                res[(v, s)] = timeit(lambda: W.wgrad_accumulate_(dy, x, gw, gb, splits=s, variant=v), a.iters)
        if (hv, hs) not in res:
            res[(hv, hs)] = timeit(lambda: W.wgrad_accumulate_(dy, x, gw, gb, splits=hs, variant=hv), a.iters)
        (bv, bs), bt = min(res.items(), key=lambda kv: kv[1])
        ht = res[(hv, hs)]
        table[f"{M}x{N_}x{K}"] = {"variant": bv, "splits": bs, "us": round(bt, 2), "heuristic": [hv, hs],
                                  "heuristic_us": round(ht, 2), "tag": tag}
        print(json.dumps({"tag": tag, "M": M, "N": N_, "K": K, "best": [bv, bs], "best_us": round(bt, 2),
                          "heuristic": [hv, hs], "heuristic_us": round(ht, 2)}), flush=True)
        del dy, x, gw, gb
        torch.cuda.empty_cache()
    os.makedirs(os.path.dirname(os.path.abspath(a.out)), exist_ok=True)
    with open(a.out, "w") as f:
        json.dump(table, f, indent=1, sort_keys=True)
    print(json.dumps({"written": a.out, "entries": len(table),
                      "heuristic_total_us": round(sum(e["heuristic_us"] for e in table.values()), 1),
                      "tuned_total_us": round(sum(e["us"] for e in table.values()), 1)}), flush=True)


def math_tiles(N_: int, K: int, tile: int) -> int:
    return -(-N_ // tile) * -(-K // tile)


if __name__ == "__main__":
    main()
