"""Go / no-go probe of the split-bf16 fp32 GEMM (csrc/hip/splitgemm.hip) on the BERT-base
projection shapes (M = 8192 tokens): forward (X . W^T), input gradient (dY . W) and weight
gradient (dY^T . X), against hipBLASLt fp32 (torch.mm, TF32 off).

For every shape: median us over interleaved rounds, and the error against an fp64 reference
for N(0, 1) operands and for operands whose magnitudes span 2^+-30
(``max |C - C64| / (|A| |B|)`` and the relative Frobenius error).  One JSON line per
(shape, op, candidate) on stdout / --out.

    python benchmarks/bench_splitgemm.py [--reps 20] [--out gpurun_out/sgemm.jsonl] [--quick]
"""
from __future__ import annotations

import argparse
import json
import os
import statistics
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(__file__), ".."))
from vodascheduler_amd.ops import splitgemm as SG  # noqa: E402

torch.backends.cuda.matmul.allow_tf32 = False
torch.backends.cudnn.allow_tf32 = False

M = 8192
LINEARS = {"qkv": (768, 2304), "o": (768, 768), "fc1": (768, 3072), "fc2": (3072, 768)}


def operands(op: str, k_in: int, n_out: int, dev, wide: bool, seed: int):
    g = torch.Generator(device="cpu").manual_seed(seed)

    def rnd(*s):
        t = torch.randn(*s, generator=g)
        if wide:
            t = t * torch.exp2(torch.randint(-30, 31, s, generator=g).float())
        return t.to(dev)

    if op == "fwd":    # Y[M, n] = X[M, k] . W[n, k]^T
        x, w = rnd(M, k_in), rnd(n_out, k_in)
        return x, w.t()
    if op == "dgrad":  # dX[M, k] = dY[M, n] . W[n, k]
        dy, w = rnd(M, n_out), rnd(n_out, k_in)
        return dy, w
    dy, x = rnd(M, n_out), rnd(M, k_in)  # wgrad: dW[n, k] = dY^T . X
    return dy.t(), x


def err(c: torch.Tensor, a: torch.Tensor, b: torch.Tensor) -> tuple[float, float]:
    a64, b64 = a.double(), b.double()
    ref = a64 @ b64
    bound = a64.abs() @ b64.abs()
    d = (c.double() - ref).abs()
    comp = (d / bound.clamp_min(1e-300)).max().item()
    fro = (torch.linalg.norm(c.double() - ref) / torch.linalg.norm(ref)).item()
    return comp, fro


def timeit(fn, reps: int) -> float:
    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(reps)]
    for s, e in ev:
        s.record()
        fn()
        e.record()
    torch.cuda.synchronize()
    return statistics.median(s.elapsed_time(e) * 1000.0 for s, e in ev)


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=20)
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--out", default="")
    ap.add_argument("--quick", action="store_true", help="one linear, no tile sweep")
    ap.add_argument("--variants", default="", help="comma list of math variants to time on tile 0 (A/B)")
    ap.add_argument("--no-sweep", action="store_true", help="no tile / split sweep")
    ap.add_argument("--variant-splits", action="store_true", help="sweep split-K for the --variants too")
    ap.add_argument("--no-err", action="store_true", help="timing only")
    ap.add_argument("--split-list", default="1,2,3,4,8,16", help="split-K counts of --variant-splits")
    ap.add_argument("--stagger-ab", action="store_true", help="also time the default without the WG stagger")
    args = ap.parse_args()
    dev = torch.device("cuda", 0)
    sink = open(args.out, "a") if args.out else None

    def emit(rec):
        line = json.dumps(rec)
        print(line, flush=True)
        if sink:
            sink.write(line + "\n")
            sink.flush()

    lins = {"qkv": LINEARS["qkv"]} if args.quick else LINEARS
    for name, (k_in, n_out) in lins.items():
        for op in ("fwd", "dgrad", "wgrad"):
            a, b = operands(op, k_in, n_out, dev, False, 1)
            Mo, Ko = a.shape
            No = b.shape[1]
            flops = 2.0 * Mo * No * Ko
            t0, s0, v0 = SG.plan(a, b)
            cands = {"hipblaslt": None, f"plan_t{t0}_s{s0}_v{v0}": (t0, s0, v0)}
            for v in [int(x) for x in args.variants.split(",") if x]:
                cands[f"var{v}_t0_s{s0}"] = (0, s0, v)
                if args.variant_splits:
                    tiles = -(-Mo // 128) * -(-No // 128)
                    for s in [int(x) for x in args.split_list.split(",")]:
                        if tiles * s <= 4096 and s * 64 <= Ko:
                            cands.setdefault(f"var{v}_t0_s{s}", (0, s, v))
            if args.stagger_ab:
                cands[f"nostag_t{t0}_s{s0}_v{v0}"] = (t0, s0, v0, 0)
            if not args.quick and not args.no_sweep:
                tiles = -(-Mo // 128) * -(-No // 96)
                for tile in (0, 1, 2, 3, 4, 7):
                    for s in (1, 2, 4, 8, 16):
                        if s > 1 and tiles * s > 2048:
                            continue
                        cands.setdefault(f"split_t{tile}_s{s}", (tile, s, 0))
            out = torch.empty(Mo, No, device=dev)
            fns = {}
            for key, cfg in cands.items():
                if cfg is None:
                    fns[key] = lambda: torch.mm(a, b, out=out)
                else:
                    tile, s, var = cfg[:3]
                    stag = cfg[3] if len(cfg) > 3 else 1

                    def fn(tile=tile, s=s, var=var, stag=stag):
                        h = SG.N.hip()
                        h.sgemm_f32_set_stagger(stag)
                        SG.matmul(a, b, out=out, tile=tile, splits=s, variant=var)
                        h.sgemm_f32_set_stagger(1)
                    fns[key] = fn
            for f in fns.values():  # warm-up / first-call costs
                f()
            torch.cuda.synchronize()
            times = {k: [] for k in fns}
            for _ in range(args.rounds):
                for k, f in fns.items():
                    times[k].append(timeit(f, args.reps))
            base = statistics.median(times["hipblaslt"])
            for k, ts in times.items():
                us = statistics.median(ts)
                emit({"linear": name, "op": op, "M": Mo, "N": No, "K": Ko, "cand": k, "us": round(us, 2),
                      "tflops": round(flops / us / 1e6, 1), "speedup_vs_hipblaslt": round(base / us, 3)})
            # accuracy: hipBLASLt vs the split variants, N(0,1) and 2^+-30 magnitudes
            for wide in (() if args.no_err else (False, True)):
                a2, b2 = operands(op, k_in, n_out, dev, wide, 2)
                res = {"hipblaslt": err(torch.mm(a2, b2), a2, b2)}
                for var, vn in SG.VARIANT_NAMES.items():
                    res[vn] = err(SG.matmul(a2, b2, tile=0, splits=1, variant=var), a2, b2)
                if not wide:
                    t1, sp1 = SG.choose(Mo, No, Ko)
                    res[f"{SG.GEMM_MATH}_t{t1}_s{sp1}"] = err(SG.matmul(a2, b2), a2, b2)
                for k, (comp, fro) in res.items():
                    emit({"linear": name, "op": op, "inputs": "wide2^30" if wide else "normal", "cand": k,
                          "err_comp": comp, "err_fro": fro,
                          "ratio_vs_hipblaslt": comp / max(res["hipblaslt"][0], 1e-300)})
                del a2, b2
            del a, b, out
            torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
