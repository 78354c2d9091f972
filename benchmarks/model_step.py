"""Single-GPU training-step timer for one workload of the model zoo, with the exact recipe
the elastic trainer uses (bf16 autocast, channels_last for convnets, fused HIP optimizer).
Meant to run standalone or under ``rocprofv3 --kernel-trace --stats`` to get the per-kernel
breakdown of one model's step.

python benchmarks/model_step.py --model bert-base --batch 64 --steps 20 --warmup 5
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from vodascheduler_amd.models import get_workload, prepare_model  # noqa: E402
from vodascheduler_amd.ops import _native  # noqa: E402
from vodascheduler_amd.ops.optim import make_optimizer  # noqa: E402
from vodascheduler_amd.runtime.stepgraph import GraphedStepper  # noqa: E402


def run(model: str, batch: int | None, steps: int, warmup: int, marker: bool = False, graph: bool = False,
        grad_dtype: str = "fp32", overlap_opt: bool = False, torch_profile: str | None = None,
        record_losses: int = 0, amp: bool = True) -> dict:
    dev = torch.device("cuda", 0)
    w = get_workload(model)
    bs = batch or w.per_gpu_batch
    torch.manual_seed(0)
    m = prepare_model(w, dev, amp)
    opt = make_optimizer(w.optimizer, m.parameters(), grad_dtype={"fp32": torch.float32, "bf16": torch.bfloat16}[grad_dtype],
                         **w.opt_kwargs)
    b = w.make_batch(bs, dev, None)
    if w.channels_last:
        b = tuple(t.to(memory_format=torch.channels_last) if t.dim() == 4 else t for t in b)

    ddp = None
    if overlap_opt:  # the trainer's path: per-bucket optimizer updates overlapping backward
        from vodascheduler_amd.parallel.ddp import ElasticDDP

        ddp = ElasticDDP(m, None, opt, overlap_optimizer=True)

    def step_fn(bb):
        (ddp or opt).zero_grad()
        with torch.autocast("cuda", dtype=torch.bfloat16, enabled=amp, cache_enabled=not graph):
            loss = w.loss(m, bb)
        loss.backward()
        (ddp or opt).step()
        return loss

    stepper = GraphedStepper(step_fn, m, opt, warmup=2, enabled=graph)

    def step():
        return stepper(b)

    losses = []
    for _ in range(record_losses):  # trajectory check (untimed): the first losses from init
        losses.append(round(float(step().detach()), 5))
    t_w = time.perf_counter()
    for i in range(warmup):
        t_i = time.perf_counter()
        step()
        torch.cuda.synchronize(dev)
        # one line per warm-up step: the first ones run MIOpen's find / library autotuning,
        # which can take minutes (fp32), and a silent run looks hung
        print(f"warm-up step {i}: {time.perf_counter() - t_i:.2f} s", file=sys.stderr, flush=True)
    warm_s = time.perf_counter() - t_w
    if marker:  # trace_window_stats.py keeps only kernels after this one
        torch.cuda._sleep(1000)
        torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    for _ in range(steps):
        loss = step()
    torch.cuda.synchronize(dev)
    dt = (time.perf_counter() - t0) / steps
    if torch_profile:  # which aten op launched each library / PyTorch kernel, by input shape
        from torch.profiler import ProfilerActivity, profile

        with profile(activities=[ProfilerActivity.CPU, ProfilerActivity.CUDA], record_shapes=True) as prof:
            for _ in range(3):
                step()
            torch.cuda.synchronize(dev)
        with open(torch_profile, "w") as f:
            f.write(prof.key_averages(group_by_input_shape=True).table(sort_by="self_device_time_total",
                                                                      row_limit=250, max_name_column_width=60,
                                                                      max_shapes_column_width=90))
            f.write("\n\n")
            f.write(prof.key_averages().table(sort_by="device_time_total", row_limit=80,
                                              max_name_column_width=60))
    return {"model": model, "batch": bs, "ms_per_step": round(dt * 1e3, 3),
            "samples_per_s": round(bs / dt, 1), "loss": float(loss.detach()), "graph": stepper.graph is not None,
            "warmup_s": round(warm_s, 3), **({"losses": losses} if losses else {})}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--model", default="resnet50")
    ap.add_argument("--batch", type=int, default=None)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--cudnn-benchmark", action="store_true", help="MIOpen exhaustive find (benchmark mode)")
    ap.add_argument("--profile-marker", action="store_true", help="launch a marker kernel before the timed steps")
    ap.add_argument("--graph", action="store_true", help="replay the whole step as one captured hipGraph")
    ap.add_argument("--grad-dtype", default="fp32", choices=["fp32", "bf16"], help="flat gradient precision")
    ap.add_argument("--overlap-opt", action="store_true", help="per-bucket optimizer overlapping backward (ElasticDDP)")
    ap.add_argument("--torch-profile", default=None, help="write a torch.profiler op table (3 steps) to this path")
    ap.add_argument("--losses", type=int, default=0, help="record the first N step losses (trajectory checks)")
    ap.add_argument("--precision", default="bf16-amp", choices=["bf16-amp", "fp32"])
    ap.add_argument("--set", action="append", default=[], metavar="MODULE:ATTR=VALUE",
                    help="set a module-level kernel-path switch before building the model (same-process A/B "
                         "of the module constants listed in docs/kernels.md), e.g. "
                         "vodascheduler_amd.models.layers:BIAS_HANDOFF=False")
    a = ap.parse_args()
    for spec in a.set:
        import ast
        import importlib

        mod, rest = spec.split(":", 1)
        attr, val = rest.split("=", 1)
        setattr(importlib.import_module(mod), attr, ast.literal_eval(val))
    if a.cudnn_benchmark:
        torch.backends.cudnn.benchmark = True
    _native.hip()
    out = run(a.model, a.batch, a.steps, a.warmup, a.profile_marker, a.graph, a.grad_dtype, a.overlap_opt,
              a.torch_profile, a.losses, a.precision != "fp32")
    out["precision"] = a.precision
    out["grad_dtype"] = a.grad_dtype
    out["overlap_opt"] = a.overlap_opt
    if a.set:
        out["set"] = a.set
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
