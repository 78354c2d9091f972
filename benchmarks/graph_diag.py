"""Which part of a training step goes wrong under whole-step hipGraph capture?

Builds a workload twice with identical weights, runs the step eagerly on one copy and as a
captured + replayed hipGraph on the other (lr = 0, so the weights stay fixed and every step
computes the same gradients), then compares every parameter's flat gradient, the loss and
the BatchNorm running statistics.  Parameters whose graph gradient deviates from the eager
one name the op whose work the capture lost (docs/kernels.md).

python benchmarks/graph_diag.py --model resnet50 --batch 32
"""
from __future__ import annotations

import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from vodascheduler_amd.models import get_workload, prepare_model  # noqa: E402
from vodascheduler_amd.ops import _native  # noqa: E402
from vodascheduler_amd.ops.optim import make_optimizer  # noqa: E402
from vodascheduler_amd.runtime.stepgraph import StepGraph  # noqa: E402
from vodascheduler_amd.utils.flat import grad_of  # noqa: E402


def build(w, dev, seed=0, frozen=True):
    """frozen: lr = 0 (and no momentum / decay) so every step sees the same weights."""
    torch.manual_seed(seed)
    m = prepare_model(w, dev)
    kw = dict(w.opt_kwargs)
    if frozen:
        kw["lr"] = 0.0
        for k in ("momentum", "weight_decay"):
            if k in kw:
                kw[k] = 0.0
    opt = make_optimizer(w.optimizer, m.parameters(), **kw)
    return m, opt


def update_check(w, dev, batch, warmup: int, steps: int) -> dict:
    """Real optimizer updates: ``steps`` eager steps vs ``steps`` graph replays after the same
    eager warm-up; parameter / optimizer-state relative differences and loss trajectories."""
    def make_step(m, opt):
        def step_fn(b):
            opt.zero_grad()
            with torch.autocast("cuda", dtype=torch.bfloat16, cache_enabled=False):
                loss = w.loss(m, b)
            loss.backward()
            opt.step()
            return loss
        return step_fn

    me, oe = build(w, dev, frozen=False)
    mg, og = build(w, dev, frozen=False)
    se, sg = make_step(me, oe), make_step(mg, og)
    side = torch.cuda.Stream()
    for _ in range(warmup):
        se(batch)
        side.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(side):
            sg(batch)
        torch.cuda.current_stream().wait_stream(side)
    torch.cuda.synchronize()
    graph = StepGraph(sg, batch, mg, og)
    le, lg = [], []
    for _ in range(steps):
        le.append(float(se(batch)))
        lg.append(float(graph.replay(batch)))
    torch.cuda.synchronize()
    worst = []
    for i, (a, b) in enumerate(zip(oe.flat_state_tensors(), og.flat_state_tensors())):
        if a.dtype.is_floating_point:
            rel = float((b.float() - a.float()).norm() / a.float().norm().clamp_min(1e-20))
            worst.append((rel, i))
    worst.sort(reverse=True)
    return {"losses_eager": le, "losses_graph": lg, "state_rel_err_max": worst[0][0] if worst else 0.0,
            "steps_host": [oe._steps, og._steps], "step_t": [oe._step_t.tolist(), og._step_t.tolist()]}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--model", default="resnet50")
    ap.add_argument("--batch", type=int, default=32)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--tol", type=float, default=2e-2)
    ap.add_argument("--update-steps", type=int, default=5, help="real-update check length (0: skip)")
    a = ap.parse_args()
    _native.hip()
    dev = torch.device("cuda", 0)
    w = get_workload(a.model)
    g = torch.Generator(device=dev).manual_seed(1)
    batch = w.make_batch(a.batch, dev, g)
    if w.channels_last:
        batch = tuple(t.to(memory_format=torch.channels_last) if t.dim() == 4 else t for t in batch)

    def make_step(m, opt):
        def step_fn(b):
            opt.zero_grad()
            with torch.autocast("cuda", dtype=torch.bfloat16, cache_enabled=False):
                loss = w.loss(m, b)
            loss.backward()
            opt.step()
            return loss
        return step_fn

    me, oe = build(w, dev)
    mg, og = build(w, dev)
    se, sg = make_step(me, oe), make_step(mg, og)
    side = torch.cuda.Stream()
    for _ in range(a.warmup):  # identical eager warm-up of both copies (algorithm selection)
        se(batch)
        side.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(side):
            sg(batch)
        torch.cuda.current_stream().wait_stream(side)
    torch.cuda.synchronize()
    le = float(se(batch))
    torch.cuda.synchronize()
    eager = {n: grad_of(p).float().clone() for n, p in me.named_parameters()}
    graph = StepGraph(sg, batch, mg, og)
    out = {"model": a.model, "batch": a.batch}
    reps = []
    for r in range(2):
        lg = float(graph.replay(batch))
        torch.cuda.synchronize()
        bad = []
        for n, p in mg.named_parameters():
            ge, gg = eager[n], grad_of(p).float()
            rel = float((gg - ge).norm() / ge.norm().clamp_min(1e-20))
            if not rel < a.tol:
                bad.append({"param": n, "rel_err": rel, "eager_norm": float(ge.norm()), "graph_norm": float(gg.norm())})
        reps.append({"replay": r, "loss_eager": le, "loss_graph": lg, "n_params": len(eager), "n_bad": len(bad),
                     "bad": bad[:40]})
    out["replays"] = reps
    bn_bad = []
    for (n, be), (_, bg) in zip(me.named_buffers(), mg.named_buffers()):
        if be.dtype.is_floating_point:
            rel = float((bg.float() - be.float()).norm() / be.float().norm().clamp_min(1e-20))
            if not rel < 0.05:
                bn_bad.append({"buffer": n, "rel_err": rel})
    out["buffers_off"] = bn_bad[:20]
    if a.update_steps > 0:
        out["update_check"] = update_check(w, dev, batch, a.warmup, a.update_steps)
    print(json.dumps(out, indent=1), flush=True)


if __name__ == "__main__":
    main()
