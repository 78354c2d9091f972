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


def update_check(w, dev, batch, warmup: int, steps: int, graphed: bool = True) -> dict:
    """Real optimizer updates: ``steps`` eager steps vs ``steps`` graph replays after the same
    eager warm-up; parameter / optimizer-state relative differences and loss trajectories.
    ``graphed=False`` is the control: the second copy also runs eagerly, which measures how far
    two eager runs drift apart on their own (non-associative reductions, chaotic training)."""
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
    graph = StepGraph(sg, batch, mg, og) if graphed else None
    le, lg = [], []
    for _ in range(steps):
        le.append(float(se(batch)))
        lg.append(float(graph.replay(batch) if graphed else sg(batch)))
    torch.cuda.synchronize()
    worst = []
    for i, (a, b) in enumerate(zip(oe.flat_state_tensors(), og.flat_state_tensors())):
        if a.dtype.is_floating_point:
            rel = float((b.float() - a.float()).norm() / a.float().norm().clamp_min(1e-20))
            worst.append((rel, i))
    worst.sort(reverse=True)
    return {"losses_eager": le, "losses_graph": lg, "state_rel_err_max": worst[0][0] if worst else 0.0,
            "steps_host": [oe._steps, og._steps], "step_t": [oe._step_t.tolist(), og._step_t.tolist()]}


def _poison(dev, gib: float = 8.0) -> None:
    t = torch.empty(int(gib * 2 ** 30) // 2, dtype=torch.bfloat16, device=dev)
    t.fill_(float("nan"))
    del t
    torch.cuda.synchronize()


def nan_probe(w, dev, batch, warmup: int, steps: int, graphed: bool = True, poison: bool = False) -> dict:
    """Real updates, replayed (or eager); after every step, which parameters have non-finite
    gradients / weights / momentum, and the gradient norm of the worst ones: locates the first
    step and the first layer where a replay goes wrong."""
    m, opt = build(w, dev, frozen=False)

    def step_fn(b):
        opt.zero_grad()
        with torch.autocast("cuda", dtype=torch.bfloat16, cache_enabled=False):
            loss = w.loss(m, b)
        loss.backward()
        opt.step()
        return loss

    side = torch.cuda.Stream()
    for _ in range(warmup):
        side.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(side):
            step_fn(batch)
        torch.cuda.current_stream().wait_stream(side)
    torch.cuda.synchronize()
    graph = StepGraph(step_fn, batch, m, opt) if graphed else None
    names = [n for n, _ in m.named_parameters()]
    rows = []
    for i in range(steps):
        if poison:  # fresh tensors of the next step start as NaN (library output-read check)
            _poison(dev)
        loss = float(graph.replay(batch) if graphed else step_fn(batch))
        torch.cuda.synchronize()
        gn = {n: float(grad_of(p).float().norm()) for n, p in m.named_parameters()}
        bad_g = [n for n in names if not torch.isfinite(torch.tensor(gn[n]))]
        bad_w = [n for n, p in m.named_parameters() if not bool(torch.isfinite(p.detach().float()).all())]
        big = sorted(gn.items(), key=lambda kv: -kv[1] if kv[1] == kv[1] else float("-inf"))[:3]
        rows.append({"step": i, "loss": loss, "bad_grads": bad_g[:8], "n_bad_grads": len(bad_g),
                     "bad_weights": bad_w[:8], "n_bad_weights": len(bad_w),
                     "top_grad_norms": [(n, round(v, 4)) for n, v in big]})
    return {"graphed": graphed, "poison": poison, "rows": rows}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--model", default="resnet50")
    ap.add_argument("--batch", type=int, default=32)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--tol", type=float, default=2e-2)
    ap.add_argument("--update-steps", type=int, default=5, help="real-update check length (0: skip)")
    ap.add_argument("--control", action="store_true", help="also run the eager-vs-eager update control")
    ap.add_argument("--skip-frozen", action="store_true", help="only the update check(s)")
    ap.add_argument("--nan-probe", type=int, default=0, help="replay N real steps, report non-finite params per step")
    ap.add_argument("--poison", action="store_true", help="nan probe: eager only, NaN-poisoned allocator per step")
    ap.add_argument("--graph-only", action="store_true", help="nan probe: skip the eager reference run")
    ap.add_argument("--no-benchmark", action="store_true",
                    help="MIOpen immediate mode (cudnn.benchmark off) instead of exhaustive find")
    a = ap.parse_args()
    _native.hip()
    dev = torch.device("cuda", 0)
    w = get_workload(a.model)
    if a.no_benchmark:  # prepare_model turns find mode on for channels_last convnets
        import vodascheduler_amd.models as _models

        _orig = _models.prepare_model

        def _prep(*args, **kw):
            m = _orig(*args, **kw)
            torch.backends.cudnn.benchmark = False
            return m

        globals()["prepare_model"] = _prep
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

    out = {"model": a.model, "batch": a.batch}
    if a.nan_probe and a.poison:
        out["probe_eager_poisoned"] = nan_probe(w, dev, batch, a.warmup, a.nan_probe, graphed=False, poison=True)
        print(json.dumps(out, indent=1), flush=True)
        return
    if a.nan_probe:
        out["probe_graph"] = nan_probe(w, dev, batch, a.warmup, a.nan_probe)
        if not a.graph_only:
            out["probe_eager"] = nan_probe(w, dev, batch, a.warmup, a.nan_probe, graphed=False)
        print(json.dumps(out, indent=1), flush=True)
        return
    if a.skip_frozen:
        out["update_check"] = update_check(w, dev, batch, a.warmup, a.update_steps)
        if a.control:
            out["update_control"] = update_check(w, dev, batch, a.warmup, a.update_steps, graphed=False)
        print(json.dumps(out, indent=1), flush=True)
        return
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
        if a.control:
            out["update_control"] = update_check(w, dev, batch, a.warmup, a.update_steps, graphed=False)
    print(json.dumps(out, indent=1), flush=True)


if __name__ == "__main__":
    main()
