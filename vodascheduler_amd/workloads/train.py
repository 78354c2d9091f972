"""Elastic data-parallel training of a registered workload (the MI355X-native counterpart of
the reference's Horovod elastic scripts).

Per step: synthetic batch (fixed pool, real shapes) -> bf16 autocast forward/backward on
PyTorch-ROCm (MIOpen/hipBLASLt + HIP LayerNorm/softmax kernels) -> bucketed all-reduce on
RCCL over xGMI overlapped with backward -> fused HIP optimizer step on flat buffers.
Elastic semantics follow the reference examples: LR = base_lr x world size on every reset
(tensorflow2_keras_cifar_elastic.py:156,210), an epoch is a fixed number of samples split
across the current workers (``steps_per_epoch // size``, :223), state committed every
``commit_every`` steps, per-epoch CSV metrics + checkpoint on rank 0.

Standalone (one process per GPU, launched by the local node agent):
    python -m vodascheduler_amd.workloads.train --model resnet50 --epochs 2 --steps-per-epoch 50 \
        --name JOB   (env: VODA_STORE=host:port, VODA_WORKER_ID, VODA_JOIN_EPOCH)
"""
from __future__ import annotations

import argparse
import contextlib
import collections
import hashlib
import json
import logging
import math
import os
import time
from dataclasses import dataclass

import torch

from ..models import get_workload, prepare_model
from ..ops.optim import make_optimizer
from ..parallel.ddp import ElasticDDP
from ..runtime.elastic import ElasticContext, TorchState, rng_state, run, set_rng_state
from ..runtime.stepgraph import GraphedStepper
from ..utils.tracing import trace_range
from .metrics_logger import MetricsCSVLogger

log = logging.getLogger("vodascheduler_amd.train")


@dataclass
class TrainConfig:
    model: str
    epochs: int = 1
    steps_per_epoch: int = 10          # in single-GPU steps: epoch = steps_per_epoch * batch samples
    per_gpu_batch: int | None = None
    lr: float | None = None            # base LR for one worker (scaled x world)
    commit_every: int = 1
    amp: bool = True                   # bf16 autocast
    compression: str | None = None     # gradient all-reduce compression: None | bf16 | fp16
    # flat gradient buffer precision: fp32 (default; bf16 compute weights keep fp32 gradients,
    # as Horovod reduces fp32 unless --fp16-allreduce) | bf16 (opt-in low-precision gradients)
    grad_dtype: str = "fp32"
    bucket_cap_mb: float = 64.0
    # per-bucket optimizer updates on the comm stream, overlapping backward: measured 1-1.5 %
    # SLOWER at world 1 on MI355X (BERT-base 11.84 vs 11.68 ms, ResNet-50 27.67 vs 27.35 ms;
    # profiles/r2_ab_overlap_optimizer.jsonl: the memory-bound updates contend with backward), so off
    overlap_optimizer: bool = False
    reduction: str = "average"         # average | adasum (Horovod op=hvd.Adasum; LR not scaled by world)
    metrics_dir: str | None = None
    checkpoint_every_epoch: bool = False
    seed: int = 0
    data_pool: int = 2                 # distinct synthetic batches cycled through
    graph: bool = True                 # capture the whole step in a hipGraph when world == 1 (graph-safe models)
    final_state_path: str | None = None  # rank 0 saves the final state (checkpoint format) here
    eval_batches: int = 0              # held-out synthetic batches evaluated after every epoch (0: no eval)
    report_progress: bool = False      # rank 0 publishes the committed step under job/<name>/progress
    progress_every_s: float = 1.0      # rank 0 rewrites <metrics_dir>/<job>.progress.json at most this often
    # lock-step oracle (tests): every step appends "step:world:lr:sha1(optimizer state)" to the
    # committed extras (workloads/replay.py); one host sync per step, never in production
    step_digests: bool = False
    # deterministic library kernels (MIOpen's deterministic solvers, no atomic split-K): a GPU
    # trajectory then repeats bit for bit, so the elastic-equivalence tests can compare a run with
    # its replay on real hardware; off in production (the atomic solvers are the fast ones)
    deterministic: bool = False


def build(cfg: TrainConfig, device: torch.device):
    w = get_workload(cfg.model)
    torch.manual_seed(cfg.seed)  # identical init everywhere (state is broadcast anyway)
    model = prepare_model(w, device, cfg.amp)
    kw = dict(w.opt_kwargs)
    if cfg.lr is not None:
        kw["lr"] = cfg.lr
    opt = make_optimizer(w.optimizer, model.parameters(), grad_dtype=GRAD_DTYPES[cfg.grad_dtype], **kw)
    return w, model, opt, kw["lr"]


GRAD_DTYPES = {"fp32": torch.float32, "bf16": torch.bfloat16, "fp16": torch.float16}


@contextlib.contextmanager
def deterministic_kernels(enabled: bool):
    """MIOpen's deterministic solvers for the duration of ONE job (cfg.deterministic), then the
    previous process-global flags again: a warm pool worker that hosted a deterministic job
    must not keep the slow solvers for every later job."""
    if not enabled:
        yield
        return
    prev = (torch.backends.cudnn.deterministic, torch.backends.cudnn.benchmark)
    torch.backends.cudnn.deterministic, torch.backends.cudnn.benchmark = True, False
    try:
        yield
    finally:
        torch.backends.cudnn.deterministic, torch.backends.cudnn.benchmark = prev


def synthetic_pool(w, cfg: TrainConfig, bs: int, device: torch.device) -> list:
    """The ``cfg.data_pool`` synthetic batches a job cycles through (seeded: every rank of
    every run of the job draws the same ones)."""
    g = torch.Generator(device=device).manual_seed(cfg.seed + 1)
    pool = []
    for _ in range(max(1, cfg.data_pool)):
        b = w.make_batch(bs, device, g)
        if w.channels_last and device.type == "cuda":
            b = tuple(t.to(memory_format=torch.channels_last) if t.dim() == 4 else t for t in b)
        pool.append(b)
    return pool


class _Warm:
    """A built workload kept resident on the worker's GPU between jobs (288 GB HBM): model,
    flat optimizer buffers, DDP hooks, synthetic batches and a device snapshot of the initial
    state.  A new job of the same kind re-initialises by one device copy instead of
    rebuilding -- job start / resize then costs only the rendezvous + state sync."""

    def __init__(self, cfg: TrainConfig, device: torch.device):
        self.w, self.model, self.opt, self.base_lr = build(cfg, device)
        self.bs = cfg.per_gpu_batch or self.w.per_gpu_batch
        self.pool = synthetic_pool(self.w, cfg, self.bs, device)
        self.ddp = ElasticDDP(self.model, None, self.opt, bucket_cap_mb=cfg.bucket_cap_mb,
                              compression=cfg.compression, reduction=cfg.reduction,
                              overlap_optimizer=cfg.overlap_optimizer)
        self._init = [t.detach().clone() for t in self._tensors()]
        self._rng0 = rng_state(device)  # generator state right after the seeded build
        self.device = device
        self.step_graph = None  # world-1 step captured by an earlier job (runtime/stepgraph.py)
        self._graph_hp = None   # optimizer hyperparameters baked into that capture

    @staticmethod
    def _hparams(opt) -> tuple:
        return tuple(tuple(sorted((k, v) for k, v in g.items() if k != "params" and isinstance(v, (int, float, bool))))
                     for g in opt.param_groups)

    def keep_graph(self, graph, opt) -> None:
        self.step_graph = graph
        self._graph_hp = self._hparams(opt)

    def reusable_graph(self, opt):
        """The cached step graph, when replaying it from a fresh optimizer state is exact: a
        capture bakes host scalars in (the LR, and the first-step flag of momentum buffers,
        captured as "not first"), so the hyperparameters must match the capture's and no
        group may use dampening (with dampening 0 the first step ``buf = d`` equals the
        general ``buf = m * 0 + d``).  Otherwise the job captures its own graph."""
        if self.step_graph is None or self._hparams(opt) != self._graph_hp:
            return None
        if any(float(g.get("dampening", 0.0) or 0.0) != 0.0 for g in opt.param_groups):
            return None
        return self.step_graph

    def _tensors(self):
        return self.opt.flat_state_tensors() + [b for b in self.model.buffers()]

    @torch.no_grad()
    def reset(self) -> None:
        for t, s in zip(self._tensors(), self._init):
            t.copy_(s)
        self.opt.after_external_update()
        self.opt.reset_steps()
        for g in self.opt.param_groups:
            g["lr"] = self.base_lr
        set_rng_state(self.device, self._rng0)  # a reused model draws the masks a fresh build would


_WARM: dict[tuple, _Warm] = {}
WARM_CACHE_MAX = 4


def _warm_key(cfg: TrainConfig, device: torch.device) -> tuple:
    return (cfg.model, cfg.per_gpu_batch, cfg.lr, cfg.compression, cfg.bucket_cap_mb, cfg.reduction, cfg.seed,
            cfg.grad_dtype, cfg.overlap_optimizer, cfg.amp, str(device))


def get_warm(cfg: TrainConfig, device: torch.device, use_cache: bool = True) -> _Warm:
    key = _warm_key(cfg, device)
    if use_cache and key in _WARM:
        wm = _WARM.pop(key)
        wm.reset()
        _WARM[key] = wm  # most recently used last
        return wm
    wm = _Warm(cfg, device)
    if use_cache:
        while len(_WARM) >= WARM_CACHE_MAX:
            old = _WARM.pop(next(iter(_WARM)))
            old.ddp.remove_hooks()
        _WARM[key] = wm
    return wm


class StepProfiler:
    """Fast online profiling: GPU-timed seconds per step at each world size.

    ``mark(step)`` at every commit records a timing event on the compute stream; events are
    resolved lazily once the GPU has passed them (``Event.query``), so no host sync is added.
    Consecutive resolved marks of one chain add ``(steps, seconds)`` to ``perf[world]``.  A
    chain restarts at every membership change, epoch boundary (eval / metric all-reduce are
    not training steps) and restore, and its first interval starts at the first commit (the
    hipGraph warm-up / capture steps are not timed).  ``perf`` lives in the elastic state's
    extras, so it is committed, restored and inherited by joining members like the step
    counter."""

    def __init__(self, device: torch.device):
        self.cuda = device.type == "cuda"
        self.marks: collections.deque = collections.deque()
        self.anchor = None

    def reset_chain(self) -> None:
        self.marks.clear()
        self.anchor = None

    def mark(self, step: int, world: int, perf: dict) -> None:
        if self.cuda:
            ev = torch.cuda.Event(enable_timing=True)
            ev.record()
        else:
            ev = time.perf_counter()
        self.marks.append((ev, step))
        self.resolve(world, perf)

    def resolve(self, world: int, perf: dict) -> None:
        while self.marks:
            ev, step = self.marks[0]
            if self.cuda and not ev.query():
                break
            self.marks.popleft()
            if self.anchor is not None:
                a_ev, a_step = self.anchor
                dt = a_ev.elapsed_time(ev) / 1e3 if self.cuda else ev - a_ev
                n = step - a_step
                if n > 0 and dt > 0:
                    rec = perf.setdefault(str(world), [0, 0.0])
                    rec[0] += n
                    rec[1] += dt
            self.anchor = (ev, step)


def write_progress(metrics_dir: str, job: str, doc: dict) -> None:
    """Atomically replace ``<metrics_dir>/<job>.progress.json`` (read by the collector)."""
    os.makedirs(metrics_dir, exist_ok=True)
    path = os.path.join(metrics_dir, f"{job}.progress.json")
    tmp = f"{path}.{os.getpid()}.tmp"
    with open(tmp, "w") as f:
        json.dump(doc, f)
    os.replace(tmp, path)


def train_elastic(ctx: ElasticContext, cfg: TrainConfig, use_cache: bool = True) -> dict | None:
    with deterministic_kernels(cfg.deterministic):
        return _train_elastic(ctx, cfg, use_cache)


def _train_elastic(ctx: ElasticContext, cfg: TrainConfig, use_cache: bool = True) -> dict | None:
    device = ctx.device
    wm = get_warm(cfg, device, use_cache)
    w, model, opt, base_lr, bs, pool, ddp = wm.w, wm.model, wm.opt, wm.base_lr, wm.bs, wm.pool, wm.ddp
    # world_log: flat [start_step, world, ...] segments -- the world size every step ran at.
    # Part of the synced / committed state, so a restore rolls it back with the step counter
    # and a joining member inherits it: ``replay_reference`` re-runs the same trajectory.
    # perf: {world: [steps, seconds]} measured by StepProfiler (fast online profiling)
    # steplog: lock-step digests (cfg.step_digests), committed / restored with the step counter
    state = TorchState(ctx, model, opt, epoch=0, samples=0, world_log=[], perf={}, steplog=[])
    logger = MetricsCSVLogger(cfg.metrics_dir, ctx.job, cfg.epochs, bs)
    samples_per_epoch = cfg.steps_per_epoch * bs
    stats = {"steps": 0, "samples": 0, "train_time": 0.0, "model": cfg.model, "resizes": 0}
    prof = StepProfiler(device)
    last_pub = [0.0]

    def publish(world: int, force: bool = False) -> None:
        """Rank 0: progress + per-world step times for the collector, at most once a second."""
        if not cfg.metrics_dir or ctx.rank != 0:
            return
        now = time.time()
        if not force and now - last_pub[0] < cfg.progress_every_s:
            return
        last_pub[0] = now
        prof.resolve(world, state.perf)
        try:
            write_progress(cfg.metrics_dir, ctx.job, {
                "job": ctx.job, "t": now, "world": world, "per_gpu_batch": bs, "epoch": state.epoch,
                "epochs": cfg.epochs, "samples_done": state.epoch * samples_per_epoch + state.samples,
                "samples_total": cfg.epochs * samples_per_epoch, "perf": state.perf})
        except OSError:
            log.warning("%s: cannot write the progress file", ctx.job, exc_info=True)

    def on_reset():
        stats["resizes"] += 1

    state.register_reset_callbacks([on_reset])

    def step_fn(batch):
        ddp.zero_grad()
        # autocast's weight-cast cache must be off inside a captured graph
        with torch.autocast(device.type, dtype=torch.bfloat16, enabled=cfg.amp and device.type == "cuda",
                            cache_enabled=False):
            loss, correct, n = w.loss_metrics(model, batch)
        loss.backward()
        ddp.step()
        # [loss, #correct, #predictions] on the device: no host sync per step
        return torch.stack([loss.detach().float(), correct.float(), n.float()])

    eval_pool = None
    if cfg.eval_batches > 0:
        g = torch.Generator(device=device).manual_seed(cfg.seed + 7919)  # held out from the training pool
        eval_pool = [w.make_batch(bs, device, g) for _ in range(cfg.eval_batches)]
        if w.channels_last and device.type == "cuda":
            eval_pool = [tuple(t.to(memory_format=torch.channels_last) if t.dim() == 4 else t for t in b)
                         for b in eval_pool]

    @torch.no_grad()
    def evaluate() -> tuple[float, float]:
        """Validation pass (reference ``test()``, pytorch_mnist_elastic.py:155-176): the
        held-out batches are sharded over the current members, per-rank sums are all-reduced,
        so the result is the exact global mean whatever the world size."""
        model.eval()
        tot = torch.zeros(3, device=device, dtype=torch.float32)
        try:
            for i in range(ctx.rank if ctx.rank >= 0 else 0, len(eval_pool), max(1, ctx.size)):
                with torch.autocast(device.type, dtype=torch.bfloat16, enabled=cfg.amp and device.type == "cuda",
                                    cache_enabled=False):
                    loss, correct, n = w.loss_metrics(model, eval_pool[i])
                tot += torch.stack([loss.float() * n.float(), correct.float(), n.float()])
        finally:
            model.train()
        s_loss, s_corr, s_n = ctx.allreduce_values(tot, "sum")
        return s_loss / max(s_n, 1.0), s_corr / max(s_n, 1.0)

    @run
    def train(state):
        ddp.set_communicator(ctx.comm)
        world = ctx.size
        lr_scaler = 1 if cfg.reduction == "adasum" else world  # Horovod examples: Adasum keeps the base LR
        for gr in opt.param_groups:
            gr["lr"] = base_lr * lr_scaler
        state.world_log = list(state.world_log) + [state.step, world]
        logger.set_params(world)
        # world 1: the whole step replays as one hipGraph (launch-bound models); collectives
        # of world > 1 stay eager.  Re-captured after every membership change.
        stepper = GraphedStepper(step_fn, model, opt, warmup=2,
                                 enabled=cfg.graph and w.graph_safe and world == 1 and device.type == "cuda",
                                 graph=wm.reusable_graph(opt) if use_cache else None)
        loss_t = None
        while state.epoch < cfg.epochs:
            t_ep = time.time()
            prof.reset_chain()
            steps = 0
            ep_acc = torch.zeros(3, device=device)  # sum over steps of [loss, #correct, #predictions]
            guard = torch.zeros((), device=device)  # graph replays: loss sum since the last commit
            while state.samples < samples_per_epoch:
                batch = pool[state.step % len(pool)]
                with trace_range("train_step", "train", world=world):
                    m_t = stepper(batch)
                ep_acc += m_t
                loss_t = m_t[0]
                if stepper.graph is not None:
                    guard += m_t[0]
                state.samples += bs * world
                state.step += 1
                steps += 1
                if cfg.step_digests:  # every member: the log is state, synced from any holder
                    from .replay import step_record

                    state.steplog = list(state.steplog) + [
                        step_record(state.step, world, float(opt.param_groups[0]["lr"]), opt.flat_state_tensors())]
                stats["steps"] += 1
                stats["samples"] += bs * world
                if state.step % cfg.commit_every == 0:
                    if stepper.graph is not None:
                        # replay guard (one host sync per commit): a captured step whose library
                        # kernels misbehave on replay shows up as a non-finite loss; roll back to
                        # the last commit and continue eagerly (docs/kernels.md, hipGraph section)
                        if not bool(torch.isfinite(guard)):
                            log.warning("%s: non-finite loss under graph replay; restoring step %d, eager from now on",
                                        ctx.job, ctx.committed_step)
                            stepper.release()
                            stepper.enabled = False
                            wm.step_graph = None
                            state.restore()
                            stats["graph_fallbacks"] = stats.get("graph_fallbacks", 0) + 1
                            prof.reset_chain()
                            ep_acc.zero_()
                            steps = 0
                            guard.zero_()
                            continue
                        guard.zero_()
                    prof.mark(state.step, world, state.perf)
                    state.commit()
                    publish(world)
                    if cfg.report_progress and ctx.rank == 0:
                        ctx.rdzv.set("progress", str(state.step))
            if device.type == "cuda":
                torch.cuda.synchronize(device)
            ep_time = time.time() - t_ep
            stats["train_time"] += ep_time
            # epoch training loss / accuracy averaged over the members (metric_average); the
            # steps since this membership began (a resize restarts the epoch's tally)
            loc = ep_acc.tolist()
            mean_loss = loc[0] / steps if steps else float("nan")
            acc = loc[1] / loc[2] if loc[2] > 0 else float("nan")
            mean_loss, acc = ctx.allreduce_values([mean_loss, acc], "avg")
            val = evaluate() if eval_pool is not None else (None, None)
            if ctx.rank == 0:
                logger.log_epoch(state.epoch, t_ep, ep_time, steps, None if steps == 0 else mean_loss, world,
                                 acc=None if acc != acc else acc, val_loss=val[0], val_acc=val[1])
            stats.setdefault("epoch_metrics", []).append({"loss": mean_loss, "acc": acc, "val_loss": val[0],
                                                          "val_acc": val[1], "world": world})
            prof.resolve(world, state.perf)  # the epoch-end sync passed every mark
            state.epoch += 1
            state.samples = 0
            state.commit()
            publish(world, force=True)
            if cfg.checkpoint_every_epoch and ctx.rank == 0:
                state.save_checkpoint()
        if device.type == "cuda":
            torch.cuda.synchronize(device)
        if use_cache and stepper.graph is not None:
            wm.keep_graph(stepper.graph, opt)  # the next job of this kind replays it directly
        digest = None
        if cfg.final_state_path:
            if ctx.rank == 0:
                state.save_checkpoint(cfg.final_state_path)
            # every member's final state, hashed: the members must hold bitwise-identical state
            h = hashlib.sha1()
            for t in state.tensors():
                h.update(t.detach().contiguous().cpu().view(-1).view(torch.uint8).numpy().tobytes())
            digest = h.hexdigest()
        return dict(stats, final_loss=float(loss_t) if loss_t is not None else None, world=ctx.size,
                    final_step=state.step, world_log=list(state.world_log), state_digest=digest,
                    perf={k: list(v) for k, v in state.perf.items()}, per_gpu_batch=bs)

    try:
        return train(state)
    finally:
        ddp.comm = None  # never keep a dead epoch's communicator alive in the warm cache
        if not use_cache:
            ddp.remove_hooks()


def replay_reference(cfg: TrainConfig, world_log: list[int], total_steps: int, device: torch.device):
    with deterministic_kernels(cfg.deterministic):
        return _replay_reference(cfg, world_log, total_steps, device)


def _replay_reference(cfg: TrainConfig, world_log: list[int], total_steps: int, device: torch.device):
    """Uninterrupted single-process replay of an elastic run: step ``s`` runs at the world
    size of the last ``world_log`` segment starting at or before ``s`` (LR = base x world,
    the same synthetic batch every rank of the elastic run used).  The elastic run's final
    state must equal this one -- exactly for worlds whose all-reduce average of identical
    per-rank gradients is exact (1, 2) -- whatever resizes, halts and restores happened.
    Returns (state tensors, extras)."""
    w, model, opt, base_lr = build(cfg, device)
    bs = cfg.per_gpu_batch or w.per_gpu_batch
    pool = synthetic_pool(w, cfg, bs, device)
    ddp = ElasticDDP(model, None, opt, bucket_cap_mb=cfg.bucket_cap_mb, compression=cfg.compression,
                     reduction=cfg.reduction, overlap_optimizer=cfg.overlap_optimizer)
    segs = [(world_log[i], world_log[i + 1]) for i in range(0, len(world_log), 2)]

    def world_at(step: int) -> int:
        wd = segs[0][1]
        for st, wv in segs:
            if st <= step:
                wd = wv
        return wd

    samples_per_epoch = cfg.steps_per_epoch * bs
    epoch = samples = 0
    steplog: list[str] = []
    for step in range(total_steps):
        world = world_at(step)
        lr_scaler = 1 if cfg.reduction == "adasum" else world
        for gr in opt.param_groups:
            gr["lr"] = base_lr * lr_scaler
        ddp.zero_grad()
        with torch.autocast(device.type, dtype=torch.bfloat16, enabled=cfg.amp and device.type == "cuda",
                            cache_enabled=False):
            loss = w.loss_metrics(model, pool[step % len(pool)])[0]
        loss.backward()
        ddp.step()
        samples += bs * world
        if samples >= samples_per_epoch:
            epoch, samples = epoch + 1, 0
        if cfg.step_digests:
            from .replay import step_record

            steplog.append(step_record(step + 1, world, float(opt.param_groups[0]["lr"]), opt.flat_state_tensors()))
    for m in model.modules():  # host-side BN counters -> buffers (as TorchState.tensors)
        if hasattr(m, "sync_batches_tracked"):
            m.sync_batches_tracked()
    ts = opt.flat_state_tensors() + [b for b in model.buffers() if b.dtype.is_floating_point or b.dtype == torch.int64]
    return [t.detach().cpu() for t in ts], {"epoch": epoch, "samples": samples, "__step__": total_steps,
                                            "steplog": steplog}


@torch.no_grad()
def evaluate_checkpoint(cfg: TrainConfig, path: str, device: torch.device) -> tuple[float, float]:
    """Single-process evaluation of a saved elastic state on the trainer's held-out batches
    (the reference's ``test()`` run once, pytorch_mnist_elastic.py:155-176): the exact global
    mean loss / accuracy the distributed eval pass must reproduce."""
    w, model, opt, _ = build(cfg, device)
    payload = torch.load(path, map_location=device, weights_only=True)
    ts = opt.flat_state_tensors() + [b for b in model.buffers() if b.dtype.is_floating_point or b.dtype == torch.int64]
    if len(ts) != len(payload["tensors"]):
        raise ValueError("checkpoint does not match the workload's state layout")
    for t, v in zip(ts, payload["tensors"]):
        t.copy_(v)
    opt.after_external_update()
    bs = cfg.per_gpu_batch or w.per_gpu_batch
    g = torch.Generator(device=device).manual_seed(cfg.seed + 7919)
    model.eval()
    s_loss = s_corr = s_n = 0.0
    for _ in range(cfg.eval_batches):
        b = w.make_batch(bs, device, g)
        with torch.autocast(device.type, dtype=torch.bfloat16, enabled=cfg.amp and device.type == "cuda",
                            cache_enabled=False):
            loss, correct, n = w.loss_metrics(model, b)
        s_loss += float(loss) * float(n)
        s_corr += float(correct)
        s_n += float(n)
    return s_loss / max(s_n, 1.0), s_corr / max(s_n, 1.0)


def main(argv=None):
    ap = argparse.ArgumentParser("vodascheduler_amd.workloads.train")
    ap.add_argument("--model", required=True)
    ap.add_argument("--name", default=os.environ.get("JOB_NAME", "job"))
    ap.add_argument("--epochs", type=int, default=1)
    ap.add_argument("--steps-per-epoch", type=int, default=10)
    ap.add_argument("--batch-size", type=int, default=None)
    ap.add_argument("--lr", type=float, default=None)
    ap.add_argument("--commit-every", type=int, default=1)
    ap.add_argument("--fp16-allreduce", action="store_true")
    ap.add_argument("--compression", default=None)
    ap.add_argument("--use-adasum", action="store_true", help="Adasum gradient reduction instead of averaging")
    ap.add_argument("--metrics-dir", default=os.environ.get("VODA_METRICS_DIR"))
    ap.add_argument("--no-amp", action="store_true")
    a = ap.parse_args(argv)
    logging.basicConfig(level=logging.INFO)
    from ..runtime.rendezvous import connect_store

    host, port = os.environ["VODA_STORE"].rsplit(":", 1)
    store = connect_store(host, int(port))
    watch = connect_store(host, int(port))
    dev = torch.device("cuda", 0) if torch.cuda.is_available() else torch.device("cpu")
    if dev.type == "cuda":
        torch.cuda.set_device(dev)
    ctx = ElasticContext(store, a.name, os.environ["VODA_WORKER_ID"], dev, watch_store=watch,
                         join_epoch=int(os.environ.get("VODA_JOIN_EPOCH", "0")))
    cfg = TrainConfig(a.model, a.epochs, a.steps_per_epoch, a.batch_size, a.lr, a.commit_every, not a.no_amp,
                      "fp16" if a.fp16_allreduce else a.compression, metrics_dir=a.metrics_dir,
                      reduction="adasum" if a.use_adasum else "average")
    out = train_elastic(ctx, cfg)
    log.info("worker %s finished job %s: %s", ctx.worker_id, a.name, out)


if __name__ == "__main__":
    main()
