"""Bucketed gradient all-reduce overlapped with backward (Horovod DistributedOptimizer
replacement; reference hvd.DistributedOptimizer(op=hvd.Average) in
examples/py/pytorch/pytorch_mnist_elastic.py:185-188).

MI355X-first design:
* gradients live in ONE flat buffer per parameter group (the fused optimizer's
  ``FlatGroup``, or a grad-only one), so a bucket is a contiguous SLICE -- no fusion-buffer
  copy on the hot path;
* buckets cover the flat buffer back-to-front (the order gradients become ready in
  backward) and are cut at parameter boundaries to ``bucket_cap_mb`` (default 64 MB: an
  8-GPU ring on 7 xGMI links needs >~43 MB per collective to amortise per-step latency,
  SURVEY.md §5.8; the first bucket is kept small so communication starts early);
* a post-accumulate-grad hook counts ready parameters; a full bucket is enqueued on a
  dedicated HIP stream (ordered after the producing compute via a stream wait), strictly in
  bucket order on every rank (collective order must match across ranks);
* averaging folds into the collective (RCCL ncclAvg) or, with ``compression='bf16'|'fp16'``
  (Horovod's fp16 compression), into the HIP cast kernel that packs the comm buffer
  (scale 1/N) -- halving xGMI bytes;
* ``reduction='adasum'`` (Horovod ``op=hvd.Adasum``, pytorch_mnist_elastic.py:188) instead
  all-gathers the bucket and runs the deterministic per-parameter Adasum tree of
  ``ops/adasum.py`` on every rank (HIP segmented combine kernels);
* ``finalize()`` flushes buckets whose parameters got no gradient this step (zeros) and makes
  the compute stream wait for the comm stream before the optimizer step;
* readiness is counted per parameter against the number of gradient contributions the
  parameter received in a calibration step (the first synced step: no overlap, every bucket
  launched by ``finalize``).  A parameter a fused layer signals itself AND autograd
  accumulates (or one used by two fused layers) therefore never launches its bucket early --
  a bucket launched before its last contribution would all-reduce a partial gradient and
  let the ranks diverge silently.  (Static-graph assumption, as PyTorch DDP's
  ``static_graph``; a step that deviates is detected at ``finalize`` and logged.)
"""
from __future__ import annotations

import logging
from contextlib import contextmanager
from dataclasses import dataclass

import torch

from ..ops.adasum import AdasumPlan, adasum_tree_
from ..ops.bucket import cast_scale_
from ..utils.flat import FlatGroup
from .comm import Communicator, LocalCommunicator

_COMPRESS = {None: None, "none": None, "bf16": torch.bfloat16, "fp16": torch.float16}
log = logging.getLogger("vodascheduler_amd.ddp")


@dataclass
class Bucket:
    group: int
    start: int           # element offset in the group's flat grad buffer
    end: int
    params: list[torch.nn.Parameter]
    pending: int = 0
    launched: bool = False
    comm_buf: torch.Tensor | None = None
    segments: list[tuple[int, int]] | None = None   # per-parameter ranges, relative to start
    plan: AdasumPlan | None = None
    opt_done: bool = False   # the optimizer update of this bucket ran this step

    @property
    def numel(self) -> int:
        return self.end - self.start


class ElasticDDP:
    """Bucketed gradient all-reduce engine (see module docstring).

    ``overlap_optimizer`` (opt-in; the trainer turns it on with a fused flat optimizer): the optimizer
    update of a bucket's parameters runs on the comm stream right after the bucket's
    all-reduce -- overlapping the remaining backward -- instead of one whole-model optimizer
    pass after backward.  Safe because a bucket launches only after every gradient
    contribution of its parameters, i.e. after every backward node that reads those weights
    has been enqueued on the compute stream, which the comm stream waits for.  At world 1
    the same per-bucket updates overlap backward with no collective.  With it on, finish a
    step with ``step()`` (``finalize()`` alone also completes the updates already begun)."""

    def __init__(self, model: torch.nn.Module, comm: Communicator, optimizer=None, bucket_cap_mb: float = 64.0,
                 first_bucket_mb: float = 8.0, compression: str | None = None, reduction: str = "average",
                 overlap_optimizer: bool = False):
        if reduction not in ("average", "adasum"):
            raise ValueError(f"unknown reduction {reduction!r} (average | adasum)")
        self.model = model
        self.reduction = reduction
        self.comm = comm
        self.optimizer = optimizer
        self.compress_dtype = _COMPRESS[compression]
        if optimizer is not None and hasattr(optimizer, "flat_groups"):
            self.groups: list[FlatGroup] = list(optimizer.flat_groups)
        else:
            # grad-only mode (no optimizer, or a stock torch.optim one that reads p.grad): the
            # flat gradient keeps each parameter's own dtype, so gradients stay visible in
            # p.grad -- an fp32 flat buffer for bf16 parameters would fold them away from it
            by_dtype: dict[torch.dtype, list] = {}
            for p in model.parameters():
                if p.requires_grad:
                    by_dtype.setdefault(p.dtype, []).append(p)
            self.groups = [FlatGroup(ps, flatten_params=False, grad_dtype=dt) for dt, ps in by_dtype.items()]
        self.device = self.groups[0].device
        self.overlap_optimizer = bool(overlap_optimizer and optimizer is not None
                                      and hasattr(optimizer, "step_range") and self.device.type == "cuda")
        self.bucket_cap_mb = bucket_cap_mb
        self.first_bucket_mb = first_bucket_mb
        self._build_buckets()
        self._hooks = []
        self._sync = True
        self._expect: dict[int, int] | None = None   # contributions per parameter per step
        self._count: dict[int, int] = {}
        self._param_bucket: dict[int, Bucket] = {}
        for b in self.buckets:
            for p in b.params:
                self._param_bucket[id(p)] = b
        for g in self.groups:
            for p in g.params:
                if p.requires_grad:
                    self._hooks.append(p.register_post_accumulate_grad_hook(self._on_grad))
                    # layers that accumulate into the flat buffer themselves (ops/dense.py)
                    # signal readiness through this attribute instead of autograd's hook
                    p._voda_grad_ready = self._on_grad
        self._next = 0
        self._opt_begun = False
        self.comm_stream = torch.cuda.Stream(self.device) if self.device.type == "cuda" else None
        if comm is not None and hasattr(comm, "stream") and self.comm_stream is not None:
            comm.stream = self.comm_stream
        self._reset()

    # ------------------------------------------------------------------ setup
    def _build_buckets(self) -> None:
        self.buckets: list[Bucket] = []
        for gi, g in enumerate(self.groups):
            esz = g.grad.element_size()
            idx = list(range(len(g.params)))[::-1]  # back-to-front: backward order
            cur: list[int] = []
            cap = self.first_bucket_mb
            for i in idx:
                cur.append(i)
                nbytes = (g.slots[cur[0]].offset + g.slots[cur[0]].numel - g.slots[i].offset) * esz
                if nbytes >= cap * 2 ** 20:
                    self._close(gi, cur)
                    cur = []
                    cap = self.bucket_cap_mb
            if cur:
                self._close(gi, cur)

    def _close(self, gi: int, idxs: list[int]) -> None:
        g = self.groups[gi]
        lo = min(g.slots[i].offset for i in idxs)
        hi_i = max(idxs, key=lambda i: g.slots[i].offset)
        hi = g.slots[hi_i].offset + g.slots[hi_i].numel
        # extend to the padded end so the bucket slices tile the flat buffer exactly
        nxt = [g.slots[i].offset for i in range(len(g.params)) if g.slots[i].offset >= hi]
        hi = min(nxt) if nxt else g.numel
        offs = sorted(g.slots[i].offset for i in idxs)
        segs = [(o - lo, (offs[k + 1] if k + 1 < len(offs) else hi) - lo) for k, o in enumerate(offs)]
        self.buckets.append(Bucket(gi, lo, hi, [g.params[i] for i in idxs], segments=segs))

    def bucket_sizes_mb(self) -> list[float]:
        return [b.numel * self.groups[b.group].grad.element_size() / 2 ** 20 for b in self.buckets]

    @property
    def world(self) -> int:
        return 1 if self.comm is None else self.comm.size

    def _reset(self) -> None:
        self._next = 0
        self._count = {}
        self._opt_begun = False
        for b in self.buckets:
            if self._expect is None:
                b.pending = sum(1 for p in b.params if p.requires_grad)
            else:
                b.pending = sum(self._expect.get(id(p), 0) for p in b.params)
            b.launched = False
            b.opt_done = False

    @property
    def calibrated(self) -> bool:
        return self._expect is not None

    def _overlap_active(self) -> bool:
        # never inside a hipGraph capture: the captured step runs the whole-model update
        return self.overlap_optimizer and not torch.cuda.is_current_stream_capturing()

    def _launching(self) -> bool:
        """Do buckets launch during backward this step?"""
        return self._sync and (self.world > 1 or self._overlap_active())

    # ------------------------------------------------------------------ hooks
    def _on_grad(self, p: torch.nn.Parameter) -> None:
        if not self._sync:
            return
        if self._expect is None:  # calibration step: count contributions, launch at finalize
            self._count[id(p)] = self._count.get(id(p), 0) + 1
            return
        if not self._launching():
            return
        b = self._param_bucket[id(p)]
        b.pending -= 1
        if b.pending == 0:
            self._launch_ready()

    def _launch_ready(self) -> None:
        while self._next < len(self.buckets) and self.buckets[self._next].pending <= 0:
            self._launch(self.buckets[self._next])
            self._next += 1

    def _launch(self, b: Bucket, apply_opt: bool = True) -> None:
        g = self.groups[b.group]
        flat = g.grad[b.start:b.end]
        use_opt = apply_opt and self._overlap_active()
        if use_opt and not self._opt_begun:
            self.optimizer.begin_step()  # step counters, on the compute stream
            self._opt_begun = True
        if self.comm_stream is not None:
            self.comm_stream.wait_stream(torch.cuda.current_stream(self.device))
            ctx = torch.cuda.stream(self.comm_stream)
        else:
            ctx = _nullctx()
        with ctx:
            if self.world > 1:
                if self.reduction == "adasum":
                    if b.plan is None:
                        b.plan = AdasumPlan(b.segments, flat.device)
                    gathered = self.comm.allgather(flat)          # [world, n]
                    flat.copy_(adasum_tree_(gathered, b.plan))
                elif self.compress_dtype is not None and flat.dtype != self.compress_dtype:
                    if b.comm_buf is None:
                        b.comm_buf = torch.empty(b.numel, dtype=self.compress_dtype, device=flat.device)
                    cast_scale_(flat, b.comm_buf, 1.0 / self.world)
                    self.comm.allreduce_(b.comm_buf, "sum")
                    cast_scale_(b.comm_buf, flat, 1.0)
                else:
                    self.comm.allreduce_(flat, "avg")
            if use_opt:
                self.optimizer.step_range(b.group, b.start, b.end)
                b.opt_done = True
        b.launched = True

    # ------------------------------------------------------------------ API
    def forward(self, *a, **kw):
        return self.model(*a, **kw)

    __call__ = forward

    @contextmanager
    def no_sync(self):
        """Accumulate gradients locally (no all-reduce) inside the context."""
        old = self._sync
        self._sync = False
        try:
            yield
        finally:
            self._sync = old

    def _flush(self, apply_opt: bool) -> None:
        """Calibration bookkeeping + launch every bucket not yet launched, then order the
        compute stream after the comm stream."""
        if self._sync and self._expect is None and self._count:
            self._expect = dict(self._count)  # calibration step done: every bucket launches below
        elif self._sync and self.world > 1:
            bad = [i for i, b in enumerate(self.buckets) if b.pending < 0]
            if bad:
                log.error("buckets %s received more gradient contributions than in the calibration step "
                          "(dynamic graph?): their all-reduce may have started early", bad)
        if self._sync and (self.world > 1 or (apply_opt and self._overlap_active())):
            while self._next < len(self.buckets):
                self._launch(self.buckets[self._next], apply_opt)
                self._next += 1
            if self.comm_stream is not None:
                torch.cuda.current_stream(self.device).wait_stream(self.comm_stream)

    def finalize(self) -> None:
        """Flush remaining buckets (gradients only) and order the compute stream after them."""
        self._flush(apply_opt=False)
        if self._opt_begun:  # some buckets already applied their update: finish the rest
            self._apply_remaining_updates()
        self._reset()

    def _apply_remaining_updates(self) -> None:
        for b in self.buckets:
            if not b.opt_done:
                self.optimizer.step_range(b.group, b.start, b.end)
                b.opt_done = True

    def allreduce_gradients(self) -> None:
        """Synchronous all-reduce of all gradients (no overlap); for debugging/tests."""
        if self.world == 1:
            return
        self._launch_ready_all()
        self.finalize()

    def _launch_ready_all(self) -> None:
        while self._next < len(self.buckets):
            self._launch(self.buckets[self._next], apply_opt=False)
            self._next += 1

    def step(self) -> None:
        """Finish the step: all-reduce what is left and apply the optimizer update (per
        bucket on the comm stream when overlapping, else one whole-model pass)."""
        if self.optimizer is None:
            self.finalize()
            return
        if self._sync and self._overlap_active():
            self._flush(apply_opt=True)
            if not self._opt_begun:
                self.optimizer.begin_step()
                self._opt_begun = True
            self._apply_remaining_updates()
            self._reset()
            return
        self.finalize()
        self.optimizer.step()

    def zero_grad(self) -> None:
        for g in self.groups:
            g.zero_grad()
        self._reset()

    def set_communicator(self, comm: Communicator) -> None:
        """Swap in the communicator of a new membership epoch (elastic resize)."""
        self.comm = comm
        if hasattr(comm, "stream") and self.comm_stream is not None:
            comm.stream = self.comm_stream
        self._reset()

    def remove_hooks(self) -> None:
        for h in self._hooks:
            h.remove()
        self._hooks = []
        for g in self.groups:
            for p in g.params:
                if getattr(p, "_voda_grad_ready", None) == self._on_grad:
                    p._voda_grad_ready = None


@contextmanager
def _nullctx():
    yield


def broadcast_tensors(comm: Communicator, tensors: list[torch.Tensor], root: int = 0,
                      small_bytes: int = 1 << 20) -> None:
    """Broadcast a list of tensors from ``root`` in place (state sync on elastic resize).

    Tensors under ``small_bytes`` (BN statistics, biases, step counters: hundreds per model)
    are packed per dtype into one flat buffer and sent as ONE collective instead of one
    latency-bound collective each; large tensors (the flat parameter / optimizer-slot
    buffers) are broadcast in place.  Non-contiguous tensors go through a contiguous copy that
    is written back."""
    if comm is None or isinstance(comm, LocalCommunicator) or comm.size == 1:
        return
    small: dict[torch.dtype, list[torch.Tensor]] = {}
    for t in tensors:
        if t.numel() == 0:
            continue
        if t.numel() * t.element_size() < small_bytes:
            small.setdefault(t.dtype, []).append(t)
        elif t.is_contiguous():
            comm.broadcast_(t, root)
        else:
            c = t.contiguous()
            comm.broadcast_(c, root)
            with torch.no_grad():
                t.copy_(c)
    for dt, ts in small.items():
        flat = torch.cat([t.detach().reshape(-1) for t in ts])
        comm.broadcast_(flat, root)
        with torch.no_grad():
            off = 0
            for t in ts:
                n = t.numel()
                t.copy_(flat[off:off + n].view_as(t))
                off += n
