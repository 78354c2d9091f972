"""Whole-training-step hipGraph capture for launch-bound jobs.

InceptionV3, VGG16, the MNIST nets and the NMT Transformer issue hundreds of small kernels
per step; on MI355X their GPU is busy only 35-50 % of the step in eager mode (rocprofv3,
profiles/) because the host cannot launch fast enough.  A captured step (zero_grad,
forward under autocast, backward, fused optimizer) replays as ONE graph launch.

Everything the step touches must be graph-safe, and is in this framework:
* every HIP kernel launches on ``torch.cuda.current_stream()`` with no host sync / allocation
  outside the caching allocator;
* the fused optimizers read their step counters from device memory (``_step_t``), so Adam's
  bias correction advances on every replay;
* gradients live in flat buffers allocated outside the graph; ``zero_grad`` is a captured memset.
Host-side counters that the captured Python ran once are re-synced per replay.

Only world-size-1 steps are captured (collectives stay eager), after ``warmup`` eager steps
on a side stream (MIOpen find, hipBLASLt heuristics, allocator warm-up).
"""
from __future__ import annotations

import logging
from typing import Callable, Sequence

import torch

log = logging.getLogger("vodascheduler_amd.stepgraph")


def _bn_modules(model: torch.nn.Module) -> list:
    return [m for m in model.modules() if hasattr(m, "sync_batches_tracked")]


class StepGraph:
    """``step_fn(batch) -> loss`` captured once; ``replay(batch)`` copies the batch into the
    static inputs and launches the graph."""

    def __init__(self, step_fn: Callable[[Sequence[torch.Tensor]], torch.Tensor], example: Sequence[torch.Tensor],
                 model: torch.nn.Module | None = None, optimizer=None):
        self.static = tuple(t.detach().clone() for t in example)
        self.optimizer = optimizer
        self.bns = _bn_modules(model) if model is not None else []
        before = [getattr(m, "_pending_batches", 0) for m in self.bns]
        steps_before = list(getattr(optimizer, "_steps", []))
        self.graph = torch.cuda.CUDAGraph()
        with torch.cuda.graph(self.graph):
            self.loss = step_fn(self.static).detach()
        # the captured Python ran once without executing anything: undo its host counters
        for m, b in zip(self.bns, before):
            m._pending_batches = b
        if optimizer is not None and steps_before:
            optimizer._steps = steps_before

    def replay(self, batch: Sequence[torch.Tensor]) -> torch.Tensor:
        for s, b in zip(self.static, batch):
            if s.data_ptr() != b.data_ptr():
                s.copy_(b, non_blocking=True)
        self.graph.replay()
        if self.optimizer is not None and hasattr(self.optimizer, "advance_host_steps"):
            self.optimizer.advance_host_steps(1)
        for m in self.bns:
            if m.momentum is not None:
                m._pending_batches = getattr(m, "_pending_batches", 0) + 1
        return self.loss


class GraphedStepper:
    """Runs training steps eagerly for ``warmup`` steps on a side stream, then captures and
    replays.  Falls back to eager for good if capture fails."""

    def __init__(self, step_fn, model=None, optimizer=None, warmup: int = 2, enabled: bool = True,
                 graph: "StepGraph | None" = None):
        """``graph``: a step captured earlier for the same model / optimizer / batch shapes (a
        warm worker's next job of the same kind replays it without warm-up or capture)."""
        self.step_fn = step_fn
        self.model = model
        self.optimizer = optimizer
        self.warmup = warmup
        self.enabled = enabled and torch.cuda.is_available()
        self.graph: StepGraph | None = graph if self.enabled else None
        self.eager_steps = 0
        self._side = None

    def __call__(self, batch) -> torch.Tensor:
        if self.graph is not None:
            return self.graph.replay(batch)
        if not self.enabled:
            return self.step_fn(batch)
        if self.eager_steps >= self.warmup:
            try:
                torch.cuda.current_stream().synchronize()
                self.graph = StepGraph(self.step_fn, batch, self.model, self.optimizer)
                return self.graph.replay(batch)
            except Exception as e:  # never fail the job on a capture problem
                log.warning("step capture failed (%s); continuing eagerly", e)
                self.enabled = False
                self.graph = None
                torch.cuda.synchronize()
                return self.step_fn(batch)
        if self._side is None:
            self._side = torch.cuda.Stream()
        self._side.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(self._side):
            loss = self.step_fn(batch)
        torch.cuda.current_stream().wait_stream(self._side)
        self.eager_steps += 1
        return loss

    def release(self) -> None:
        self.graph = None
