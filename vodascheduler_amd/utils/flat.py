"""Flat (contiguous) parameter / gradient storage.

Every parameter of a group is re-pointed into ONE contiguous buffer (fp32 master, plus an
optional low-precision copy the model computes with) and every gradient into ONE
contiguous buffer.  This is the layout the fused HIP optimizers (one launch per group) and
the bucketed all-reduce engine (buckets are slices of the flat gradient buffer, no pack
step) are built around.  Each tensor starts on a 64-element boundary so every slice is
>= 128-byte aligned for the 8/16-B vector loads of the kernels.  On a 288 GB MI355X the
padding and the resident snapshots (``snapshot()``) are free.

Gradient precision: the flat gradient buffer is fp32 by default, also for a model whose
GEMM/conv weights are stored in bf16 (Horovod reduces fp32 gradients unless
``--fp16-allreduce`` is given; reference pytorch_mnist_elastic.py:116).  Such a parameter
cannot carry an fp32 ``.grad`` (autograd requires grad dtype == param dtype), so its flat
gradient view is published as ``p._voda_gview`` instead:
* the fused layers (ops/dense.py, conv1x1.py, conv3x3.py, layernorm.py, batchnorm.py)
  accumulate their weight gradients straight into it (the MFMA weight-gradient kernels
  round their fp32 accumulators once, into fp32);
* for every other op autograd produces the usual bf16 ``.grad``; a post-accumulate hook
  adds it into the fp32 slot and drops it (one small cast-add per such parameter).
``grad_of(p)`` returns the flat gradient view in either mode.
"""
from __future__ import annotations

import os

from dataclasses import dataclass

import torch

ALIGN_ELEMS = 64


def _pad(n: int) -> int:
    return (n + ALIGN_ELEMS - 1) // ALIGN_ELEMS * ALIGN_ELEMS


def _dense_extent(t: torch.Tensor) -> bool:
    """True if ``t`` covers a dense block of numel() elements (any permuted layout)."""
    if t.numel() == 0:
        return True
    span = 1 + sum((s - 1) * st for s, st in zip(t.shape, t.stride()) if s > 1)
    return span == t.numel()


@dataclass
class Slot:
    offset: int
    numel: int


def grad_of(p: torch.Tensor) -> torch.Tensor | None:
    """The optimizer-owned flat gradient view of ``p`` (any dtype), else ``p.grad``."""
    g = getattr(p, "_voda_gview", None)
    return g if g is not None else p.grad


def flat_grad(p: torch.Tensor | None) -> torch.Tensor | None:
    """The flat gradient view a fused layer may accumulate into in place, or None."""
    if p is None:
        return None
    return getattr(p, "_voda_gview", None)


class FlatGroup:
    """Contiguous storage for a list of parameters.

    Args:
        params: parameters (all on one device).
        flatten_params: re-point ``p.data`` into the flat buffers (needed by the fused
            optimizers); False keeps the parameters where they are and only flattens
            gradients (the all-reduce engine's grad-only mode).
        grad_dtype: dtype of the flat gradient buffer (default: fp32).
    """

    def __init__(self, params, flatten_params: bool = True, grad_dtype: torch.dtype | None = None):
        self.params: list[torch.nn.Parameter] = [p for p in params]
        if not self.params:
            raise ValueError("FlatGroup needs at least one parameter")
        devs = {p.device for p in self.params}
        if len(devs) != 1:
            raise ValueError(f"parameters live on several devices: {devs}")
        self.device = devs.pop()
        pdts = {p.dtype for p in self.params}
        if len(pdts) != 1:
            raise ValueError(f"mixed parameter dtypes in one group: {pdts}")
        self.param_dtype = pdts.pop()
        self.grad_dtype = grad_dtype or torch.float32
        # mixed: bf16/fp16 parameters with an fp32 flat gradient (see module docstring)
        self.mixed = self.grad_dtype != self.param_dtype
        self._hooks: list = []
        self.slots: list[Slot] = []
        off = 0
        for p in self.params:
            if not _dense_extent(p):
                raise ValueError("parameter is not a dense tensor (overlapping/strided view)")
            self.slots.append(Slot(off, p.numel()))
            off += _pad(p.numel())
        self.numel = off
        self.flatten_params = flatten_params
        self.master: torch.Tensor | None = None  # fp32 master weights
        self.lowp: torch.Tensor | None = None    # model-dtype copy when params are 16-bit
        if flatten_params:
            self.master = torch.zeros(self.numel, dtype=torch.float32, device=self.device)
            if self.param_dtype != torch.float32:
                self.lowp = torch.zeros(self.numel, dtype=self.param_dtype, device=self.device)
            with torch.no_grad():
                for p, s in zip(self.params, self.slots):
                    self.view(self.master, p, s).copy_(p.detach())
                    target = self.lowp if self.lowp is not None else self.master
                    v = self.view(target, p, s)
                    v.copy_(p.detach())
                    p.data = v
        self.grad = torch.zeros(self.numel, dtype=self.grad_dtype, device=self.device)
        self.attach_grads()

    @staticmethod
    def view(flat: torch.Tensor, p: torch.Tensor, s: Slot) -> torch.Tensor:
        """View of ``flat`` with ``p``'s shape AND strides (keeps channels_last etc.)."""
        return torch.as_strided(flat, p.shape, p.stride(), s.offset)

    def attach_grads(self) -> None:
        """(Re-)point every parameter's gradient into the flat buffer.  ``_voda_gview`` tells
        the fused layers (ops/dense.py) they may accumulate into it in place; when the dtypes
        match it is also ``p.grad`` (autograd accumulates into it in place)."""
        for p, s in zip(self.params, self.slots):
            v = self.view(self.grad, p, s)
            p._voda_gview = v
            p._voda_flat_grad = True
            if self.mixed:
                p.grad = None
            else:
                p.grad = v
        if self.mixed and not self._hooks and any(p.requires_grad for p in self.params):
            for p in self.params:
                if p.requires_grad:
                    self._hooks.append(p.register_post_accumulate_grad_hook(_fold_lowp_grad))

    def zero_grad(self) -> None:
        self.grad.zero_()
        # autograd may have replaced a grad (e.g. user set p.grad = None); re-attach
        for p, s in zip(self.params, self.slots):
            g = p.grad
            if self.mixed:
                if g is not None:
                    p.grad = None
            elif g is None or g.data_ptr() != self.grad.data_ptr() + s.offset * self.grad.element_size():
                p.grad = self.view(self.grad, p, s)

    def remove_hooks(self) -> None:
        for h in self._hooks:
            h.remove()
        self._hooks = []

    def param_storage(self) -> torch.Tensor:
        """The buffer holding the authoritative parameter values (fp32 master)."""
        if self.master is None:
            raise RuntimeError("grad-only FlatGroup has no flat parameter storage")
        return self.master

    def sync_lowp_from_master(self) -> None:
        if self.lowp is not None and self.master is not None:
            self.lowp.copy_(self.master)


# FOLD_CAST = False: fold with a mixed-dtype add (module switch)
FOLD_CAST = True


def _fold_lowp_grad(p: torch.Tensor) -> None:
    """Post-accumulate hook of a low-precision parameter with an fp32 flat gradient: add the
    autograd-produced ``.grad`` into the fp32 slot and drop it.  Registered before the
    data-parallel engine's readiness hook, so a bucket is launched only after the fold."""
    g = p.grad
    if g is None:
        return
    v = p._voda_gview
    if FOLD_CAST and g.dtype != v.dtype:
        # cast first: PyTorch-ROCm's mixed-dtype add (vectorized_templated_elementwise_kernel)
        # took 30-70 us even for a 1000-element bias (ResNet-50 profile, ~0.34 ms per step)
        g = g.to(v.dtype)
    v.add_(g)
    p.grad = None
