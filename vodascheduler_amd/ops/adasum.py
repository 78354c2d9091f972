"""Adasum reduction (csrc/hip/adasum.hip) with its fp32 PyTorch reference.

Horovod's ``op=hvd.Adasum`` (reference examples/py/pytorch/pytorch_mnist_elastic.py:32,
102,108-109,188): gradients of N workers are combined pairwise along a
binary tree, per parameter tensor, by

    adasum(a, b) = (1 - a.b / (2|a|^2)) a + (1 - a.b / (2|b|^2)) b

which is the plain sum for orthogonal gradients and the average for identical ones, so the
learning rate is NOT scaled by the world size (Horovod's examples use ``lr_scaler = 1``).

Data-plane design (see ``parallel/ddp.py``): a bucket is all-gathered once over RCCL
(``[N, n]``, 288 GB HBM makes the N copies free), then every rank runs the same
deterministic tree of segmented combine kernels on it -- no atomics, bit-identical results
on every rank, so replicas never drift.
"""
from __future__ import annotations

from typing import Sequence

import torch

from . import _native as N

CHUNK = 16384  # elements per workgroup slice (64 KB fp32): >=256 workgroups for a 4M-element bucket


class AdasumPlan:
    """Device block table for one bucket: ``segments`` are ``(start, end)`` element ranges
    (one per parameter) tiling ``[0, numel)``."""

    def __init__(self, segments: Sequence[tuple[int, int]], device: torch.device, chunk: int = CHUNK):
        segs = [(int(s), int(e)) for s, e in segments if e > s]
        if not segs:
            raise ValueError("AdasumPlan needs at least one non-empty segment")
        pos = 0
        for s, e in segs:
            if s != pos:
                raise ValueError(f"segments must tile the buffer contiguously (gap/overlap at {s}, expected {pos})")
            pos = e
        self.numel = pos
        self.segments = segs
        blk_seg, blk_lo, blk_hi, seg_first, seg_nblk = [], [], [], [], []
        for si, (s, e) in enumerate(segs):
            seg_first.append(len(blk_seg))
            n = 0
            for lo in range(s, e, chunk):
                blk_seg.append(si)
                blk_lo.append(lo)
                blk_hi.append(min(lo + chunk, e))
                n += 1
            seg_nblk.append(n)
        self.nblk, self.nseg = len(blk_seg), len(segs)
        meta = torch.tensor(blk_seg + blk_lo + blk_hi + seg_first + seg_nblk, dtype=torch.int64)
        self.device = device
        self.meta = meta.to(device) if device.type == "cuda" else meta
        self.partials = torch.empty(3 * self.nblk, dtype=torch.float32, device=device)


def adasum_pair_ref(a: torch.Tensor, b: torch.Tensor, segments: Sequence[tuple[int, int]]) -> torch.Tensor:
    """fp32 reference of one segmented pairwise combine (returns a new fp32 tensor)."""
    a32, b32 = a.float(), b.float()
    out = torch.empty_like(a32)
    for s, e in segments:
        x, y = a32[s:e], b32[s:e]
        dot = torch.dot(x, y)
        aa, bb = torch.dot(x, x), torch.dot(y, y)
        ca = 1.0 - 0.5 * dot / aa if aa >= 1e-30 else torch.tensor(1.0)
        cb = 1.0 - 0.5 * dot / bb if bb >= 1e-30 else torch.tensor(1.0)
        out[s:e] = ca * x + cb * y
    return out


def adasum_pair_(a: torch.Tensor, b: torch.Tensor, out: torch.Tensor, plan: AdasumPlan) -> torch.Tensor:
    """``out = adasum(a, b)`` per segment; ``out`` may alias ``a``."""
    for t in (a, b, out):
        if t.numel() != plan.numel or t.dtype != a.dtype:
            raise ValueError("adasum_pair_: operands must match the plan size and share one dtype")
    if not a.is_cuda:
        out.copy_(adasum_pair_ref(a, b, plan.segments).to(out.dtype))
        return out
    align = 4 * a.element_size()
    for name, t in (("a", a), ("b", b), ("out", out)):
        N.check_gpu_tensor(t, name, align=align)
    N.hip().adasum_combine(a.data_ptr(), b.data_ptr(), out.data_ptr(), N.dtype_code(a.dtype), plan.meta.data_ptr(),
                           plan.nblk, plan.nseg, plan.partials.data_ptr(), N.stream_of(a))
    return out


def adasum_tree_(stack: torch.Tensor, plan: AdasumPlan) -> torch.Tensor:
    """Reduce the rows of ``stack`` ([N, n], e.g. an all-gathered bucket) with Adasum along
    a binary tree (rows 2k and 2k+1, then 4k and 4k+2, ...) -- Horovod's recursive-doubling
    pairing; a non-power-of-two remainder carries up unchanged.  Returns ``stack[0]``."""
    n = stack.shape[0]
    stride = 1
    while stride < n:
        for i in range(0, n - stride, 2 * stride):
            adasum_pair_(stack[i], stack[i + stride], stack[i], plan)
        stride *= 2
    return stack[0]


def adasum_tree_ref(rows: Sequence[torch.Tensor], segments: Sequence[tuple[int, int]]) -> torch.Tensor:
    """fp32 reference of :func:`adasum_tree_` (same pairing order)."""
    vals = [r.float().clone() for r in rows]
    stride = 1
    while stride < len(vals):
        for i in range(0, len(vals) - stride, 2 * stride):
            vals[i] = adasum_pair_ref(vals[i], vals[i + stride], segments)
        stride *= 2
    return vals[0]
