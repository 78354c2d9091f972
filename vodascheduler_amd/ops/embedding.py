"""Embedding lookup whose backward scatters straight into the optimizer's flat gradient.

Stock ``nn.Embedding`` backward (``embedding_dense_backward``) materialises a dense
[vocab, dim] gradient in the weight dtype -- a memset, a sort of the indices and a segment
reduce -- which autograd then adds to the tied MLM decoder's gradient and the trainer folds
into the fp32 flat slot: ~0.3 ms of a BERT-base step on MI355X for a 30522 x 768 table
(profiles/r2_rocprof_bert_final.md: FillFunctor, sum_and_scatter, two vocab-sized adds).
With a flat fp32 gradient (utils/flat.py) the backward here is one ``index_add_`` of the
[tokens, dim] output gradient into that slot (fp32 atomics: the summation order of repeated
tokens is not fixed), then the data-parallel readiness signal, as ops/dense.py does for
Linear weights.  Without a flat gradient it returns the ordinary dense gradient.
"""
from __future__ import annotations

import os

import torch
import torch.nn.functional as F

from ..utils.flat import flat_grad
from .dense import _direct, _ready, colsum_accumulate_

USE_FUSED_EMBEDDING = True


class _EmbeddingFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, ids, weight):
        ctx.save_for_backward(ids)
        ctx.weight = weight
        return F.embedding(ids, weight)

    @staticmethod
    def backward(ctx, dy):
        (ids,) = ctx.saved_tensors
        weight = ctx.weight
        ctx.weight = None
        idx = ids.reshape(-1)
        src = dy.reshape(-1, weight.shape[1])
        if _direct(weight):
            g = flat_grad(weight)
            g.index_add_(0, idx, src.to(g.dtype))
            _ready(weight)
            return None, None
        gw = torch.zeros(weight.shape, dtype=torch.float32, device=weight.device)
        gw.index_add_(0, idx, src.float())
        return None, gw.to(weight.dtype)


class FusedEmbedding(torch.nn.Embedding):
    """Drop-in ``nn.Embedding`` (no padding_idx / max_norm / sparse) using :class:`_EmbeddingFn`."""

    def forward(self, ids):
        if not USE_FUSED_EMBEDDING or self.padding_idx is not None or self.max_norm is not None or self.sparse:
            return super().forward(ids)
        return _EmbeddingFn.apply(ids, self.weight)


class _AddRowsFn(torch.autograd.Function):
    """``x + weight[start:start+count]`` broadcast over x's leading dims (count == 1: one row
    over every token, e.g. BERT's token-type embedding of segment 0; count == T: position
    embeddings over the batch).  The weight gradient -- a column sum of dY -- goes straight
    into the rows' flat gradient slot with the HIP column-sum kernel, instead of autograd's
    broadcast reduction + select / embedding backward + fold into the fp32 slot.  (Those
    PyTorch reductions over 512-8192 rows also lost their result on the second whole-step
    graph replay: profiles/r2_graph_resnet50_investigation.md, BERT / NMT section.)"""

    @staticmethod
    def forward(ctx, x, weight, start, count):
        ctx.weight, ctx.start, ctx.count = weight, start, count
        rows = weight[start] if count == 1 else weight[start:start + count]
        return x + rows

    @staticmethod
    def backward(ctx, dy):
        w, a, c = ctx.weight, ctx.start, ctx.count
        ctx.weight = None
        dy2 = dy.reshape(-1, c * w.shape[1])
        if _direct(w):
            colsum_accumulate_(dy2.contiguous(), flat_grad(w)[a:a + c].reshape(-1))
            _ready(w)
            return dy, None, None, None
        gw = torch.zeros(w.shape, dtype=torch.float32, device=w.device)
        gw[a:a + c] = dy2.float().sum(0).view(c, w.shape[1])
        return dy, gw.to(w.dtype), None, None


def add_rows(x: torch.Tensor, weight: torch.Tensor, start: int = 0, count: int = 1) -> torch.Tensor:
    """``x + weight[start]`` (count 1) or ``x + weight[start:start+count]`` (x [..., count, D]),
    with the flat-gradient backward of :class:`_AddRowsFn`."""
    if not USE_FUSED_EMBEDDING or not torch.is_grad_enabled() or not weight.requires_grad:
        return x + (weight[start] if count == 1 else weight[start:start + count])
    return _AddRowsFn.apply(x, weight, start, count)
