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
from .dense import _direct, _ready

USE_FUSED_EMBEDDING = os.environ.get("VODA_FUSED_EMBEDDING", "1") != "0"


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
