"""Scaled dot-product attention with key-padding + causal masks.

Dispatch (GPU): the fused MFMA attention HIP kernels (csrc/hip/attention.hip, ops/flash.py)
when the shape is supported (bf16, head dim 32/64/128/256, Tq, Tk <= 4096, no dropout);
otherwise the materialised path -- scores by hipBLASLt GEMM, the hand-written
masked-softmax HIP kernel, dropout, PV GEMM.  The reference's Transformer materialises
the full [B, H, Tq, S] scores (layers_tf25.py:450-461).  CPU: the same materialised math
with the fp32 reference softmax.

Layouts: ``attention_qkvpacked`` takes the fused projection [B, T, 3, H, D] and
``attention_q_kvpacked`` q [B, Tq, H, D] + kv [B, Tk, 2, H, D]; both return
[B, Tq, H, D] (= the [B, Tq, H*D] input of the output projection, no copy).
"""
from __future__ import annotations

import torch

from . import flash
from .softmax import masked_softmax


def _flash_ok(q: torch.Tensor, Tk: int, dropout_p: float) -> bool:
    return dropout_p == 0.0 and q.is_cuda and flash.supported(q.shape[-1], q.shape[1], Tk, q.dtype)


def materialized_attention(q, k, v, key_mask=None, causal=False, scale=1.0, dropout_p=0.0):
    """q/k/v [B, H, T, D] -> [B, H, Tq, D]."""
    scores = torch.matmul(q, k.transpose(-1, -2))
    km = None
    if key_mask is not None:
        km = key_mask.view(key_mask.shape[0], 1, 1, key_mask.shape[-1]) if key_mask.dim() == 2 else key_mask
    p = masked_softmax(scores, km, causal, scale)
    if dropout_p > 0.0:
        p = torch.nn.functional.dropout(p, dropout_p)
    return torch.matmul(p, v)


def attention_qkvpacked(qkv: torch.Tensor, key_mask=None, causal: bool = False, scale: float | None = None,
                        dropout_p: float = 0.0) -> torch.Tensor:
    """qkv [B, T, 3, H, D] -> [B, T, H, D]."""
    D = qkv.shape[-1]
    scale = D ** -0.5 if scale is None else scale
    if _flash_ok(qkv[:, :, 0], qkv.shape[1], dropout_p):
        return flash.attention_qkvpacked(qkv, key_mask, causal, scale)
    q, k, v = (qkv[:, :, i].transpose(1, 2) for i in range(3))
    return materialized_attention(q, k, v, key_mask, causal, scale, dropout_p).transpose(1, 2)


def attention_q_kvpacked(q: torch.Tensor, kv: torch.Tensor, key_mask=None, causal: bool = False,
                         scale: float | None = None, dropout_p: float = 0.0) -> torch.Tensor:
    """q [B, Tq, H, D], kv [B, Tk, 2, H, D] -> [B, Tq, H, D]."""
    D = q.shape[-1]
    scale = D ** -0.5 if scale is None else scale
    if _flash_ok(q, kv.shape[1], dropout_p):
        return flash.attention_q_kvpacked(q, kv, key_mask, causal, scale)
    k, v = kv[:, :, 0].transpose(1, 2), kv[:, :, 1].transpose(1, 2)
    return materialized_attention(q.transpose(1, 2), k, v, key_mask, causal, scale, dropout_p).transpose(1, 2)


def fused_attention(q: torch.Tensor, k: torch.Tensor, v: torch.Tensor, key_mask: torch.Tensor | None = None,
                    causal: bool = False, scale: float | None = None, dropout_p: float = 0.0) -> torch.Tensor:
    """q: [B, H, Tq, D], k/v: [B, H, Tk, D], key_mask: [B, Tk] (nonzero = attend) -> [B, H, Tq, D]."""
    if scale is None:
        scale = q.shape[-1] ** -0.5
    if dropout_p == 0.0 and q.is_cuda and flash.supported(q.shape[-1], q.shape[2], k.shape[2], q.dtype):
        return flash.flash_attention(q, k, v, key_mask, causal, scale)
    return materialized_attention(q, k, v, key_mask, causal, scale, dropout_p)
