"""Scaled dot-product attention with key-padding + causal masks.

Dispatch (GPU): the fused MFMA flash-attention HIP kernel (csrc/hip/attention.hip) when the
extension provides it for the shape (bf16/fp16, supported head dim, no dropout); otherwise
the materialised path -- scores by hipBLASLt GEMM, the hand-written masked-softmax HIP
kernel, dropout, PV GEMM.  The reference's Transformer materialises the full
[B, H, Tq, S] scores too (layers_tf25.py:450-461).  CPU: the same materialised math with the
fp32 reference softmax.
"""
from __future__ import annotations

import torch

from . import _native as N
from .softmax import masked_softmax


def _flash_supported(q, k, v, key_mask, dropout_p) -> bool:
    if not q.is_cuda or dropout_p > 0.0 or q.dtype not in (torch.bfloat16, torch.float16):
        return False
    try:
        h = N.hip()
    except RuntimeError:
        return False
    if not hasattr(h, "attention_supported"):
        return False
    B, H, Tq, D = q.shape
    return bool(h.attention_supported(D, k.shape[2], N.dtype_code(q.dtype)))


def materialized_attention(q, k, v, key_mask=None, causal=False, scale=1.0, dropout_p=0.0):
    scores = torch.matmul(q, k.transpose(-1, -2))
    km = None
    if key_mask is not None:
        km = key_mask.view(key_mask.shape[0], 1, 1, key_mask.shape[-1]) if key_mask.dim() == 2 else key_mask
    p = masked_softmax(scores, km, causal, scale)
    if dropout_p > 0.0:
        p = torch.nn.functional.dropout(p, dropout_p)
    return torch.matmul(p, v)


def fused_attention(q: torch.Tensor, k: torch.Tensor, v: torch.Tensor, key_mask: torch.Tensor | None = None,
                    causal: bool = False, scale: float | None = None, dropout_p: float = 0.0) -> torch.Tensor:
    """q: [B, H, Tq, D], k/v: [B, H, Tk, D], key_mask: [B, Tk] (nonzero = attend)."""
    if scale is None:
        scale = q.shape[-1] ** -0.5
    if _flash_supported(q, k, v, key_mask, dropout_p):
        from .flash import flash_attention

        return flash_attention(q, k, v, key_mask, causal, scale)
    return materialized_attention(q, k, v, key_mask, causal, scale, dropout_p)
