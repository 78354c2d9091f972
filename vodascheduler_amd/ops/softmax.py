"""Scaled, masked softmax over attention scores (csrc/hip/softmax.hip).

``masked_softmax(scores, key_mask=None, causal=False, scale=1.0)`` with ``scores`` of shape
[B, H, Tq, S]; ``key_mask`` broadcastable to [B, 1, Tq|1, S] with nonzero = attend.  Masked
logits get the reference's additive -1e9 (reference examples/py/tensorflow2/
advanced_activations_tf25.py:300-318).  Causal masking aligns the last query with the
last key (``key > q + S - Tq`` is masked).
"""
from __future__ import annotations

import torch

from . import _native as N

MAX_S = 2048


def _mask_strides(mask: torch.Tensor, B: int, Tq: int, S: int) -> tuple[torch.Tensor, int, int]:
    """Normalise a keep-mask to a contiguous [B, Tq|1, S] tensor; return (mask, bstride, qstride)."""
    m = mask
    while m.dim() < 4:
        m = m.unsqueeze(0)
    if m.shape[1] != 1:
        raise ValueError("key mask must broadcast over heads (dim 1 == 1)")
    m = m[:, 0]
    if m.shape[-1] != S or m.shape[0] not in (1, B) or m.shape[1] not in (1, Tq):
        raise ValueError(f"key mask shape {tuple(mask.shape)} incompatible with B={B} Tq={Tq} S={S}")
    m = m.contiguous()
    if m.dtype not in (torch.float32, torch.bfloat16, torch.float16):
        m = m.to(torch.float32)
    bstride = 0 if m.shape[0] == 1 else m.shape[1] * S
    qstride = 0 if m.shape[1] == 1 else S
    return m, bstride, qstride


def reference_masked_softmax(scores, key_mask=None, causal=False, scale=1.0):
    """fp32 PyTorch reference."""
    B, H, Tq, S = scores.shape
    x = scores.float() * scale
    keep = torch.ones(B, 1, Tq, S, dtype=torch.bool, device=scores.device)
    if key_mask is not None:
        km = key_mask
        while km.dim() < 4:
            km = km.unsqueeze(0)
        keep = keep & (km != 0)
    if causal:
        q = torch.arange(Tq, device=scores.device).view(Tq, 1)
        k = torch.arange(S, device=scores.device).view(1, S)
        keep = keep & (k <= q + (S - Tq))
    x = torch.where(keep, x, torch.full_like(x, -1e9))
    return torch.softmax(x, dim=-1).to(scores.dtype)


class _MaskedSoftmaxFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, scores, key_mask, causal, scale):
        B, H, Tq, S = scores.shape
        x = scores.contiguous()
        y = torch.empty_like(x)
        mptr, mdt, bs, qs = 0, 0, 0, 0
        if key_mask is not None:
            m, bs, qs = _mask_strides(key_mask, B, Tq, S)
            ctx.mask_keep = m
            mptr, mdt = m.data_ptr(), N.dtype_code(m.dtype)
        N.check_gpu_tensor(x, "scores", align=8)
        N.hip().masked_softmax_fwd(x.data_ptr(), mptr, mdt, y.data_ptr(), B, H, Tq, S, bs, qs, bool(causal),
                                   float(scale), N.dtype_code(x.dtype), N.stream_of(x))
        ctx.save_for_backward(y)
        ctx.scale = scale
        return y

    @staticmethod
    def backward(ctx, dy):
        (y,) = ctx.saved_tensors
        S = y.shape[-1]
        dyc = dy.contiguous()
        dx = torch.empty_like(y)
        N.hip().masked_softmax_bwd(y.data_ptr(), dyc.data_ptr(), dx.data_ptr(), y.numel() // S, S,
                                   float(ctx.scale), N.dtype_code(y.dtype), N.stream_of(y))
        return dx, None, None, None


def masked_softmax(scores: torch.Tensor, key_mask: torch.Tensor | None = None, causal: bool = False,
                   scale: float = 1.0) -> torch.Tensor:
    if scores.dim() != 4:
        raise ValueError("scores must be [B, H, Tq, S]")
    S = scores.shape[-1]
    if scores.is_cuda and S % 4 == 0 and S <= MAX_S and scores.dtype in (torch.float32, torch.bfloat16, torch.float16):
        return _MaskedSoftmaxFn.apply(scores, key_mask, causal, scale)
    if scores.is_cuda:
        # documented generic path for ragged S (e.g. S % 4 != 0): PyTorch ops
        return reference_masked_softmax(scores, key_mask, causal, scale)
    return reference_masked_softmax(scores, key_mask, causal, scale)
