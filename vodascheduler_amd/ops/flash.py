"""Fused MFMA attention (csrc/hip/attention.hip): forward, dQ pass and dK/dV pass.

Entry points (bf16 on v_mfma_f32_32x32x16_bf16, or fp32 -- the reference's precision -- on
v_mfma_f32_32x32x2_f32, csrc/hip/attention_f32.hip; head dim 32/64/128/256, Tq, Tk <= 4096;
the streamed operand goes through LDS in 32-row tiles, so long sequences -- BERT at 512 --
stay on the fused path):

* ``attention_qkvpacked(qkv)`` -- self-attention straight from the packed projection
  ``qkv`` [B, T, 3, H, D] (one fused QKV GEMM); the gradient is written into ONE
  [B, T, 3, H, D] buffer, so no split / transpose / concat copies exist in either direction.
* ``attention_q_kvpacked(q, kv)`` -- cross-attention: q [B, Tq, H, D], kv [B, Tk, 2, H, D].
* ``flash_attention(q, k, v)`` -- generic [B, H, T, D] tensors (used by ``fused_attention``).

Outputs are [B, Tq, H, D] contiguous, i.e. already the [B, Tq, H*D] input of the output
projection.  Masks: ``key_mask`` [B, Tk] (nonzero = attend; masked scores get the
reference's additive -1e9) and ``causal``.
"""
from __future__ import annotations

import torch

from . import _native as N

import os

MAX_T = 4096
# head dims the flash kernels cover (larger ones take the materialised path)
HEAD_DIMS = tuple(d for d in (32, 64, 128, 256) if d <= 256)


DTYPES = {torch.bfloat16: "DT_BF16", torch.float32: "DT_F32"}


def supported(D: int, Tq: int, Tk: int, dtype: torch.dtype, device_is_cuda: bool = True) -> bool:
    if not device_is_cuda or dtype not in DTYPES or D not in HEAD_DIMS or Tq > MAX_T or Tk > MAX_T:
        return False
    try:
        h = N.hip()
    except RuntimeError:
        return False
    return bool(h.attention_supported(D, Tq, Tk, getattr(N, DTYPES[dtype])))


def _d(t: torch.Tensor | None, b: int, h: int, r: int) -> list[int]:
    """(ptr, batch stride, head stride, row stride) of a tensor addressed as [b][h][row][D]."""
    if t is None:
        return [0, 0, 0, 0]
    return [t.data_ptr(), t.stride(b), t.stride(h), t.stride(r)]


def _mask_args(key_mask: torch.Tensor | None, B: int, Tk: int) -> tuple[int, int, torch.Tensor | None]:
    if key_mask is None:
        return 0, 0, None
    m = key_mask
    if m.dim() != 2 or m.shape[0] != B or m.shape[1] != Tk:
        raise ValueError(f"key_mask must be [B, Tk] = [{B}, {Tk}], got {tuple(m.shape)}")
    if m.dtype not in (torch.bool, torch.uint8):
        m = m != 0
    if m.stride(1) != 1:
        m = m.contiguous()
    return m.data_ptr(), m.stride(0), m


def _slices5(x5: torch.Tensor, n: int) -> list[torch.Tensor]:
    """[B, T, n, H, D] -> n views addressed as (B, T, H, D) (dims b=0, row=1, head=2)."""
    return [x5[:, :, i] for i in range(n)]


def _launch(fwd: bool, q, k, v, o, dout, out, dk, dv, lse, delta, mptr, msb, B, H, Tq, Tk, D, scale, causal,
            stream):
    # every [b, t, h, d] view: dims (0, 2, 1) -> batch, head, row
    t = (_d(q, 0, 2, 1) + _d(k, 0, 2, 1) + _d(v, 0, 2, 1) + _d(o, 0, 2, 1) + _d(dout, 0, 2, 1)
         + _d(out, 0, 2, 1) + _d(dk, 0, 2, 1) + _d(dv, 0, 2, 1)
         + [N.ptr(lse), N.ptr(delta), mptr, msb])
    h = N.hip()
    if q.dtype == torch.float32:
        fn = h.attention_fwd_f32 if fwd else h.attention_bwd_f32
    else:
        fn = h.attention_fwd if fwd else h.attention_bwd
    fn(t, B, H, Tq, Tk, D, float(scale), bool(causal), stream)


def _check(*ts):
    dt = ts[0].dtype
    for x in ts:
        if x.stride(-1) != 1 or x.data_ptr() % 16 != 0 or not x.is_cuda or x.dtype != dt:
            raise ValueError("attention operands must be 16-byte aligned CUDA tensors of one dtype with a "
                             "contiguous last dim")
        if dt == torch.float32 and any(st % 4 for st in x.stride()[:-1]):
            raise ValueError("fp32 attention operands need row strides that are multiples of 4 elements")


class _AttnFn(torch.autograd.Function):
    """q_src: [B, Tq, H, D] or packed [B, T, 3, H, D] (kv_src None); kv_src: [B, Tk, 2, H, D]."""

    @staticmethod
    def forward(ctx, q_src, kv_src, key_mask, causal, scale):
        if kv_src is None:
            q, k, v = _slices5(q_src, 3)
        else:
            q = q_src
            k, v = _slices5(kv_src, 2)
        B, Tq, H, D = q.shape
        Tk = k.shape[1]
        _check(q, k, v)
        mptr, msb, m = _mask_args(key_mask, B, Tk)
        o = torch.empty(B, Tq, H, D, dtype=q.dtype, device=q.device)
        lse = torch.empty(B * H * Tq, dtype=torch.float32, device=q.device)
        _launch(True, q, k, v, None, None, o, None, None, lse, None, mptr, msb, B, H, Tq, Tk, D, scale, causal,
                N.stream_of(q))
        ctx.save_for_backward(q_src, kv_src if kv_src is not None else q_src, o, lse, m if m is not None else o)
        ctx.packed = kv_src is None
        ctx.has_mask = m is not None
        ctx.causal, ctx.scale = causal, scale
        return o

    @staticmethod
    def backward(ctx, dout):
        q_src, kv_src, o, lse, m = ctx.saved_tensors
        if ctx.packed:
            q, k, v = _slices5(q_src, 3)
            dsrc = torch.empty_like(q_src)
            dq, dk, dv = _slices5(dsrc, 3)
            dkv = None
        else:
            q = q_src
            k, v = _slices5(kv_src, 2)
            dq = torch.empty_like(q_src)
            dkv = torch.empty_like(kv_src)
            dk, dv = _slices5(dkv, 2)
        if dout.dtype != q.dtype:
            dout = dout.to(q.dtype)
        if (dout.stride(-1) != 1 or dout.data_ptr() % 16 != 0
                or (dout.dtype == torch.float32 and any(st % 4 for st in dout.stride()[:-1]))):
            dout = dout.contiguous()
        B, Tq, H, D = q.shape
        Tk = k.shape[1]
        mptr, msb = (m.data_ptr(), m.stride(0)) if ctx.has_mask else (0, 0)
        delta = torch.empty(B * H * Tq, dtype=torch.float32, device=q.device)
        _launch(False, q, k, v, o, dout, dq, dk, dv, lse, delta, mptr, msb, B, H, Tq, Tk, D, ctx.scale, ctx.causal,
                N.stream_of(q))
        if ctx.packed:
            return dsrc, None, None, None, None
        return dq, dkv, None, None, None


def attention_qkvpacked(qkv: torch.Tensor, key_mask=None, causal: bool = False, scale: float | None = None):
    """qkv [B, T, 3, H, D] -> out [B, T, H, D]."""
    D = qkv.shape[-1]
    return _AttnFn.apply(qkv, None, key_mask, causal, D ** -0.5 if scale is None else scale)


def attention_q_kvpacked(q: torch.Tensor, kv: torch.Tensor, key_mask=None, causal: bool = False,
                         scale: float | None = None):
    """q [B, Tq, H, D], kv [B, Tk, 2, H, D] -> out [B, Tq, H, D]."""
    D = q.shape[-1]
    return _AttnFn.apply(q, kv, key_mask, causal, D ** -0.5 if scale is None else scale)


def flash_attention(q, k, v, key_mask=None, causal=False, scale=None):
    """Generic entry: q/k/v [B, H, T, D] -> [B, H, Tq, D] (a transposed view of [B, Tq, H, D])."""
    q4 = q.transpose(1, 2).contiguous()
    kv5 = torch.stack([k.transpose(1, 2), v.transpose(1, 2)], dim=2)
    return attention_q_kvpacked(q4, kv5, key_mask, causal, scale).transpose(1, 2)
