"""tanh-approximated GELU on the HIP kernels of ``csrc/hip/activation.hip``.

The reference's Transformer / BERT FFN activation (reference
examples/py/tensorflow2/transformer.py: ``Dense(dff, activation=...)``; BERT uses GELU).
On GPU both passes are one vectorised kernel each; the backward saves only the
pre-activation.  CPU falls back to ``torch.nn.functional.gelu(approximate="tanh")``.
"""
from __future__ import annotations

import torch

from . import _native as N


class _GeluTanhFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, h):
        hc = h.contiguous()
        y = torch.empty_like(hc)
        N.check_gpu_tensor(hc, "h", align=16)
        N.hip().gelu_tanh_fwd(hc.data_ptr(), y.data_ptr(), hc.numel(), N.dtype_code(hc.dtype), N.stream_of(hc))
        ctx.save_for_backward(hc)
        return y.view_as(h)

    @staticmethod
    def backward(ctx, dy):
        (h,) = ctx.saved_tensors
        dyc = dy.contiguous()
        if dyc.data_ptr() % 16 != 0:
            dyc = dyc.clone()  # 16-B vector loads
        dh = torch.empty_like(h)
        N.check_gpu_tensor(dyc, "dy", align=16)
        N.hip().gelu_tanh_bwd(h.data_ptr(), dyc.data_ptr(), dh.data_ptr(), h.numel(), N.dtype_code(h.dtype),
                              N.stream_of(h))
        return dh.view_as(dy)


def gelu_tanh(h: torch.Tensor) -> torch.Tensor:
    """GELU with the tanh approximation (``F.gelu(h, approximate="tanh")``)."""
    if h.is_cuda and h.dtype in (torch.float32, torch.bfloat16, torch.float16):
        if h.is_contiguous() and h.data_ptr() % 16 != 0:
            h = h.clone()  # offset view: the kernel's 16-B vector loads need an aligned base
        return _GeluTanhFn.apply(h)
    return torch.nn.functional.gelu(h, approximate="tanh")


class GeluTanh(torch.nn.Module):
    def forward(self, h):
        return gelu_tanh(h)
