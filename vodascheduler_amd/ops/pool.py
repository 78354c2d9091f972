"""Max pooling on channels_last activations with the HIP forward (argmax bytes) and
gather backward (csrc/hip/pool.hip).  Other layouts / dtypes and CPU tensors use
``torch.nn.functional.max_pool2d``."""
from __future__ import annotations

import torch
import torch.nn.functional as F

from . import _native as N


def _out(n: int, k: int, s: int, p: int) -> int:
    return (n + 2 * p - k) // s + 1


def _supported(x: torch.Tensor, k: int) -> bool:
    return (x.is_cuda and x.dim() == 4 and x.dtype in (torch.bfloat16, torch.float32) and x.shape[1] % 8 == 0
            and x.is_contiguous(memory_format=torch.channels_last) and k * k < 256)


class _MaxPoolFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, k, s, p):
        Nb, C, H, W = x.shape
        Ho, Wo = _out(H, k, s, p), _out(W, k, s, p)
        y = torch.empty(Nb, C, Ho, Wo, dtype=x.dtype, device=x.device, memory_format=torch.channels_last)
        idx = torch.empty(Nb * Ho * Wo * C, dtype=torch.uint8, device=x.device)
        N.hip().maxpool2d_fwd(x.data_ptr(), y.data_ptr(), idx.data_ptr(), Nb, H, W, C, Ho, Wo, k, s, p,
                              N.dtype_code(x.dtype), N.stream_of(x))
        ctx.save_for_backward(idx)
        ctx.geom = (Nb, H, W, C, Ho, Wo, k, s, p)
        ctx.dt = x.dtype
        return y

    @staticmethod
    def backward(ctx, dy):
        (idx,) = ctx.saved_tensors
        Nb, H, W, C, Ho, Wo, k, s, p = ctx.geom
        dy = dy.contiguous(memory_format=torch.channels_last).to(ctx.dt)
        dx = torch.empty(Nb, C, H, W, dtype=ctx.dt, device=dy.device, memory_format=torch.channels_last)
        N.hip().maxpool2d_bwd(dy.data_ptr(), idx.data_ptr(), dx.data_ptr(), Nb, H, W, C, Ho, Wo, k, s, p,
                              N.dtype_code(ctx.dt), N.stream_of(dy))
        return dx, None, None, None


def max_pool2d(x: torch.Tensor, kernel_size: int, stride: int | None = None, padding: int = 0) -> torch.Tensor:
    s = kernel_size if stride is None else stride
    if _supported(x, kernel_size) and 2 * padding <= kernel_size:
        return _MaxPoolFn.apply(x, kernel_size, s, padding)
    return F.max_pool2d(x, kernel_size, s, padding)


class FusedMaxPool2d(torch.nn.MaxPool2d):
    """``nn.MaxPool2d`` (square kernel, no dilation / ceil_mode) on the HIP kernels."""

    def forward(self, x):
        k, s, p = self.kernel_size, self.stride, self.padding
        if isinstance(k, int) and isinstance(s, int) and isinstance(p, int) and self.dilation == 1 \
                and not self.ceil_mode and not self.return_indices:
            return max_pool2d(x, k, s, p)
        return super().forward(x)


class _GlobalAvgPoolFn(torch.autograd.Function):
    """mean over H, W of a channels_last [N, C, H, W] tensor -> [N, C, 1, 1]; the backward
    writes the broadcast gradient straight into channels_last (``global_avgpool_bwd``)."""

    @staticmethod
    def forward(ctx, x):
        ctx.shape = x.shape
        ctx.dt = x.dtype
        return x.mean((2, 3), keepdim=True)

    @staticmethod
    def backward(ctx, g):
        Nb, C, H, W = ctx.shape
        g2 = g.reshape(Nb, C)
        if g2.dtype not in (torch.float32, torch.bfloat16) or (g2.dtype == torch.bfloat16 and ctx.dt != g2.dtype):
            g2 = g2.float()
        g2 = g2.contiguous()
        dx = torch.empty(Nb, C, H, W, dtype=ctx.dt, device=g.device, memory_format=torch.channels_last)
        N.hip().global_avgpool_bwd(g2.data_ptr(), dx.data_ptr(), Nb, H * W, C, 1.0 / (H * W),
                                   N.dtype_code(g2.dtype), N.dtype_code(ctx.dt), N.stream_of(g))
        return dx


class GlobalAvgPool2d(torch.nn.AdaptiveAvgPool2d):
    """``nn.AdaptiveAvgPool2d(1)`` (no state) whose training backward on channels_last GPU
    tensors is one HIP kernel."""

    def __init__(self):
        super().__init__(1)

    def forward(self, x):
        if (x.is_cuda and x.dim() == 4 and x.requires_grad and x.dtype in (torch.bfloat16, torch.float32)
                and x.shape[1] % 8 == 0 and x.is_contiguous(memory_format=torch.channels_last)
                and x.data_ptr() % 16 == 0):
            return _GlobalAvgPoolFn.apply(x)
        return super().forward(x)
