"""ResNet ImageNet stem -- conv 7x7/2 (3 -> 64) + BN + ReLU + max pool 3x3/2 -- as one
training op (csrc/hip/stem.hip + the fused BN/pool kernels of csrc/hip/batchnorm.hip).

Forward: the image is packed once to NHWC-4 bf16 (``stem_pack``, also the fp32 -> bf16
cast autocast would run), the convolution is a persistent MFMA implicit GEMM whose epilogue
writes the per-workgroup BN sums / sums of squares, and the BN finalize + ReLU + max pool
kernel takes those partials instead of re-reading the 411 MB (bs 256) conv output.
Backward: the fused BN/pool backward, then the weight gradient as an MFMA GEMM over the
output pixels (``stem_conv_wgrad``: transposed LDS reads of the dY rows and of overlapping
im2col rows of the packed image, fp32 straight into the optimizer's flat gradient).

The module keeps the ``nn.Sequential(conv, bn_pool)`` state dict (``stem.0.weight``,
``stem.1.*``) of the reference ResNet-50 (examples/py/tensorflow2/
tensorflow2_keras_cifar_elastic.py builds Keras ResNet50; torchvision layout here).  Anything
the kernels do not cover -- evaluation, CPU, other geometry, output width > 128 -- runs the
composition.  The reference-precision (fp32) run takes ``_StemF32Fn``: the fp32 MFMA
convolution of csrc/hip/stem_f32.hip with the statistics epilogue, the same fused BN/pool
kernels, and MIOpen's weight gradient.
"""
from __future__ import annotations

import os

import torch
import torch.nn as nn

from ..utils.flat import FOLD_CAST, flat_grad
from . import _native as N
from .batchnorm import FusedBNReLUMaxPool2d, bn_pool_backward, bn_pool_forward
from .conv1x1 import _direct, _ready

USE_STEM = os.environ.get("VODA_STEM", "1") != "0"
# USE_STEM_WGRAD = False: the weight gradient runs MIOpen's igemm_wrw on the packed image (module switch)
USE_STEM_WGRAD = True
COUT = 64


def _out(n: int) -> int:
    return (n + 2 * 3 - 7) // 2 + 1


def pack_nhwc4(x: torch.Tensor) -> torch.Tensor:
    """[N, C<=4, H, W] (any strides, fp32/bf16/fp16) -> [N, H, W, 4] bf16, zero channels
    from C on."""
    n, c, hh, ww = x.shape
    x4 = torch.empty(n, hh, ww, 4, dtype=torch.bfloat16, device=x.device)
    N.hip().stem_pack(x.data_ptr(), x4.data_ptr(), n, c, hh, ww, *x.stride(), N.dtype_code(x.dtype), N.stream_of(x))
    return x4


def stem_conv_stats(x4: torch.Tensor, weight: torch.Tensor, cin: int, ws: torch.Tensor | None = None):
    """conv7x7/2 of the packed image with the BN partial sums: returns (y [N,64,Ho,Wo]
    channels_last bf16, workspace, partial-row count)."""
    n, hh, ww, _ = x4.shape
    ho, wo = _out(hh), _out(ww)
    h = N.hip()
    nb = h.stem_partial_rows(n, ho)
    y = torch.empty(n, COUT, ho, wo, dtype=torch.bfloat16, device=x4.device, memory_format=torch.channels_last)
    need = max(2 * nb * COUT + 3 * COUT, h.bn_pool_workspace_floats(n, ho, COUT))
    if ws is None or ws.numel() < need:
        ws = torch.empty(need, dtype=torch.float32, device=x4.device)
    h.stem_conv_fwd(x4.data_ptr(), weight.data_ptr(), *weight.stride(), cin, COUT, y.data_ptr(), ws.data_ptr(), nb,
                    n, hh, ww, ho, wo, N.stream_of(x4))
    return y, ws, nb


def stem_wgrad(x4: torch.Tensor, dyc: torch.Tensor, weight: torch.Tensor, cin: int) -> torch.Tensor | None:
    """Filter gradient of the stem conv: accumulated in fp32 into the optimizer's flat
    gradient when it owns one (returns None), else returned in the weight's dtype."""
    n, hh, ww, _ = x4.shape
    ho, wo = dyc.shape[2], dyc.shape[3]
    h = N.hip()
    ws = torch.empty(h.stem_wgrad_workspace_floats(n, ho), dtype=torch.float32, device=x4.device)
    gw = flat_grad(weight) if _direct(weight) else None
    if gw is not None and gw.dtype in (torch.float32, torch.bfloat16):
        h.stem_conv_wgrad(x4.data_ptr(), dyc.data_ptr(), gw.data_ptr(), *gw.stride(), cin, ws.data_ptr(), n, hh, ww,
                          ho, wo, True, N.dtype_code(gw.dtype), N.stream_of(x4))
        _ready(weight)
        return None
    dw = torch.empty(weight.shape, dtype=torch.float32, device=weight.device)
    h.stem_conv_wgrad(x4.data_ptr(), dyc.data_ptr(), dw.data_ptr(), *dw.stride(), cin, ws.data_ptr(), n, hh, ww, ho,
                      wo, False, N.dtype_code(dw.dtype), N.stream_of(x4))
    return dw.to(weight.dtype)


class _StemFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, weight, gamma, beta, running_mean, running_var, momentum, eps):
        cin = x.shape[1]
        x4 = pack_nhwc4(x)
        yc, ws, nb = stem_conv_stats(x4, weight, cin)
        y, idx, save_mean, save_invstd = bn_pool_forward(yc, gamma, beta, running_mean, running_var, momentum, eps,
                                                         3, 2, 1, ws=ws, pre_nb=nb)
        ctx.cin = cin
        ctx.x_dtype = x.dtype
        ctx.bias = beta
        ctx.save_for_backward(x4, weight, yc, idx, gamma, save_mean, save_invstd)
        return y

    @staticmethod
    def backward(ctx, dy):
        x4, weight, yc, idx, gamma, save_mean, save_invstd = ctx.saved_tensors
        need_g = gamma is not None and ctx.needs_input_grad[2]
        dyc, dgamma, dbeta, _ = bn_pool_backward(dy, yc, idx, gamma, ctx.bias, save_mean, save_invstd, 3, 2, 1,
                                                 need_g, ctx.needs_input_grad[3])
        cin = ctx.cin
        dx = dw = None
        if ctx.needs_input_grad[1] and USE_STEM_WGRAD:
            dw = stem_wgrad(x4, dyc, weight, cin)
        mask = [bool(ctx.needs_input_grad[0]), bool(ctx.needs_input_grad[1]) and not USE_STEM_WGRAD, False]
        if mask[0] or mask[1]:
            x4v = x4.permute(0, 3, 1, 2)  # [N, 4, H, W], channels_last
            w4 = weight.new_empty((COUT, 4, 7, 7)).contiguous(memory_format=torch.channels_last)
            dx4, dw4, _ = torch.ops.aten.convolution_backward(dyc, x4v, w4, None, [2, 2], [3, 3], [1, 1], False,
                                                              [0, 0], 1, mask)
            if mask[0]:
                dx = dx4[:, :cin].to(ctx.x_dtype)
            if mask[1]:
                dw = dw4[:, :cin]
                gw = flat_grad(weight) if _direct(weight) else None
                if gw is not None:  # fold into the optimizer's flat gradient (see utils/flat.FOLD_CAST)
                    gw.add_(dw.to(gw.dtype) if FOLD_CAST else dw)
                    _ready(weight)
                    dw = None
        return dx, dw, dgamma, dbeta, None, None, None, None


def stem_conv_stats_f32(x: torch.Tensor, weight: torch.Tensor, ws: torch.Tensor | None = None):
    """fp32 conv7x7/2 of the image (read through its strides) with the BN partial sums
    (csrc/hip/stem_f32.hip): returns (y [N,64,Ho,Wo] channels_last fp32, workspace, partial-row
    count)."""
    n, cin, hh, ww = x.shape
    ho, wo = _out(hh), _out(ww)
    h = N.hip()
    nb = h.stem_partial_rows(n, ho)
    y = torch.empty(n, COUT, ho, wo, dtype=torch.float32, device=x.device, memory_format=torch.channels_last)
    need = max(2 * nb * COUT + 3 * COUT, h.bn_pool_workspace_floats(n, ho, COUT))
    if ws is None or ws.numel() < need:
        ws = torch.empty(need, dtype=torch.float32, device=x.device)
    h.stem_conv_fwd_f32(x.data_ptr(), *x.stride(), cin, weight.data_ptr(), *weight.stride(), y.data_ptr(),
                        ws.data_ptr(), nb, n, hh, ww, ho, wo, N.stream_of(x))
    return y, ws, nb


def stem_wgrad_f32(x: torch.Tensor, dyc: torch.Tensor, weight: torch.Tensor) -> torch.Tensor | None:
    """fp32 filter gradient of the stem conv on the own MFMA kernel (csrc/hip/stem_f32.hip):
    accumulated into the optimizer's flat gradient when it owns one (returns None), else
    returned."""
    n, cin, hh, ww = x.shape
    ho, wo = dyc.shape[2], dyc.shape[3]
    h = N.hip()
    ws = torch.empty(h.stem_wgrad_f32_workspace_floats(n, ho), dtype=torch.float32, device=x.device)
    gw = flat_grad(weight) if _direct(weight) else None
    direct = gw is not None and gw.dtype == torch.float32
    out = gw if direct else torch.empty(weight.shape, dtype=torch.float32, device=weight.device)
    h.stem_conv_wgrad_f32(x.data_ptr(), *x.stride(), cin, dyc.data_ptr(), out.data_ptr(), *out.stride(),
                          ws.data_ptr(), n, hh, ww, ho, wo, direct, N.stream_of(x))
    if direct:
        _ready(weight)
        return None
    return out


class _StemF32Fn(torch.autograd.Function):
    """The reference-precision stem: own fp32 MFMA convolution with the BN statistics in its
    epilogue (no zero-fill, no statistics pass), the fused BN + ReLU + max pool, and the own
    fp32 MFMA weight gradient (MIOpen's for output widths > 112)."""

    @staticmethod
    def forward(ctx, x, weight, gamma, beta, running_mean, running_var, momentum, eps):
        yc, ws, nb = stem_conv_stats_f32(x, weight)
        y, idx, save_mean, save_invstd = bn_pool_forward(yc, gamma, beta, running_mean, running_var, momentum, eps,
                                                         3, 2, 1, ws=ws, pre_nb=nb)
        ctx.bias = beta
        ctx.save_for_backward(x, weight, yc, idx, gamma, save_mean, save_invstd)
        return y

    @staticmethod
    def backward(ctx, dy):
        x, weight, yc, idx, gamma, save_mean, save_invstd = ctx.saved_tensors
        need_g = gamma is not None and ctx.needs_input_grad[2]
        dyc, dgamma, dbeta, _ = bn_pool_backward(dy, yc, idx, gamma, ctx.bias, save_mean, save_invstd, 3, 2, 1,
                                                 need_g, ctx.needs_input_grad[3])
        mask = [bool(ctx.needs_input_grad[0]), bool(ctx.needs_input_grad[1]), False]
        dx = dw = None
        if (mask[1] and USE_STEM_WGRAD and dyc.is_contiguous(memory_format=torch.channels_last)
                and N.hip().stem_wgrad_f32_supported(dyc.shape[3])):
            dw = stem_wgrad_f32(x, dyc, weight)
            mask[1] = False
        if mask[0] or mask[1]:
            dx, dw, _ = torch.ops.aten.convolution_backward(dyc, x, weight, None, [2, 2], [3, 3], [1, 1], False,
                                                            [0, 0], 1, mask)
            gw = flat_grad(weight) if (mask[1] and _direct(weight)) else None
            if gw is not None:  # fold into the optimizer's flat gradient
                gw.add_(dw.to(gw.dtype))
                _ready(weight)
                dw = None
        return dx, dw, dgamma, dbeta, None, None, None, None


class FusedStem(nn.Sequential):
    """``nn.Sequential(Conv2d(cin, 64, 7, 2, 3, bias=False), FusedBNReLUMaxPool2d(64))``
    whose training forward runs :class:`_StemFn`."""

    def __init__(self, in_channels: int = 3, out_channels: int = COUT):
        super().__init__(nn.Conv2d(in_channels, out_channels, 7, stride=2, padding=3, bias=False),
                         FusedBNReLUMaxPool2d(out_channels, 3, stride=2, padding=1))

    def _fast_ok(self, x: torch.Tensor) -> bool:
        conv, bn = self[0], self[1]
        return (USE_STEM and self.training and x.is_cuda and x.dim() == 4 and 1 <= x.shape[1] <= 4
                and x.dtype in (torch.float32, torch.bfloat16, torch.float16)
                and conv.weight.dtype == torch.bfloat16 and conv.out_channels == COUT and conv.groups == 1
                and conv.kernel_size == (7, 7) and conv.stride == (2, 2) and conv.padding == (3, 3)
                and conv.dilation == (1, 1) and conv.bias is None and 1 <= _out(x.shape[3]) <= 128
                and bn.pool == (3, 2, 1) and bn.track_running_stats and bn.momentum is not None
                and all(t is None or t.dtype == torch.float32
                        for t in (bn.weight, bn.bias, bn.running_mean, bn.running_var))
                and (x.dtype == torch.bfloat16 or torch.is_autocast_enabled("cuda")))

    def _fast_f32_ok(self, x: torch.Tensor) -> bool:
        """The reference-precision path (fp32 image and weights, no autocast)."""
        conv, bn = self[0], self[1]
        return (USE_STEM and self.training and x.is_cuda and x.dim() == 4 and 1 <= x.shape[1] <= 3
                and x.dtype == torch.float32 and conv.weight.dtype == torch.float32
                and not torch.is_autocast_enabled("cuda") and x.data_ptr() % 4 == 0
                and conv.out_channels == COUT and conv.groups == 1 and conv.kernel_size == (7, 7)
                and conv.stride == (2, 2) and conv.padding == (3, 3) and conv.dilation == (1, 1)
                and conv.bias is None and 1 <= _out(x.shape[3]) <= 128 and min(x.stride()) >= 0
                and bn.pool == (3, 2, 1) and bn.track_running_stats and bn.momentum is not None
                and all(t is None or t.dtype == torch.float32
                        for t in (bn.weight, bn.bias, bn.running_mean, bn.running_var)))

    def forward(self, x):
        if self._fast_f32_ok(x):
            bn = self[1]
            bn._pending_batches = getattr(bn, "_pending_batches", 0) + 1
            return _StemF32Fn.apply(x, self[0].weight, bn.weight, bn.bias, bn.running_mean, bn.running_var,
                                    bn.momentum, bn.eps)
        if not self._fast_ok(x):
            return super().forward(x)
        bn = self[1]
        bn._pending_batches = getattr(bn, "_pending_batches", 0) + 1
        with torch.autocast("cuda", enabled=False):
            return _StemFn.apply(x, self[0].weight, bn.weight, bn.bias, bn.running_mean, bn.running_var, bn.momentum,
                                 bn.eps)
