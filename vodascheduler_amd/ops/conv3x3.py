"""KxK convolutions (ResNet 3x3) whose weight gradient is an implicit-GEMM split-K MFMA
kernel (csrc/hip/wgrad.hip, ``wgrad_conv``) accumulated straight into the optimizer's flat
bf16 gradient.

    forward          MIOpen (F.conv2d, exhaustive find)
    input gradient   MIOpen (aten.convolution_backward, input only)
    weight gradient  dW[co][kh][kw][ci] (+)= sum_{img,ho,wo} dY[img,ho,wo][co] *
                                              X[img, ho*s+kh-p, wo*s+kw-p][ci]

MIOpen runs the weight gradient of these layers as atomic split-K ``igemm_wrw`` kernels plus
a workspace clear and a cast pass; autograd then adds the result into ``.grad`` with another
elementwise kernel.  Here the KH*KW taps are KH*KW "reduction over output pixels" GEMMs of
the same kind as the Linear / 1x1 weight gradients (``ops/wgrad.py``), launched as one grid:
the LDS-DMA loader gathers the input row of each output pixel under the tap (zero rows
outside the image), and the epilogue (or the split-K reduce) writes the tap's Cin columns of
the channels_last weight gradient with beta = 1.  The layer is a drop-in ``nn.Conv2d``;
anything the kernel does not cover (CPU, non-bf16, groups, dilation, a layout that is not
channels_last, channel counts not multiples of 8 or below 128, no flat gradient) runs stock
autograd.
"""
from __future__ import annotations

import math
import os

import torch
import torch.nn.functional as F

from . import _native as N
from . import splitgemm as SG
from . import wgrad as W
from . import winograd as Wg
from ..utils.flat import FOLD_CAST, flat_grad
from .conv1x1 import _direct, _ready

USE_CONV_WGRAD = True
# fp32 weight gradients of the C >= 128 layers (stride 1 and 2) as one implicit GEMM on the
# split-bf16 MFMA kernel (ops/splitgemm.conv_wgrad_) instead of MIOpen's igemm_wrw (A/B switch)
USE_SPLIT_WGRAD_F32 = True
# fp32 forwards the Winograd kernel does not take (ResNet-50's three stride-2 3x3 layers) as one
# implicit GEMM on the split-bf16 MFMA kernel (ops/splitgemm.conv_fwd, input gathered per tap while
# staged) instead of MIOpen's igemm_fwd (A/B switch)
USE_SPLIT_CONV_FWD = True
# fp32 weight gradients of the 64-channel 3x3 layers (ResNet stage 1) on the split GEMM with 64 x 192
# tiles instead of the f32-MFMA c64 kernel.  Off: the step lost 60.94 -> 61.32 ms (same-box A/B,
# profiles/r6/ab_split_wgrad_c64_resnet50_fp32.jsonl); kept tested as the alternative
USE_SPLIT_WGRAD_C64 = False
# ... and their input gradients as four polyphase implicit GEMMs (ops/splitgemm.conv_dgrad_s2)
# instead of MIOpen's igemm_bwd + zero fill.  Off: the parity classes with 1-2 taps reduce over
# only 128-512 k (8-32 stages per tile), and the step lost 58.95 -> 59.12 ms (same-box A/B,
# profiles/r6/ab_split_conv_dgrad_s2_resnet50_fp32.jsonl); kept tested (fp64) as the alternative
USE_SPLIT_CONV_DGRAD = False
# USE_WINOGRAD (module switch): fp32 3x3 stride-1 pad-1 forwards and input gradients (as forward
# convolutions) on the own Winograd F(2x2, 3x3) kernel (ops/winograd.py) instead of MIOpen
USE_WINOGRAD = True
WINO_BN_STATS = True  # the Winograd epilogue also hands the following BN its partial statistics
# DGRAD_FWD (module switch, default on): the input gradient of a stride-1 KxK convolution runs as a
# FORWARD convolution of dy with the transposed, spatially flipped filter
#     dX[n, ci, h, w] = sum_{co, kh, kw} dY[n, co, h - kh + p, w - kw + p] * W[co, ci, kh, kw]
#                     = conv2d(dY, W^T flipped, padding = K - 1 - p)
# so MIOpen runs its forward solvers on it (the bottleneck 3x3 layers have Cin == Cout: the
# very shape the forward pass already found) instead of the backward-data igemm solvers and
# their output zero-fill (VERDICT r2 Next #4).  ResNet-50 bs-256 step, same box back to back:
# 25.87 -> 25.57 ms (profiles/r3/ab_dgrad_fwd.md).
DGRAD_FWD = True


# CONV_F32_FN (module switch, default on): fp32 (reference-precision) stride-1 KxK convolutions take the
# same autograd function, i.e. their input gradient also runs as a forward convolution (their
# weight gradient stays on MIOpen, folded into the flat gradient).  fp32 ResNet-50 step, same
# lease: 70.21 -> 70.08 ms kernel time (igemm_bwd 7.79 -> 1.63 ms, igemm_fwd 8.0 -> 14.0 ms;
# gpurun_out/r4v, profiles/r4/README.md)
CONV_F32_FN = True

# USE_C64_WGRAD = False: the 64 -> 64 channel 3x3 weight gradient runs MIOpen (module switch);
# USE_C64_WGRAD_F32 = False: fp32 activations keep MIOpen's.  The f32-MFMA twin runs 564 us vs
# MIOpen's 579 us at bs 256, 56 x 56 (benchmarks/bench_c64_wgrad.py); in the fp32 ResNet-50 step
# it is even with MIOpen's kernel + zero fill (69.39 vs 69.40 ms, profiles/r4/README.md) and
# writes the flat gradient directly (the bf16 kernel: 126 vs 171 us)
USE_C64_WGRAD = True
USE_C64_WGRAD_F32 = True


def c64_ok(dy: torch.Tensor, x: torch.Tensor, weight: torch.Tensor, stride: int, padding: int) -> bool:
    """The 64-channel 3x3 / stride-1 weight-gradient kernel (csrc/hip/conv3x3_c64.hip) covers
    these operands: channels_last bf16 (or fp32: the f32-MFMA twin) activations, width <= 64."""
    cl = torch.channels_last
    dts = (torch.bfloat16, torch.float32) if USE_C64_WGRAD_F32 else (torch.bfloat16,)
    return (USE_C64_WGRAD and dy.is_cuda and stride == 1 and padding == 1 and tuple(weight.shape) == (64, 64, 3, 3)
            and x.dtype in dts and dy.dtype == x.dtype and x.dim() == 4
            and x.shape == dy.shape and x.shape[3] <= 64 and x.is_contiguous(memory_format=cl)
            and dy.is_contiguous(memory_format=cl) and x.data_ptr() % 16 == 0 and dy.data_ptr() % 16 == 0)


def conv_c64_wgrad(dy: torch.Tensor, x: torch.Tensor, weight: torch.Tensor) -> torch.Tensor | None:
    """dW of a 64 -> 64 3x3 / stride-1 convolution: added in fp32 into the optimizer's flat
    gradient when it owns one (returns None), else returned in the weight's dtype."""
    n, _, hh, ww = x.shape
    h = N.hip()
    ws = torch.empty(h.conv3x3_c64_wgrad_workspace_floats(n, hh), dtype=torch.float32, device=x.device)
    gw = flat_grad(weight) if _direct(weight) else None
    if gw is not None and gw.dtype in (torch.float32, torch.bfloat16):
        h.conv3x3_c64_wgrad(x.data_ptr(), dy.data_ptr(), gw.data_ptr(), *gw.stride(), ws.data_ptr(), n, hh, ww, True,
                            N.dtype_code(gw.dtype), N.stream_of(x), N.dtype_code(x.dtype))
        _ready(weight)
        return None
    dw = torch.empty(weight.shape, dtype=torch.float32, device=x.device)
    h.conv3x3_c64_wgrad(x.data_ptr(), dy.data_ptr(), dw.data_ptr(), *dw.stride(), ws.data_ptr(), n, hh, ww, False,
                        N.dtype_code(dw.dtype), N.stream_of(x), N.dtype_code(x.dtype))
    return dw.to(weight.dtype)


def dgrad_as_forward(dy: torch.Tensor, weight: torch.Tensor, padding: int) -> torch.Tensor:
    """Input gradient of a stride-1 KxK convolution as the forward convolution of ``dy`` with
    the flipped, channel-transposed filter (channels_last in, channels_last out)."""
    k = weight.shape[-1]
    return F.conv2d(dy, flipped_filter(weight, dy.dtype), None, 1, k - 1 - padding)


def flipped_filter(weight: torch.Tensor, dtype: torch.dtype | None = None) -> torch.Tensor:
    """``weight.transpose(0, 1).flip(2, 3)`` as a channels_last tensor of ``dtype`` (default the
    weight's): on GPU one HIP launch (csrc/hip/conv3x3_c64.hip filter_flip_t) instead of a flip,
    a layout copy and, under autocast, a cast."""
    dtype = dtype or weight.dtype
    co, ci, kh, kw = weight.shape
    ok = (weight.is_cuda and kh == kw and weight.dtype in (torch.float32, torch.bfloat16)
          and dtype in (torch.float32, torch.bfloat16))
    if not ok:
        return weight.transpose(0, 1).flip(2, 3).contiguous(memory_format=torch.channels_last).to(dtype)
    out = torch.empty((ci, co, kh, kw), dtype=dtype, device=weight.device, memory_format=torch.channels_last)
    s0, s1, s2, s3 = weight.stride()
    N.hip().filter_flip_t(weight.data_ptr(), N.dtype_code(weight.dtype), s0, s1, s2, s3, out.data_ptr(),
                          N.dtype_code(dtype), co, ci, kh, N.stream_of(weight))
    return out


def dgrad_fwd_ok(weight: torch.Tensor, stride: int, padding: int) -> bool:
    kh, kw = weight.shape[-2:]
    return DGRAD_FWD and stride == 1 and kh == kw and 0 <= padding <= kh - 1


def default_splits(M: int, Cout: int, Cin: int, taps: int, target_blocks: int = 432) -> int:
    tiles = math.ceil(Cout / W.TILE) * math.ceil(Cin / W.TILE) * taps
    s = math.ceil(target_blocks / tiles)
    return max(1, min(s, 256, M // 256 if M >= 256 else 1))


def conv_wgrad_ref(dy: torch.Tensor, x: torch.Tensor, weight_shape, stride: int, padding: int) -> torch.Tensor:
    """fp32 reference of the weight gradient [Cout, Cin, KH, KW]."""
    return torch.nn.grad.conv2d_weight(x.float(), weight_shape, dy.float(), stride=stride, padding=padding)


def conv_wgrad_accumulate_(dy: torch.Tensor, x: torch.Tensor, gw: torch.Tensor, stride: int, padding: int,
                           accumulate: bool = True, splits: int | None = None) -> None:
    """``gw (+)= dW`` in place; dy [N, Cout, Ho, Wo], x [N, Cin, H, W] channels_last bf16, gw
    [Cout, Cin, KH, KW] channels_last bf16 or fp32 (memory [Cout][KH][KW][Cin])."""
    if not dy.is_cuda:
        w = conv_wgrad_ref(dy, x, gw.shape, stride, padding)
        gw.copy_((w + gw.float() if accumulate else w).to(gw.dtype))
        return
    if not supported(dy, x, gw):
        raise ValueError(f"conv_wgrad: unsupported operands dy {tuple(dy.shape)} {dy.dtype}, x {tuple(x.shape)} "
                         f"{x.dtype}, dw {tuple(gw.shape)} {gw.dtype}")
    n, cin, H, Wd = x.shape
    cout, _, kh, kw = gw.shape
    ho, wo = dy.shape[2], dy.shape[3]
    M = n * ho * wo
    s = splits if splits is not None else default_splits(M, cout, cin, kh * kw)
    h = N.hip()
    nws = h.wgrad_conv_workspace_floats(M, cout, cin, kh * kw, s)
    ws = torch.empty(nws, dtype=torch.float32, device=dy.device) if nws else None
    h.wgrad_conv(dy.data_ptr(), x.data_ptr(), gw.data_ptr(), n, H, Wd, cin, ho, wo, cout, kh, kw, int(stride),
                 int(padding), s, N.ptr(ws), bool(accumulate), W._zero_rows(dy.device).data_ptr(),
                 N.dtype_code(gw.dtype), N.stream_of(dy))


def supported(dy: torch.Tensor, x: torch.Tensor, gw: torch.Tensor) -> bool:
    cl = torch.channels_last
    if not (dy.is_cuda and x.is_cuda and gw.is_cuda):
        return False
    if dy.dtype != torch.bfloat16 or x.dtype != torch.bfloat16 or gw.dtype not in (torch.bfloat16, torch.float32):
        return False
    if dy.dim() != 4 or x.dim() != 4 or gw.dim() != 4:
        return False
    if not (dy.is_contiguous(memory_format=cl) and x.is_contiguous(memory_format=cl)
            and gw.is_contiguous(memory_format=cl)):
        return False
    n, cin, _, _ = x.shape
    cout = gw.shape[0]
    if gw.shape[1] != cin or dy.shape[0] != n or dy.shape[1] != cout or cin % 8 or cout % 8:
        return False
    return dy.data_ptr() % 16 == 0 and x.data_ptr() % 16 == 0 and gw.data_ptr() % 16 == 0


class _ConvKxKFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, weight, stride: int, padding: int, kernel_wgrad: bool = True, holder=None):
        """``holder`` (ops/conv1x1.StatsHolder): the Winograd epilogue's BN partial statistics
        of y for the BN that follows (attached to the output by ConvKxK.forward)."""
        if USE_WINOGRAD and Wg.supported(x, weight, stride, padding):
            y = Wg.conv3x3_wino(x, weight, holder=holder)
        elif USE_SPLIT_CONV_FWD and SG.conv_fwd_ok(x, weight):
            y = SG.conv_fwd(x, weight, stride, padding)  # fp32 stride-2: implicit GEMM, split-bf16 MFMA
        else:
            y = F.conv2d(x, weight, None, stride, padding)
        ctx.save_for_backward(x, weight)
        ctx.conf = (stride, padding, kernel_wgrad)
        return y

    @staticmethod
    def backward(ctx, dy):
        x, weight = ctx.saved_tensors
        stride, padding, kernel_wgrad = ctx.conf
        if not dy.is_contiguous(memory_format=torch.channels_last):
            dy = dy.contiguous(memory_format=torch.channels_last)
        dx = None
        if ctx.needs_input_grad[0] and USE_WINOGRAD and Wg.supported(dy, weight, stride, padding, flip=True):
            dx = Wg.conv3x3_wino(dy, weight, flip=True)
        elif (ctx.needs_input_grad[0] and USE_SPLIT_CONV_DGRAD and stride == 2 and padding == 1
              and SG.conv_dgrad_s2_ok(dy, weight, x.shape)):
            dx = SG.conv_dgrad_s2(dy, weight, x.shape)  # fp32: four polyphase implicit GEMMs
        elif ctx.needs_input_grad[0] and dgrad_fwd_ok(weight, stride, padding):
            dx = dgrad_as_forward(dy, weight, padding)
        elif ctx.needs_input_grad[0]:
            dx = torch.ops.aten.convolution_backward(dy, x, weight, None, [stride, stride], [padding, padding],
                                                     [1, 1], False, [0, 0], 1, [True, False, False])[0]
        dw = None
        gw64 = flat_grad(weight) if (ctx.needs_input_grad[1] and USE_SPLIT_WGRAD_C64 and x.dtype == torch.float32
                                     and weight.shape[0] == 64 and _direct(weight)) else None
        if gw64 is not None and SG.conv_wgrad_ok(dy, x, gw64):
            # fp32 64-channel layers: the implicit GEMM on the split-bf16 MFMA, 64 x 192 tiles
            SG.conv_wgrad_(dy, x, gw64, stride, padding)
            _ready(weight)
            dw = None
        elif ctx.needs_input_grad[1] and not kernel_wgrad and c64_ok(dy, x, weight, stride, padding):
            dw = conv_c64_wgrad(dy, x, weight)
        elif ctx.needs_input_grad[1]:
            gw = flat_grad(weight) if _direct(weight) else None
            if gw is not None and kernel_wgrad and supported(dy, x, gw):
                conv_wgrad_accumulate_(dy, x, gw, stride, padding)
                _ready(weight)
            elif gw is not None and kernel_wgrad and USE_SPLIT_WGRAD_F32 and SG.conv_wgrad_ok(dy, x, gw):
                SG.conv_wgrad_(dy, x, gw, stride, padding)  # fp32: implicit GEMM on the split-bf16 MFMA
                _ready(weight)
            else:
                dw = torch.ops.aten.convolution_backward(dy, x, weight, None, [stride, stride], [padding, padding],
                                                         [1, 1], False, [0, 0], 1, [False, True, False])[1]
                if gw is not None:  # flat gradient the kernel cannot take: fold it here
                    gw.add_(dw.to(gw.dtype) if FOLD_CAST else dw)  # see utils/flat.FOLD_CAST
                    _ready(weight)
                    dw = None
        return dx, dw, None, None, None, None


class ConvKxK(torch.nn.Conv2d):
    """``nn.Conv2d(cin, cout, k, stride, padding, bias=False)`` whose weight gradient runs on the
    implicit-GEMM MFMA kernel when the optimizer owns a flat bf16 gradient for it."""

    def __init__(self, in_channels: int, out_channels: int, kernel_size: int = 3, stride: int = 1,
                 padding: int = 1, **kw):
        super().__init__(in_channels, out_channels, kernel_size, stride=stride, padding=padding, bias=False, **kw)

    def _layout_ok(self, x: torch.Tensor) -> bool:
        dt = (torch.bfloat16, torch.float32) if CONV_F32_FN else (torch.bfloat16,)
        return (x.is_cuda and x.dim() == 4 and x.dtype in dt
                and self.weight.dtype == x.dtype and self.groups == 1 and self.dilation == (1, 1)
                and self.stride[0] == self.stride[1] and self.padding[0] == self.padding[1]
                and isinstance(self.padding[0], int) and x.is_contiguous(memory_format=torch.channels_last)
                and self.weight.is_contiguous(memory_format=torch.channels_last)
                and self.in_channels % 8 == 0 and self.out_channels % 8 == 0)

    def _fast_ok(self, x: torch.Tensor) -> bool:
        # 64-channel layers fill a quarter of the 128 x 128 MFMA tile: ResNet-50's layer1 3x3
        # weight gradient took 360 us here vs 150 us (+35 us of workspace passes) on MIOpen;
        # from 128 channels on this kernel is the faster one (profiles/r1_conv3x3_wgrad.md)
        return (USE_CONV_WGRAD and self._layout_ok(x)
                and self.in_channels >= 128 and self.out_channels >= 128)

    def _holder(self, x: torch.Tensor):
        """A statistics side channel when the Winograd forward runs for a training-mode layer
        (its output feeds a BN, ResNet's bn2)."""
        if (USE_WINOGRAD and WINO_BN_STATS and self.training and torch.is_grad_enabled()
                and Wg.supported(x, self.weight, self.stride[0], self.padding[0])):
            from .conv1x1 import StatsHolder

            return StatsHolder()
        return None

    def forward(self, x):
        if x.is_cuda and x.dtype != self.weight.dtype and torch.is_autocast_enabled("cuda"):
            x = x.to(self.weight.dtype)
        if self._fast_ok(x):
            holder = self._holder(x)
            with torch.autocast("cuda", enabled=False):
                y = _ConvKxKFn.apply(x, self.weight, self.stride[0], self.padding[0], True, holder)
            return self._attach(y, holder)
        c64 = (USE_C64_WGRAD and self.in_channels == 64 and self.out_channels == 64 and self.kernel_size == (3, 3)
               and self.stride[0] == 1 and self.padding[0] == 1)
        if self._layout_ok(x) and (c64 or dgrad_fwd_ok(self.weight, self.stride[0], self.padding[0])):
            # input gradient as a forward convolution (DGRAD_FWD); weight gradient on the
            # 64-channel kernel (conv3x3_c64.hip) or MIOpen
            holder = self._holder(x)
            with torch.autocast("cuda", enabled=False):
                y = _ConvKxKFn.apply(x, self.weight, self.stride[0], self.padding[0], False, holder)
            return self._attach(y, holder)
        return super().forward(x)

    @staticmethod
    def _attach(y: torch.Tensor, holder) -> torch.Tensor:
        if holder is not None and holder.stats is not None:
            from .batchnorm import attach_stats

            attach_stats(y, *holder.stats)
        return y
