"""fp32 3x3 stride-1 pad-1 convolution as Winograd F(2x2, 3x3) on the f32 MFMA
(csrc/hip/winograd_f32.hip): 2.25x fewer multiply-adds than the direct / implicit-GEMM
convolution, transforms fused into the kernel (nothing transformed goes to HBM).

``conv3x3_wino(x, w)`` takes NHWC (channels_last) fp32 activations and any-layout fp32 filters;
the filter transform U = G g G^T runs per call (the weights change every step).

``USE_SX`` (round 6): the 16 tile GEMMs on the bf16 matrix cores at fp32 accuracy -- U and each
V fragment split exactly into hi / mid / lo bf16 parts, six cross products per 16 channels
(v_mfma_f32_32x32x16_bf16, the split of ops/splitgemm.py) -- instead of the f32 MFMA: 267-379 vs
337-450 us per ResNet-50 3x3 layer at batch 256, with a lower error vs fp64
(profiles/r6/winograd_sx_vs_f32.jsonl); ResNet-50 fp32 step 62.34 -> 60.43 ms (same-box A/B,
profiles/r6/ab_winograd_sx_resnet50_fp32.jsonl).
"""
from __future__ import annotations

import torch
import torch.nn.functional as F

from . import _native as N

USE_SX = True
# SX2 (round 6): the split kernel at 64 output channels per 8-wave workgroup (one V split feeds 12
# MFMAs instead of 6; half the patch loads / transforms per output), where Cout % 64 == 0 and
# Cin <= WIDE_MAX_C: per ResNet-50 layer 335 vs 377 us at C = 64, 305 vs 310 at 128, but 294 vs 281
# at 256 and 340 vs 322 at 512, where the per-workgroup U stream (64 output channels x all input
# channels x 16 positions x 3 planes, re-read by every 32-tile block) and not the split's VALU sets
# the pace (profiles/r6/winograd_sx2_layers.jsonl).  ResNet-50 fp32 step 60.90 -> 60.74 ms (same-box
# A/B, profiles/r6/ab_winograd_wide_resnet50_fp32.jsonl).
USE_WIDE = True
WIDE_MAX_C = 64  # 128 until the one-position form below: 272 (one-position) vs 295 us (wide) at C = 128
# the 32-channel split kernel one Winograd position at a time (no scratch spills; the position-
# pair form spills 116 bytes per lane at 256 VGPRs): per ResNet-50 layer 354 vs 378 us (C = 64),
# 272 vs 301 (128), 255 vs 272 (256), 306 vs 315 (512) (profiles/r6/winograd_onepos_layers.jsonl);
# ResNet-50 fp32 step 58.59 -> 58.54 ms with WIDE_MAX_C = 128 (ab_winograd_onepos_resnet50_fp32.jsonl)
ONEPOS = True
_applied = {"onepos": None}


def supported(x: torch.Tensor, w: torch.Tensor, stride: int = 1, padding: int = 1, flip: bool = False) -> bool:
    """fp32 NHWC x, fp32 3x3 filter, stride 1, pad 1, channels multiples of 32.  ``flip``: x is a
    layer's output gradient and w that layer's filter (the input gradient as a forward conv)."""
    cin, cout = (int(w.shape[0]), int(w.shape[1])) if flip else (int(w.shape[1]), int(w.shape[0]))
    return (x.is_cuda and x.dtype == torch.float32 and w.dtype == torch.float32 and x.dim() == 4
            and tuple(w.shape[2:]) == (3, 3) and stride == 1 and padding == 1 and x.shape[1] == cin
            and x.is_contiguous(memory_format=torch.channels_last) and x.data_ptr() % 16 == 0
            and N.hip().wino_f23_supported(cin, cout))


def filter_transform(w: torch.Tensor, flip: bool = False, sx: bool | None = None) -> torch.Tensor:
    """U = G g G^T per (co, ci), stored [16][Cin / 8][Cout][8] fp32, or (``sx``) as three exact bf16
    planes [16][3][Cin / 8][Cout][8]; ``flip``: of the 180-degree-rotated, channel-transposed filter
    (Cout and Cin of the result are w's Cin and Cout)."""
    sx = USE_SX if sx is None else sx
    co, ci = (int(w.shape[1]), int(w.shape[0])) if flip else (int(w.shape[0]), int(w.shape[1]))
    u = (torch.empty(16, 3, co, ci, dtype=torch.bfloat16, device=w.device) if sx
         else torch.empty(16, co, ci, dtype=torch.float32, device=w.device))
    s0, s1, s2, s3 = w.stride()
    N.hip().wino_f23_filter(w.data_ptr(), s0, s1, s2, s3, u.data_ptr(), co, ci, bool(flip), bool(sx),
                            N.stream_of(w))
    return u


def conv3x3_wino(x: torch.Tensor, w: torch.Tensor, u: torch.Tensor | None = None, flip: bool = False,
                 holder=None) -> torch.Tensor:
    """y = conv2d(x, w, padding=1) for NHWC fp32 x; ``flip``: dX = conv2d(dY, w^T rotated 180,
    padding=1), the input gradient of a 3x3 stride-1 pad-1 layer.  CPU / unsupported: F.conv2d.
    ``holder`` (ops/conv1x1.StatsHolder): receives y's BN partial statistics from the epilogue."""
    if not supported(x, w, flip=flip):
        wf = w.transpose(0, 1).flip(2, 3) if flip else w
        return F.conv2d(x, wf, None, 1, 1)
    n, c, h, wd = x.shape
    co = int(w.shape[1]) if flip else int(w.shape[0])
    if u is None:
        u = filter_transform(w, flip)
    sx = u.dtype == torch.bfloat16
    hip = N.hip()
    wide = sx and USE_WIDE and c <= WIDE_MAX_C and hip.wino_f23_sx2_supported(c, co)
    G = hip.wino_f23_groups2(n, h, wd, c, co) if wide else hip.wino_f23_groups(n, h, wd, c, co)
    ws = None
    if holder is not None:
        ws = torch.empty(max(2 * G * co + 3 * co, hip.bn_workspace_floats(n * h * wd, co)), dtype=torch.float32,
                         device=x.device)
        holder.stats = (ws, G)
    y = torch.empty((n, co, h, wd), dtype=torch.float32, device=x.device, memory_format=torch.channels_last)
    if _applied["onepos"] != ONEPOS:
        hip.wino_f23_set_onepos(int(bool(ONEPOS)))
        _applied["onepos"] = ONEPOS
    if wide:
        hip.wino_f23_fwd2(x.data_ptr(), u.data_ptr(), y.data_ptr(), N.ptr(ws), n, h, wd, c, co, G, N.stream_of(x))
    else:
        hip.wino_f23_fwd(x.data_ptr(), u.data_ptr(), y.data_ptr(), N.ptr(ws), n, h, wd, c, co, G, sx,
                         N.stream_of(x))
    return y
