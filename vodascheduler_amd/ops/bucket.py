"""Bucket pack / scale / cast ops (csrc/hip/bucket.hip) with CPU references."""
from __future__ import annotations

from typing import Sequence

import torch

from . import _native as N


def cast_scale_(src: torch.Tensor, dst: torch.Tensor, scale: float = 1.0) -> torch.Tensor:
    """``dst[:] = (src * scale).to(dst.dtype)`` over flat contiguous buffers."""
    if src.numel() != dst.numel():
        raise ValueError(f"size mismatch {src.numel()} vs {dst.numel()}")
    if src.device != dst.device:
        raise ValueError("src/dst on different devices")
    if not src.is_cuda:
        dst.copy_(src.float().mul(scale).view(dst.shape) if scale != 1.0 else src.view(dst.shape))
        return dst
    N.check_gpu_tensor(src, "src", align=8)
    N.check_gpu_tensor(dst, "dst", align=8)
    N.hip().cast_scale(src.data_ptr(), N.dtype_code(src.dtype), dst.data_ptr(), N.dtype_code(dst.dtype),
                       src.numel(), float(scale), N.stream_of(src))
    return dst


def multi_tensor_copy_(srcs: Sequence[torch.Tensor], dsts: Sequence[torch.Tensor], scale: float = 1.0) -> None:
    """Copy (and scale / cast) a list of tensors in one launch per 64 tensors.

    All sources must share one dtype and all destinations one dtype; each pair must have
    the same number of elements and both sides must be dense contiguous.
    """
    if len(srcs) != len(dsts):
        raise ValueError("length mismatch")
    if not srcs:
        return
    sdt, ddt = srcs[0].dtype, dsts[0].dtype
    for s, d in zip(srcs, dsts):
        if s.dtype != sdt or d.dtype != ddt:
            raise ValueError("multi_tensor_copy_: mixed dtypes")
        if s.numel() != d.numel():
            raise ValueError("multi_tensor_copy_: numel mismatch")
    if not srcs[0].is_cuda:
        with torch.no_grad():
            for s, d in zip(srcs, dsts):
                d.view(-1).copy_(s.reshape(-1).float().mul(scale) if scale != 1.0 else s.reshape(-1))
        return
    for s, d in zip(srcs, dsts):
        N.check_gpu_tensor(s, "src", align=2)
        N.check_gpu_tensor(d, "dst", align=2)
    N.hip().multi_tensor_copy([s.data_ptr() for s in srcs], [d.data_ptr() for d in dsts],
                              [s.numel() for s in srcs], N.dtype_code(sdt), N.dtype_code(ddt), float(scale),
                              N.stream_of(srcs[0]))
