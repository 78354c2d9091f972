"""Convolution bias as its own op: forward ``y + b`` (channel broadcast), backward
``db (+)= sum over (N, H, W) of dy`` on the column-sum HIP kernel (csrc/hip/dense.hip) over
the channels_last ``[N*H*W, C]`` view, accumulated straight into the optimizer's flat
gradient, and ``dy`` passed through for the input.

Why: with ``nn.Conv2d(bias=True)`` the bias gradient comes from MIOpen's backward-bias path,
which is not hipGraph-capture safe in this ROCm build -- a captured step's SECOND replay
already returns wrong conv-bias gradients for VGG16 (``benchmarks/graph_diag.py``,
profiles/r2_graph_diag_vgg16.json: replay 0 exact, replay 1 off by up to 2e5x), i.e. that
path reads a buffer it expects zeroed by work the capture did not record.  The column sum
here has no such state, so VGG16 (the reference's W1 workload) can run as one graph.
"""
from __future__ import annotations

import torch
import torch.nn.functional as F

from ..utils.flat import flat_grad
from .dense import _ready, colsum_accumulate_


class _BiasAddFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, y, bias):
        ctx.has_bias = bias is not None
        ctx.bias = bias
        return y + bias.to(y.dtype).view(1, -1, 1, 1)

    @staticmethod
    def backward(ctx, dy):
        bias = ctx.bias
        db = None
        if ctx.needs_input_grad[1]:
            C = dy.shape[1]
            d2 = dy.permute(0, 2, 3, 1).reshape(-1, C) if dy.is_contiguous(memory_format=torch.channels_last) \
                else dy.transpose(0, 1).reshape(C, -1).t()
            g = flat_grad(bias)
            if g is not None and g.is_contiguous():
                if not d2.is_contiguous():
                    d2 = d2.contiguous()
                colsum_accumulate_(d2, g)
                _ready(bias)
            else:
                db = d2.float().sum(0).to(bias.dtype)
        return dy, db


class Conv2dSepBias(torch.nn.Conv2d):
    """``nn.Conv2d`` (same parameters / state dict) whose bias add and bias gradient run as a
    separate op (``_BiasAddFn``) after a bias-free convolution."""

    def forward(self, x):
        if x.is_cuda and x.dtype != self.weight.dtype and torch.is_autocast_enabled("cuda"):
            x = x.to(self.weight.dtype)
        with torch.autocast(x.device.type, enabled=False):
            y = F.conv2d(x, self.weight, None, self.stride, self.padding, self.dilation, self.groups)
            if self.bias is None:
                return y
            return _BiasAddFn.apply(y, self.bias)
