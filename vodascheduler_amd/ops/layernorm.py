"""LayerNorm with hand-written CDNA4 forward/backward kernels (csrc/hip/layernorm.hip).

``layer_norm(x, weight, bias, eps)`` normalises over the last dimension.  On GPU it runs
the wave-per-row HIP kernels (output in the input dtype, statistics in fp32); on CPU the
PyTorch reference ``torch.nn.functional.layer_norm`` in fp32.
"""
from __future__ import annotations

import os

import torch

from ..utils.flat import flat_grad
from . import _native as N
from .dense import _ready

MAX_N = 4096
LN_DIRECT_GRADS = True


def _direct(p) -> bool:
    """The optimizer's flat gradient owns p's gradient (ops/dense.py contract)."""
    g = flat_grad(p)
    return g is not None and g.is_contiguous()


def _supported(x: torch.Tensor, weight: torch.Tensor | None) -> bool:
    n = x.shape[-1]
    if not x.is_cuda or n % 4 != 0 or n > MAX_N or x.dtype not in (torch.float32, torch.bfloat16, torch.float16):
        return False
    if weight is not None and weight.dtype not in (torch.float32, x.dtype):
        return False
    return True


class _LayerNormFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, weight, bias, eps, residual=None, sink=None, bias_handoff=None):
        """``residual``: normalise ``x + residual`` (the kernel writes the sum, which the backward
        normalises again); ``sink`` (ops/conv1x1.GradSink): hand the residual's gradient to the
        GEMM that consumed the residual stream instead of returning it."""
        n = x.shape[-1]
        xc = x.contiguous()
        if xc.data_ptr() % 16 != 0:
            xc = xc.clone()
        m = xc.numel() // n
        y = torch.empty_like(xc)
        mean = torch.empty(m, dtype=torch.float32, device=x.device)
        rstd = torch.empty(m, dtype=torch.float32, device=x.device)
        wdt = weight.dtype if weight is not None else (torch.float32 if x.dtype == torch.float32 else x.dtype)
        w = weight.contiguous() if weight is not None else None
        b = bias.to(wdt).contiguous() if bias is not None else None
        rc = residual.contiguous() if residual is not None else None
        if rc is not None and rc.data_ptr() % 16 != 0:
            rc = rc.clone()  # the kernel reads the residual with 16-B vector loads
        sm = torch.empty_like(xc) if residual is not None else None
        for t, nm in ((xc, "x"), (y, "y")) + (((rc, "residual"),) if rc is not None else ()):
            N.check_gpu_tensor(t, nm, align=8)
        N.hip().layernorm_fwd(xc.data_ptr(), N.ptr(w), N.ptr(b), y.data_ptr(), mean.data_ptr(), rstd.data_ptr(),
                              m, n, float(eps), N.dtype_code(x.dtype), N.dtype_code(wdt), N.ptr(rc), N.ptr(sm),
                              N.stream_of(x))
        ctx.save_for_backward(sm if sm is not None else xc, w, mean, rstd)
        ctx.has_bias = bias is not None
        ctx.params = (weight, bias)
        ctx.wdt = wdt
        ctx.has_res = residual is not None
        ctx.sink = sink if residual is not None else None
        ctx.bias_handoff = bias_handoff
        return y.view_as(x)

    @staticmethod
    def backward(ctx, dy):
        xc, w, mean, rstd = ctx.saved_tensors
        n = xc.shape[-1]
        m = xc.numel() // n
        dyc = dy.contiguous()
        if dyc.data_ptr() % 16 != 0:
            dyc = dyc.clone()  # offset view: the kernel reads dy with vector loads
        dx = torch.empty_like(xc)
        need_w = w is not None and ctx.needs_input_grad[1]
        need_b = ctx.has_bias and ctx.needs_input_grad[2]
        dgamma = dbeta = ws = None
        weight, bias = ctx.params
        # gamma / beta gradients summed straight into the optimizer's flat buffer (one column-sum
        # launch for both, no autograd add afterwards) when it owns them
        direct = (LN_DIRECT_GRADS and need_w and need_b and _direct(weight) and _direct(bias)
                  and flat_grad(weight).dtype == ctx.wdt and flat_grad(bias).dtype == ctx.wdt)
        # the bias gradient of the Linear that produced x (BiasHandoff): column sums of dx,
        # folded into this pass (needs the direct gamma / beta path and the same dtype)
        hb = ctx.bias_handoff
        tgt = hb.target(ctx.wdt) if (hb is not None and direct and ctx.needs_input_grad[0]) else None
        if tgt is not None and tgt.numel() != n:
            tgt = None
        if need_w or need_b:
            rows = N.hip().layernorm_bwd_partial_rows(m)
            ws = torch.empty((3 if tgt is not None else 2) * rows * n, dtype=torch.float32, device=xc.device)
            if direct:
                dgamma, dbeta = flat_grad(weight), flat_grad(bias)
            else:
                dgamma = torch.empty(n, dtype=ctx.wdt, device=xc.device)
                dbeta = torch.empty(n, dtype=ctx.wdt, device=xc.device)
        N.hip().layernorm_bwd(dyc.data_ptr(), xc.data_ptr(), mean.data_ptr(), rstd.data_ptr(), N.ptr(w),
                              dx.data_ptr(), N.ptr(dgamma), N.ptr(dbeta), N.ptr(ws), m, n,
                              N.dtype_code(xc.dtype), N.dtype_code(ctx.wdt), bool(direct), N.stream_of(xc),
                              N.ptr(tgt))
        if tgt is not None:
            hb.done = True
            _ready(hb.bias)
        dx = dx.view_as(dy)
        dres = None
        if ctx.has_res:
            if ctx.sink is not None and ctx.needs_input_grad[4]:
                ctx.sink.put(dx)  # the consumer accumulates into it after x's branch is done
            elif ctx.needs_input_grad[4]:
                dres = dx
        gw = None if direct or not need_w else dgamma
        gb = None if direct or not need_b else dbeta
        if direct:
            _ready(weight)
            _ready(bias)
        return dx if ctx.needs_input_grad[0] else None, gw, gb, None, dres, None, None


def layer_norm(x: torch.Tensor, weight: torch.Tensor | None = None, bias: torch.Tensor | None = None,
               eps: float = 1e-5, residual: torch.Tensor | None = None, sink=None,
               bias_handoff=None) -> torch.Tensor:
    """LayerNorm over the last dimension; with ``residual``, of ``x + residual`` (one fused pass
    on GPU).  ``sink``: see ops/conv1x1.GradSink (the residual's gradient is handed over);
    ``bias_handoff``: ops/dense.BiasHandoff of the Linear that produced ``x``."""
    if residual is not None and (not x.is_cuda or residual.shape != x.shape or residual.dtype != x.dtype):
        from .dense import residual_add

        x, residual = residual_add(residual, x, sink), None
    if x.is_cuda:
        if not _supported(x, weight):
            raise ValueError(f"fused layer_norm: unsupported shape/dtype {tuple(x.shape)} {x.dtype}")
        if residual is not None:
            return _LayerNormFn.apply(x, weight, bias, eps, residual, sink, bias_handoff)
        return _LayerNormFn.apply(x, weight, bias, eps, None, None, bias_handoff)
    n = x.shape[-1]
    y = torch.nn.functional.layer_norm(x.float(), (n,), None if weight is None else weight.float(),
                                       None if bias is None else bias.float(), eps)
    return y.to(x.dtype)


class FusedLayerNorm(torch.nn.Module):
    """Drop-in for ``torch.nn.LayerNorm`` over the last dimension."""

    def __init__(self, normalized_shape: int, eps: float = 1e-5, elementwise_affine: bool = True,
                 device=None, dtype=None):
        super().__init__()
        if isinstance(normalized_shape, (tuple, list)):
            if len(normalized_shape) != 1:
                raise ValueError("FusedLayerNorm normalises over the last dimension only")
            normalized_shape = normalized_shape[0]
        self.normalized_shape = (int(normalized_shape),)
        self.eps = eps
        if elementwise_affine:
            self.weight = torch.nn.Parameter(torch.ones(normalized_shape, device=device, dtype=dtype))
            self.bias = torch.nn.Parameter(torch.zeros(normalized_shape, device=device, dtype=dtype))
        else:
            self.register_parameter("weight", None)
            self.register_parameter("bias", None)

    def forward(self, x, residual=None, sink=None, bias_handoff=None):
        """``LN(x)``, or ``LN(x + residual)`` with the add fused into the normalisation pass."""
        if x.is_cuda and torch.is_autocast_enabled("cuda"):
            # keep the input dtype (bf16 out, fp32 statistics inside the kernel)
            with torch.autocast("cuda", enabled=False):
                return layer_norm(x, self.weight, self.bias, self.eps, residual, sink, bias_handoff)
        return layer_norm(x, self.weight, self.bias, self.eps, residual, sink, bias_handoff)

    def extra_repr(self):
        return f"{self.normalized_shape}, eps={self.eps}"
