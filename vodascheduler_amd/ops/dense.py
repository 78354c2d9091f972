"""Linear layer whose backward writes its weight / bias gradients straight into the fused
optimizer's flat gradient buffer (csrc/hip/dense.hip for the bias column sums).

Stock autograd computes ``dW = dY^T X`` and ``db = dY.sum(0)`` into fresh tensors and then
ADDS them into ``p.grad`` (two extra elementwise kernels + a latency-bound reduction per
Linear per step; ~1.3 ms of a 15 ms BERT-base step on MI355X, profiles/).  Here, when the
parameter's ``.grad`` is a view of a :class:`~vodascheduler_amd.utils.flat.FlatGroup`
buffer (marked ``_voda_flat_grad``), the backward accumulates in place -- ``grad.addmm_``
(one GEMM with beta = 1) and the HIP column-sum kernel -- and then signals the
data-parallel engine's readiness hook (``_voda_grad_ready``) itself, exactly as autograd's
post-accumulate hook would.  Otherwise it returns ordinary gradients.

On GPU the in-place weight gradient (and the bias gradient with it) is the split-K MFMA
kernel of ``ops/wgrad.py`` (csrc/hip/wgrad.hip): the "reduction over tokens" GEMMs are
too narrow for hipBLASLt to fill 256 CUs.  ``USE_WGRAD_KERNEL = False`` (or
``USE_WGRAD_KERNEL = False``) switches back to ``addmm_`` + the column-sum kernel.
"""
from __future__ import annotations

import os

import torch
import torch.nn.functional as F

from ..utils.flat import flat_grad
from . import _native as N
from . import splitgemm as SG
from . import wgrad as W

USE_WGRAD_KERNEL = True
USE_SPLIT_DGRAD = True
_BMM_F32: bool | None = None  # torch.bmm(..., out_dtype=float32) available (probed once)


def _split_count(M: int, n_out: int, K: int) -> int:
    """Splits of the reduction (output-feature) dimension for dX = dY . W, or 1.

    A vocab-sized head's input gradient (BERT MLM: [1280 x 30528] . [30528 x 768]) has a long
    reduction and only ~60 output tiles of 128 x 128, so hipBLASLt runs it on a quarter of the
    CUs (233 us, profiles/r2_rocprof_bert_final.md).  Splitting the reduction into S batched
    GEMMs (fp32 partials, summed after) fills the chip; chunks stay multiples of 8 columns."""
    tiles = -(-M // 128) * -(-K // 128)
    if n_out < 8192 or tiles >= 128:
        return 1
    target = max(2, min(16, 256 // max(tiles, 1)))
    for s in range(target, 1, -1):
        if n_out % (8 * s) == 0:
            return s
    return 1


def _dgrad(dy2: torch.Tensor, weight: torch.Tensor) -> torch.Tensor:
    """dY [M, n_out] . W [n_out, K] -> [M, K] in dY's dtype (split-K for long reductions).
    fp32 operands run on the split-bf16 MFMA kernel (ops/splitgemm.py) when it takes them."""
    global _BMM_F32
    if SG.supported(dy2, weight):
        return SG.matmul(dy2, weight)
    M, n_out = dy2.shape
    K = weight.shape[1]
    S = _split_count(M, n_out, K) if (USE_SPLIT_DGRAD and dy2.is_cuda and weight.is_contiguous()) else 1
    if S == 1:
        return dy2 @ weight
    c = n_out // S
    a = dy2.view(M, S, c).transpose(0, 1)   # [S, M, c], row stride n_out
    b = weight.view(S, c, K)
    if _BMM_F32 is not False:
        try:
            part = torch.bmm(a, b, out_dtype=torch.float32)
            _BMM_F32 = True
        except (RuntimeError, TypeError):
            _BMM_F32 = False
    if _BMM_F32 is False:
        part = torch.bmm(a, b).float()
    return part.sum(0).to(dy2.dtype)


def _direct(p: torch.Tensor | None) -> bool:
    g = flat_grad(p)
    return g is not None and g.is_contiguous()


def _ready(p: torch.Tensor) -> None:
    fn = getattr(p, "_voda_grad_ready", None)
    if fn is not None:
        fn(p)


def colsum_accumulate_(dy2: torch.Tensor, out: torch.Tensor) -> None:
    """out += dy2.sum(0) for dy2 [M, N] (GPU: HIP kernel; CPU: torch)."""
    if not dy2.is_cuda:
        out.add_(dy2.sum(0).to(out.dtype))
        return
    M, Nc = dy2.shape
    if Nc % 8 != 0 or dy2.stride(1) != 1 or dy2.stride(0) != Nc or dy2.data_ptr() % 16 != 0:
        out.add_(dy2.float().sum(0).to(out.dtype))
        return
    h = N.hip()
    ws = torch.empty(h.colsum_workspace_floats(M, Nc), dtype=torch.float32, device=dy2.device)
    h.colsum_accumulate(dy2.data_ptr(), M, Nc, N.dtype_code(dy2.dtype), out.data_ptr(), N.dtype_code(out.dtype), True,
                        ws.data_ptr(), N.stream_of(dy2))


def linear_weight_grads(dy2: torch.Tensor, x2: torch.Tensor, weight: torch.Tensor, bias: torch.Tensor | None,
                        need_w: bool, need_b: bool):
    """Weight / bias gradients of ``y = x W^T + b`` from dY [M, n_out] and X [M, K].  When the
    optimizer owns flat gradients for them they are accumulated in place (split-K MFMA kernel
    with the fused bias gradient, ops/wgrad.py) and the DDP engine is signalled; returns the
    (dw, db) autograd must still deliver (None for the in-place ones)."""
    dw = db = None
    fused = (USE_WGRAD_KERNEL and need_w and _direct(weight) and (not need_b or _direct(bias))
             and W.supported(dy2, x2, flat_grad(weight), flat_grad(bias) if need_b else None))
    if fused:
        W.wgrad_accumulate_(dy2, x2, flat_grad(weight), flat_grad(bias) if need_b else None)
        _ready(weight)
        if need_b:
            _ready(bias)
        return None, None
    if need_w:
        if _direct(weight):
            gw = flat_grad(weight)
            if gw.dtype == torch.float32 and SG.supported(dy2.t(), x2):
                # fp32: split-bf16 MFMA, beta = 1; the bias gradient (column sums of dY) from the same
                # launch's A staging when the layout allows
                gb = flat_grad(bias) if need_b and _direct(bias) else None
                tile, _, variant = SG.plan(dy2.t(), x2)
                if gb is not None and SG.row_sums_ok(dy2.t(), gb, tile, variant):
                    SG.matmul(dy2.t(), x2, out=gw, accumulate=True, row_sums=gb)
                    _ready(weight)
                    _ready(bias)
                    return None, None
                SG.matmul(dy2.t(), x2, out=gw, accumulate=True)
            elif gw.dtype == dy2.dtype:
                gw.addmm_(dy2.t(), x2)
            else:  # fp32 flat gradient of a bf16 weight (cast first: see utils/flat.FOLD_CAST)
                gw.add_((dy2.t() @ x2).to(gw.dtype))
            _ready(weight)
        else:
            dw = dy2.t() @ x2
    if need_b:
        if _direct(bias):
            colsum_accumulate_(dy2, flat_grad(bias))
            _ready(bias)
        else:
            db = dy2.float().sum(0).to(bias.dtype)
    return dw, db


class BiasHandoff:
    """The bias gradient of a Linear computed by the NEXT op's backward, which reads the
    Linear's output gradient anyway: the FFN's GELU backward for fc1 (``gelu_tanh_bwd_colsum``)
    and a post-LN sublayer's LayerNorm backward for its last projection (``layernorm_bwd`` with
    ``dbias_in``).  That op sums the gradient's columns into the bias's flat fp32 gradient,
    signals it ready and sets ``done``; the Linear's backward then skips its column-sum pass.
    Only valid when nothing between the two ops changes the gradient (no dropout), which the
    model wiring guarantees (models/layers.py)."""

    __slots__ = ("bias", "done")

    def __init__(self, bias):
        self.bias, self.done = bias, False

    def target(self, dtype: torch.dtype):
        """The flat gradient to accumulate into, or None (no flat gradient of that dtype)."""
        if self.bias is None or not _direct(self.bias):
            return None
        g = flat_grad(self.bias)
        return g if g.dtype == dtype else None


class _DenseFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, weight, bias, sink_in=None, bias_handoff=None):
        """``sink_in`` (ops/conv1x1.GradSink): accumulate the input gradient into the
        residual-stream gradient a producer left there (one GEMM with beta = 1);
        ``bias_handoff`` (BiasHandoff): the bias gradient may arrive from the next op."""
        if x.dtype != weight.dtype and torch.is_autocast_enabled(x.device.type):
            x = x.to(weight.dtype)
        with torch.autocast(x.device.type, enabled=False):
            x2 = x.reshape(-1, x.shape[-1])
            if x.dim() >= 1 and SG.supported(x2, weight.t()):  # fp32: split-bf16 MFMA kernel
                y = SG.matmul(x2, weight.t(), bias=bias).view(*x.shape[:-1], weight.shape[0])
            else:
                y = F.linear(x, weight, bias.to(weight.dtype) if bias is not None else None)
        ctx.save_for_backward(x, weight)
        ctx.bias = bias
        ctx.sink_in = sink_in
        ctx.bias_handoff = bias_handoff
        return y

    @staticmethod
    def backward(ctx, dy):
        x, weight = ctx.saved_tensors
        bias = ctx.bias
        K = weight.shape[1]
        x2 = x.reshape(-1, K)
        dy2 = dy.reshape(-1, weight.shape[0])
        if dy2.dtype != weight.dtype:
            dy2 = dy2.to(weight.dtype)
        if not dy2.is_contiguous():
            dy2 = dy2.contiguous()
        dx = dw = db = None
        acc = ctx.sink_in.take() if ctx.sink_in is not None and ctx.needs_input_grad[0] else None
        if acc is not None:
            if acc.shape != x.shape or acc.dtype != dy2.dtype or not acc.is_contiguous():
                acc = acc.to(dy2.dtype).contiguous()
            if SG.supported(dy2, weight):
                SG.matmul(dy2, weight, out=acc.view(-1, K), accumulate=True)
            else:
                acc.view(-1, K).addmm_(dy2, weight)  # dX = residual gradient + dY . W
            dx = acc
        elif ctx.needs_input_grad[0]:
            dx = _dgrad(dy2, weight).view(x.shape)
        need_w, need_b = ctx.needs_input_grad[1], bias is not None and ctx.needs_input_grad[2]
        hb = ctx.bias_handoff
        if need_b and hb is not None and hb.done:
            need_b = False  # summed into the flat gradient by the next op's backward
            hb.done = False
        dw, db = linear_weight_grads(dy2, x2, weight, bias, need_w, need_b)
        return dx, dw, db, None, None


class _ResidualAddFn(torch.autograd.Function):
    """``x + y`` whose backward hands the gradient of ``x`` to ``sink`` (a later consumer
    accumulates into it in place) and returns it for ``y`` only."""

    @staticmethod
    def forward(ctx, x, y, sink):
        ctx.sink = sink
        return x + y

    @staticmethod
    def backward(ctx, g):
        if ctx.needs_input_grad[0]:
            # a fresh copy only when the y branch could still read g after the consumer ran;
            # here the consumer is the first GEMM applied to x, which autograd can reach only
            # after the whole y branch has been back-propagated (same stream)
            ctx.sink.put(g)
        return None, (g if ctx.needs_input_grad[1] else None), None


def residual_add(x: torch.Tensor, y: torch.Tensor, sink=None) -> torch.Tensor:
    """``x + y``; with a GradSink, x's gradient is accumulated by the GEMM that consumes x
    first (``FusedLinear(..., sink_in=sink)``) instead of by an autograd add."""
    if sink is None or x.shape != y.shape or x.dtype != y.dtype:
        return x + y
    return _ResidualAddFn.apply(x, y, sink)

class FusedLinear(torch.nn.Linear):
    """Drop-in ``nn.Linear`` using :class:`_DenseFn` (state-dict compatible)."""

    def forward(self, x, sink_in=None, bias_handoff=None):
        return _DenseFn.apply(x, self.weight, self.bias, sink_in, bias_handoff)
