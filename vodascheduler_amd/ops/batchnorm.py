"""Fused BatchNorm2d (+ residual add) (+ ReLU) on channels_last activations
(csrc/hip/batchnorm.hip).

``batch_norm_act(x, weight, bias, running_mean, running_var, training, momentum, eps,
residual=None, relu=True)`` computes ``relu(bn(x) + residual)`` (either extra optional) in
one statistics pass + one apply pass forward and one reduction pass + one apply pass
backward, instead of MIOpen BN + separate ReLU / add / ReLU-backward kernels.  The ReLU
mask of the backward is a 1-bit-per-element map written by the forward apply pass.
Statistics, running-stat updates and the affine parameters stay fp32; activations are
bf16/fp16/fp32.

GPU requirements: 4-D input in channels_last memory format (or a contiguous [M, C]
matrix) with C % 8 == 0; anything else, and CPU tensors, use the PyTorch reference
composition (which the GPU tests compare against).
"""
from __future__ import annotations

import os

import torch
import torch.nn.functional as F

from ..utils.flat import flat_grad
from . import _native as N
from .dense import _ready

# VODA_FUSED_BN=0: every BatchNorm takes the PyTorch reference composition (A/B and bisection
# runs, e.g. benchmarks/graph_diag.py)
USE_FUSED_BN = os.environ.get("VODA_FUSED_BN", "1") != "0"
# USE_FUSED_BN_POOL = False: the ResNet stem runs BN+ReLU and the max pool as two ops (module switch;
# fused: stem fwd+bwd 1014-1051 -> 744 us, ResNet-50 bs-256 step 26.43/26.47 -> 26.17/26.18 ms,
# profiles/raw/r2_ab_fused_stem.jsonl)
USE_FUSED_BN_POOL = True


def _rows_view_ok(x: torch.Tensor) -> bool:
    if x.dim() == 4:
        return x.is_contiguous(memory_format=torch.channels_last)
    return x.dim() == 2 and x.is_contiguous()


def _supported(x, residual) -> bool:
    if not x.is_cuda or x.dtype not in (torch.bfloat16, torch.float16, torch.float32):
        return False
    C = x.shape[1]
    if C % 8 != 0 or not _rows_view_ok(x) or x.numel() == 0:
        return False
    if residual is not None and (residual.shape != x.shape or residual.dtype != x.dtype
                                 or residual.stride() != x.stride()):
        return False
    return True


def _direct_fp32(p) -> bool:
    g = flat_grad(p)
    return g is not None and g.dtype == torch.float32 and g.is_contiguous()


class BwdHandoff:
    """Side channel from the GEMM that produces a BN's output gradient to that BN's backward.

    A ResNet block output ``x_b = relu(bn3(y3) + shortcut)`` feeds the next block's conv1,
    whose input-gradient GEMM (conv1x1_f32.hip ``gemm_f32_dgrad_bn``) writes x_b's gradient.
    The forward attaches this object to x_b (``HANDOFF_ATTR``) with what bn3's backward reduce
    pass would read -- its ReLU bits and input(s) -- so the GEMM's epilogue accumulates the
    reduce pass's sums (sum g, sum g*y3 [, sum g*y_ds]) and ``put``s them here; bn3's backward
    ``take``s them and runs only its finalize and apply passes.  The sums are used only when
    the gradient bn3 receives IS the tensor they were computed over."""

    __slots__ = ("mask", "x", "x2", "part", "nb", "grad")

    def __init__(self, mask, x, x2=None):
        self.mask, self.x, self.x2 = mask, x, x2
        self.part, self.nb, self.grad = None, 0, None

    def put(self, part: torch.Tensor, nb: int, grad: torch.Tensor) -> None:
        self.part, self.nb, self.grad = part, int(nb), grad

    def take(self, dy: torch.Tensor):
        """(partials, nb) when ``dy`` is the tensor the sums were computed over, else None."""
        got, g = (self.part, self.nb), self.grad
        self.part, self.nb, self.grad = None, 0, None
        # the same storage, and dy a dense row-major [M][C] view of it (channels_last or 2-D)
        if got[0] is None or g is None or dy.data_ptr() != g.data_ptr() or dy.numel() != g.numel() \
                or not _rows_view_ok(dy):
            return None
        return got


HANDOFF_ATTR = "_voda_bn_bwd_handoff"


class MaskedGrad:
    """A shortcut gradient ``g * relu_bits`` handed through a GradSink WITHOUT being
    materialised: the consuming input-gradient GEMM reads ``g`` and the 1-bit ReLU mask of
    the BN forward in its epilogue (ops/conv1x1.py fused path)."""

    __slots__ = ("g", "mask")

    def __init__(self, g: torch.Tensor, mask: torch.Tensor):
        self.g, self.mask = g, mask

    def dense(self) -> torch.Tensor:
        """The masked gradient as a tensor (fallback consumers)."""
        C = self.g.shape[1]
        bits = (self.mask.view(-1, 1) >> torch.arange(8, device=self.mask.device, dtype=torch.uint8)) & 1
        m = bits.view(-1, C).to(self.g.dtype)  # [M][C] in channels_last row order
        g2 = self.g.permute(0, 2, 3, 1).reshape(-1, C) if self.g.dim() == 4 else self.g
        out = (g2 * m)
        if self.g.dim() == 4:
            n, _, h, w = self.g.shape
            return out.view(n, h, w, C).permute(0, 3, 1, 2)
        return out


class _BNActFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, residual, weight, bias, running_mean, running_var, momentum, eps, relu, sink=None,
                stats=None, handoff=None):
        """``stats``: (workspace, nb) whose first 2 x nb x C floats are the producing GEMM's
        per-block sums / sums of squares of ``x`` (ops/conv1x1.py, gemm_bnstats.hip): the
        statistics pass is skipped."""
        C = x.shape[1]
        M = x.numel() // C
        h = N.hip()
        y = torch.empty_like(x)
        save_mean = torch.empty(C, dtype=torch.float32, device=x.device)
        save_invstd = torch.empty(C, dtype=torch.float32, device=x.device)
        if stats is not None:
            ws, pre_nb = stats
        else:
            ws, pre_nb = torch.empty(h.bn_workspace_floats(M, C), dtype=torch.float32, device=x.device), 0
        mask = torch.empty(M * (C // 8), dtype=torch.uint8, device=x.device) if relu else None
        h.bn_fwd_train(x.data_ptr(), N.ptr(residual), N.ptr(weight), N.ptr(bias), N.ptr(running_mean),
                       N.ptr(running_var), save_mean.data_ptr(), save_invstd.data_ptr(), y.data_ptr(), N.ptr(mask),
                       ws.data_ptr(), M, C, float(eps), float(momentum), bool(relu), N.dtype_code(x.dtype),
                       N.stream_of(x), int(pre_nb))
        ctx.relu = bool(relu)
        ctx.has_res = residual is not None
        ctx.bias = bias
        ctx.sink = sink if residual is not None else None
        ctx.handoff = handoff
        if handoff is not None:
            handoff.mask, handoff.x = mask, x
        ctx.save_for_backward(x, mask, weight, save_mean, save_invstd)
        return y

    @staticmethod
    def backward(ctx, dy):
        x, mask, weight, save_mean, save_invstd = ctx.saved_tensors
        C = x.shape[1]
        M = x.numel() // C
        h = N.hip()
        if not _rows_view_ok(dy) or dy.stride() != x.stride():
            dy = dy.contiguous(memory_format=torch.channels_last) if dy.dim() == 4 else dy.contiguous()
        dx = torch.empty_like(x)
        pre = ctx.handoff.take(dy) if ctx.handoff is not None else None
        # a sink whose consumer reads the masked shortcut gradient in its GEMM epilogue: hand
        # over (dy, ReLU bits) instead of writing dres = dy * bits
        lazy = (ctx.sink is not None and getattr(ctx.sink, "lazy", False) and ctx.relu and ctx.has_res
                and ctx.needs_input_grad[1])
        dres = torch.empty_like(x) if ctx.has_res and ctx.needs_input_grad[1] and not lazy else None
        need_w = weight is not None and ctx.needs_input_grad[2]
        need_b = ctx.needs_input_grad[3]
        bias = ctx.bias
        # fp32 gamma/beta grads go straight into the optimizer's flat grad buffer when it
        # owns them (same contract as ops/dense.py), else into fresh tensors
        direct = (need_b and _direct_fp32(bias) and ((need_w and _direct_fp32(weight)) or weight is None))
        if direct:
            dw, db = flat_grad(weight), flat_grad(bias)
        else:
            dw = torch.empty(C, dtype=torch.float32, device=x.device) if need_w else None
            db = torch.empty(C, dtype=torch.float32, device=x.device) if need_b else None
        ws = torch.empty(h.bn_workspace_floats(M, C), dtype=torch.float32, device=x.device)
        h.bn_bwd(dy.data_ptr(), N.ptr(mask), x.data_ptr(), save_mean.data_ptr(), save_invstd.data_ptr(), N.ptr(weight),
                 dx.data_ptr(), N.ptr(dres), N.ptr(dw), N.ptr(db), ws.data_ptr(), M, C, ctx.relu, direct,
                 N.dtype_code(x.dtype), N.stream_of(x), N.ptr(pre[0]) if pre else 0, pre[1] if pre else 0)
        if lazy:
            ctx.sink.put(MaskedGrad(dy, mask))
        elif dres is not None and ctx.sink is not None:
            ctx.sink.put(dres)  # a fresh tensor: the consumer may accumulate into it in place
            dres = None
        if dres is None and ctx.has_res and ctx.needs_input_grad[1] and ctx.sink is None:
            dres = dy
        if direct:
            if weight is not None:
                _ready(weight)
            _ready(bias)
            return dx, dres, None, None, None, None, None, None, None, None, None, None
        return dx, dres, dw, db, None, None, None, None, None, None, None, None


class _BNAct2Fn(torch.autograd.Function):
    """``relu?(bn(x) + bn2(x2))`` in training mode (csrc/hip/batchnorm.hip ``bn2_*``): the
    second BN's output -- a ResNet downsample block's shortcut -- is never materialised, and
    both BNs share one reduce pass and one apply pass backward."""

    @staticmethod
    def forward(ctx, x, x2, weight, bias, running_mean, running_var, weight2, bias2, running_mean2, running_var2,
                momentum, eps, relu, stats, stats2, handoff=None):
        C = x.shape[1]
        M = x.numel() // C
        h = N.hip()
        y = torch.empty_like(x)
        f32 = dict(dtype=torch.float32, device=x.device)
        sm, si, sm2, si2 = (torch.empty(C, **f32) for _ in range(4))
        ws, nb = stats if stats is not None else (torch.empty(h.bn_workspace_floats(M, C), **f32), 0)
        ws2, nb2 = stats2 if stats2 is not None else (torch.empty(h.bn_workspace_floats(M, C), **f32), 0)
        mask = torch.empty(M * (C // 8), dtype=torch.uint8, device=x.device) if relu else None
        h.bn2_fwd_train(x.data_ptr(), x2.data_ptr(), N.ptr(weight), N.ptr(bias), N.ptr(running_mean),
                        N.ptr(running_var), sm.data_ptr(), si.data_ptr(), N.ptr(weight2), N.ptr(bias2),
                        N.ptr(running_mean2), N.ptr(running_var2), sm2.data_ptr(), si2.data_ptr(), y.data_ptr(),
                        N.ptr(mask), ws.data_ptr(), ws2.data_ptr(), M, C, float(eps), float(momentum), bool(relu),
                        N.dtype_code(x.dtype), N.stream_of(x), int(nb), int(nb2))
        ctx.relu = bool(relu)
        ctx.biases = (bias, bias2)
        ctx.handoff = handoff
        if handoff is not None:
            handoff.mask, handoff.x, handoff.x2 = mask, x, x2
        ctx.save_for_backward(x, x2, mask, weight, weight2, sm, si, sm2, si2)
        return y

    @staticmethod
    def backward(ctx, dy):
        x, x2, mask, weight, weight2, sm, si, sm2, si2 = ctx.saved_tensors
        bias, bias2 = ctx.biases
        C = x.shape[1]
        M = x.numel() // C
        h = N.hip()
        if not _rows_view_ok(dy) or dy.stride() != x.stride():
            dy = dy.contiguous(memory_format=torch.channels_last) if dy.dim() == 4 else dy.contiguous()
        dx, dx2 = torch.empty_like(x), torch.empty_like(x2)
        nw = (weight is not None and ctx.needs_input_grad[2], weight2 is not None and ctx.needs_input_grad[6])
        nbias = (ctx.needs_input_grad[3], ctx.needs_input_grad[7])
        # fp32 gamma / beta gradients straight into the optimizer's flat buffers when it owns
        # all four, else into fresh tensors (same contract as _BNActFn)
        direct = all(nbias) and all(_direct_fp32(b) for b in (bias, bias2)) and all(
            (n and _direct_fp32(w_)) or w_ is None for n, w_ in zip(nw, (weight, weight2)))
        f32 = dict(dtype=torch.float32, device=x.device)
        if direct:
            dw, db, dw2, db2 = flat_grad(weight), flat_grad(bias), flat_grad(weight2), flat_grad(bias2)
        else:
            dw = torch.empty(C, **f32) if nw[0] else None
            db = torch.empty(C, **f32) if nbias[0] else None
            dw2 = torch.empty(C, **f32) if nw[1] else None
            db2 = torch.empty(C, **f32) if nbias[1] else None
        pre = ctx.handoff.take(dy) if ctx.handoff is not None else None
        ws = torch.empty(h.bn2_workspace_floats(M, C), **f32)
        h.bn2_bwd(dy.data_ptr(), N.ptr(mask), x.data_ptr(), x2.data_ptr(), sm.data_ptr(), si.data_ptr(), N.ptr(weight),
                  sm2.data_ptr(), si2.data_ptr(), N.ptr(weight2), dx.data_ptr(), dx2.data_ptr(), N.ptr(dw), N.ptr(db),
                  N.ptr(dw2), N.ptr(db2), ws.data_ptr(), M, C, ctx.relu, direct, N.dtype_code(x.dtype),
                  N.stream_of(x), N.ptr(pre[0]) if pre else 0, pre[1] if pre else 0)
        if direct:
            for t in (weight, bias, weight2, bias2):
                if t is not None:
                    _ready(t)
            return dx, dx2, None, None, None, None, None, None, None, None, None, None, None, None, None, None
        return dx, dx2, dw, db, None, None, dw2, db2, None, None, None, None, None, None, None, None


STATS_ATTR = "_voda_bn_stats"


def attach_stats(y: torch.Tensor, ws: torch.Tensor, nb: int) -> torch.Tensor:
    """Mark ``y`` as carrying its BN partial statistics (first 2 x nb x C floats of ``ws``,
    which must also hold the finalize's 3 x C tail)."""
    setattr(y, STATS_ATTR, (ws, int(nb)))
    return y


def take_stats(x: torch.Tensor):
    """The partial statistics a producing GEMM attached to ``x`` (consumed once), or None."""
    st = getattr(x, STATS_ATTR, None)
    if st is not None:
        delattr(x, STATS_ATTR)
    return st


def _reference(x, weight, bias, running_mean, running_var, training, momentum, eps, residual, relu):
    y = F.batch_norm(x, running_mean, running_var, weight, bias, training, momentum, eps)
    if residual is not None:
        y = y + residual
    return F.relu(y) if relu else y


def batch_norm_act(x: torch.Tensor, weight: torch.Tensor | None, bias: torch.Tensor | None,
                   running_mean: torch.Tensor | None, running_var: torch.Tensor | None, training: bool = True,
                   momentum: float = 0.1, eps: float = 1e-5, residual: torch.Tensor | None = None,
                   relu: bool = True, sink=None) -> torch.Tensor:
    """``sink``: hand the residual's gradient to a consumer (ops/conv1x1.GradSink) instead of
    returning it; ignored (gradient returned normally) on the reference path."""
    # the kernels read gamma / beta / running statistics as fp32 (normalisation parameters
    # stay fp32 under cast_compute_weights_); anything else takes the reference path
    params_fp32 = all(t is None or t.dtype == torch.float32 for t in (weight, bias, running_mean, running_var))
    if not USE_FUSED_BN or not params_fp32 or not _supported(x, residual):
        return _reference(x, weight, bias, running_mean, running_var, training, momentum, eps, residual, relu)
    if training or running_mean is None:
        stats = take_stats(x)
        hand = BwdHandoff(None, None) if (relu and residual is not None and x.dtype == torch.float32) else None
        y = _BNActFn.apply(x, residual, weight, bias, running_mean, running_var, momentum, eps, relu, sink, stats,
                           hand)
        if hand is not None:
            setattr(y, HANDOFF_ATTR, hand)
        return y
    # inference: per-channel affine from the running statistics, one apply pass
    C = x.shape[1]
    invstd = torch.rsqrt(running_var.float() + eps)
    a = invstd * (weight.float() if weight is not None else 1.0)
    b = (bias.float() if bias is not None else 0.0) - running_mean.float() * a
    ab = torch.cat([a.reshape(C), b.reshape(C)]).contiguous()
    y = torch.empty_like(x)
    N.hip().bn_apply(x.data_ptr(), N.ptr(residual), ab.data_ptr(), y.data_ptr(), x.numel() // C, C, bool(relu),
                     N.dtype_code(x.dtype), N.stream_of(x))
    return y


def _pool_out(n: int, k: int, s: int, p: int) -> int:
    return (n + 2 * p - k) // s + 1


def bn_pool_forward(x, weight, bias, running_mean, running_var, momentum, eps, k, s, p, ws=None, pre_nb=0):
    """maxpool(relu(bn(x))) training forward; ``ws`` / ``pre_nb``: a workspace whose first
    2 x pre_nb x C floats already hold the per-block sums / sums of squares of ``x`` (the
    producing convolution's epilogue, ops/stem.py) -- the statistics pass is skipped.
    Returns (y, idx, save_mean, save_invstd)."""
    Nb, C, H, W = x.shape
    Ho, Wo = _pool_out(H, k, s, p), _pool_out(W, k, s, p)
    h = N.hip()
    y = torch.empty(Nb, C, Ho, Wo, dtype=x.dtype, device=x.device, memory_format=torch.channels_last)
    idx = torch.empty(Nb * Ho * Wo * C, dtype=torch.uint8, device=x.device)
    save_mean = torch.empty(C, dtype=torch.float32, device=x.device)
    save_invstd = torch.empty(C, dtype=torch.float32, device=x.device)
    if ws is None:
        ws = torch.empty(h.bn_pool_workspace_floats(Nb, H, C), dtype=torch.float32, device=x.device)
    h.bn_pool_fwd_train(x.data_ptr(), N.ptr(weight), N.ptr(bias), N.ptr(running_mean), N.ptr(running_var),
                        save_mean.data_ptr(), save_invstd.data_ptr(), y.data_ptr(), idx.data_ptr(), ws.data_ptr(),
                        Nb, H, W, C, Ho, Wo, k, s, p, float(eps), float(momentum), N.dtype_code(x.dtype),
                        N.stream_of(x), int(pre_nb))
    return y, idx, save_mean, save_invstd


def bn_pool_backward(dy, x, idx, weight, bias, save_mean, save_invstd, k, s, p, need_w, need_b):
    """Gradients of :func:`bn_pool_forward`: (dx, dgamma, dbeta, direct) -- ``direct``: the
    affine gradients went straight into the optimizer's flat fp32 buffers."""
    Nb, C, H, W = x.shape
    Ho, Wo = _pool_out(H, k, s, p), _pool_out(W, k, s, p)
    h = N.hip()
    dy = dy.to(x.dtype).contiguous(memory_format=torch.channels_last)
    dx = torch.empty_like(x)
    direct = (need_b and _direct_fp32(bias) and ((need_w and _direct_fp32(weight)) or weight is None))
    if direct:
        dw, db = flat_grad(weight), flat_grad(bias)
    else:
        dw = torch.empty(C, dtype=torch.float32, device=x.device) if need_w else None
        db = torch.empty(C, dtype=torch.float32, device=x.device) if need_b else None
    ws = torch.empty(h.bn_pool_workspace_floats(Nb, H, C), dtype=torch.float32, device=x.device)
    h.bn_pool_bwd(dy.data_ptr(), idx.data_ptr(), x.data_ptr(), save_mean.data_ptr(), save_invstd.data_ptr(),
                  N.ptr(weight), dx.data_ptr(), N.ptr(dw), N.ptr(db), ws.data_ptr(), Nb, H, W, C, Ho, Wo, k, s, p,
                  direct, N.dtype_code(x.dtype), N.stream_of(x))
    if direct:
        if weight is not None:
            _ready(weight)
        _ready(bias)
        return dx, None, None, True
    return dx, dw, db, False


class _BNPoolFn(torch.autograd.Function):
    """maxpool(relu(bn(x))) in training mode (csrc/hip/batchnorm.hip ``bn_pool_*``): the
    full-resolution BN output and its gradient are never written to memory."""

    @staticmethod
    def forward(ctx, x, weight, bias, running_mean, running_var, momentum, eps, k, s, p):
        y, idx, save_mean, save_invstd = bn_pool_forward(x, weight, bias, running_mean, running_var, momentum, eps,
                                                         k, s, p)
        ctx.pool = (k, s, p)
        ctx.bias = bias
        ctx.save_for_backward(x, idx, weight, save_mean, save_invstd)
        return y

    @staticmethod
    def backward(ctx, dy):
        x, idx, weight, save_mean, save_invstd = ctx.saved_tensors
        need_w = weight is not None and ctx.needs_input_grad[1]
        dx, dw, db, _ = bn_pool_backward(dy, x, idx, weight, ctx.bias, save_mean, save_invstd, *ctx.pool, need_w,
                                         ctx.needs_input_grad[2])
        return dx, dw, db, None, None, None, None, None, None, None


class FusedBatchNorm2d(torch.nn.BatchNorm2d):
    """``BatchNorm2d`` whose forward optionally adds a residual and applies ReLU:
    ``forward(x, residual=None) = relu?(bn(x) + residual)``.  State dict compatible with
    ``torch.nn.BatchNorm2d``."""

    def __init__(self, num_features: int, eps: float = 1e-5, momentum: float = 0.1, relu: bool = False,
                 scale: bool = True, **kw):
        """``scale=False``: no gamma (Keras ``BatchNormalization(scale=False)``, used by the
        reference's InceptionV3 conv2d_bn blocks); beta and the running statistics remain."""
        super().__init__(num_features, eps=eps, momentum=momentum, **kw)
        self.relu = relu
        if not scale and self.affine:
            self.register_parameter("weight", None)

    def _load_from_state_dict(self, state_dict, prefix, *args, **kwargs):
        self._pending_batches = 0
        super()._load_from_state_dict(state_dict, prefix, *args, **kwargs)

    def _save_to_state_dict(self, destination, prefix, keep_vars):
        self.sync_batches_tracked()
        super()._save_to_state_dict(destination, prefix, keep_vars)

    def sync_batches_tracked(self) -> None:
        """Fold the host-side step count into the ``num_batches_tracked`` buffer."""
        n = getattr(self, "_pending_batches", 0)
        if n and self.num_batches_tracked is not None:
            self.num_batches_tracked.add_(n)
            self._pending_batches = 0

    def forward(self, x, residual=None, sink=None):
        if self.training and self.track_running_stats:
            if self.momentum is None:  # cumulative average needs the device count now
                self.num_batches_tracked.add_(1)
            else:  # only informational: count on the host (saves a kernel per BN per step)
                self._pending_batches = getattr(self, "_pending_batches", 0) + 1
        use_batch = self.training or not self.track_running_stats
        momentum = self.momentum if self.momentum is not None else 0.1
        if x.is_cuda and torch.is_autocast_enabled("cuda"):
            with torch.autocast("cuda", enabled=False):  # keep the activation dtype, fp32 stats
                return batch_norm_act(x, self.weight, self.bias, self.running_mean if self.track_running_stats
                                      else None, self.running_var if self.track_running_stats else None,
                                      use_batch, momentum, self.eps, residual, self.relu, sink)
        return batch_norm_act(x, self.weight, self.bias,
                              self.running_mean if self.track_running_stats else None,
                              self.running_var if self.track_running_stats else None,
                              use_batch, momentum, self.eps, residual, self.relu, sink)

    def _count_batch(self) -> None:
        if self.training and self.track_running_stats:
            if self.momentum is None:
                self.num_batches_tracked.add_(1)
            else:
                self._pending_batches = getattr(self, "_pending_batches", 0) + 1

    def forward_pair(self, x, other: "FusedBatchNorm2d", x2):
        """``relu?(self(x) + other(x2))`` -- a ResNet downsample block's output with its
        shortcut BN folded in (``_BNAct2Fn``: no materialised shortcut, one shared backward
        reduce / apply).  Falls back to the two-module composition off the fused path."""
        ok = (USE_FUSED_BN and self.training and other.training and self.track_running_stats
              and other.track_running_stats and not other.relu and self.momentum is not None
              and other.momentum is not None and self.momentum == other.momentum and self.eps == other.eps
              and _supported(x, x2) and x.shape == x2.shape
              and all(t is None or t.dtype == torch.float32 for m_ in (self, other)
                      for t in (m_.weight, m_.bias, m_.running_mean, m_.running_var)))
        if not ok:
            return self(x, other(x2))
        self._count_batch()
        other._count_batch()
        hand = BwdHandoff(None, None) if (self.relu and x.dtype == torch.float32) else None
        with torch.autocast("cuda", enabled=False):
            y = _BNAct2Fn.apply(x, x2, self.weight, self.bias, self.running_mean, self.running_var, other.weight,
                                other.bias, other.running_mean, other.running_var, self.momentum, self.eps,
                                self.relu, take_stats(x), take_stats(x2), hand)
        if hand is not None:
            setattr(y, HANDOFF_ATTR, hand)
        return y

    def extra_repr(self):
        return super().extra_repr() + f", relu={self.relu}"


class FusedBNReLUMaxPool2d(FusedBatchNorm2d):
    """``maxpool(relu(bn(x)))`` -- the ResNet stem's BN + ReLU + MaxPool2d(k, s, p) -- as one
    module (state dict of the ``BatchNorm2d``).  Training on the GPU path runs the fused
    kernels (``_BNPoolFn``); evaluation and unsupported inputs run the composition."""

    def __init__(self, num_features: int, kernel_size: int = 3, stride: int = 2, padding: int = 1, **kw):
        super().__init__(num_features, relu=True, **kw)
        self.pool = (kernel_size, stride, padding)

    def _fused_ok(self, x) -> bool:
        k, s, p = self.pool
        return (USE_FUSED_BN and USE_FUSED_BN_POOL and self.training and self.track_running_stats
                and x.is_cuda and x.dim() == 4 and x.dtype in (torch.bfloat16, torch.float32)
                and x.is_contiguous(memory_format=torch.channels_last) and x.shape[1] % 8 == 0
                and x.shape[1] <= 2048 and (k, s) == (3, 2) and 2 * p <= k
                and all(t is None or t.dtype == torch.float32 for t in (self.weight, self.bias)))

    def forward(self, x, residual=None, sink=None):
        from .pool import max_pool2d

        if residual is None and self._fused_ok(x):
            if self.momentum is None:
                self.num_batches_tracked.add_(1)
            else:
                self._pending_batches = getattr(self, "_pending_batches", 0) + 1
            k, s, p = self.pool
            with torch.autocast("cuda", enabled=False):
                return _BNPoolFn.apply(x, self.weight, self.bias, self.running_mean, self.running_var,
                                       self.momentum if self.momentum is not None else 0.1, self.eps, k, s, p)
        return max_pool2d(super().forward(x, residual, sink), *self.pool)

    def extra_repr(self):
        return super().extra_repr() + f", pool={self.pool}"
