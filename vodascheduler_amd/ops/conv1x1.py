"""1x1 convolution of channels_last activations as GEMMs (ResNet bottlenecks).

A 1x1 convolution over an NHWC tensor is a plain GEMM on its ``[N*H*W, C]`` view:

    forward          Y[m, co] = X[m, :] . W[co, :]          hipBLASLt (view, no copy)
    input gradient   dX[m, ci] = dY[m, :] . W[:, ci]        hipBLASLt
    weight gradient  dW[co, ci] (+)= sum_m dY[m, co] X[m, ci]  split-K MFMA kernel
                                                           (csrc/hip/wgrad.hip), accumulated
                                                           straight into the optimizer's
                                                           flat gradient (fp32)

MIOpen runs these as implicit-GEMM convolution kernels; the weight-gradient ones are the
"reduction over 800k pixels" shape the split-K kernel is built for.  Stride-2 1x1
convolutions (ResNet downsample) subsample the input first and scatter the input gradient
back.  Convolutions with fewer than 128 input channels (ResNet stage 1: K = 64 is half an
MFMA tile) stay on MIOpen, which is faster there (benchmarks/bench_conv1x1.py,
profiles/raw/r1_bench_conv1x1.log: 11.7 -> 9.0 ms for all 1x1 convolutions of a ResNet-50
bs256 step, 0.68-0.96x on the Cin = 64 shapes).  The layer is a drop-in ``nn.Conv2d`` (same parameters / state dict); anything it does
not cover (CPU tensors, non-bf16, groups, padding, bias, a layout that is not
channels_last) runs ``F.conv2d``.
"""
from __future__ import annotations

import os

import torch
import torch.nn.functional as F

from ..utils.flat import FOLD_CAST, flat_grad
from . import _native as N
from . import splitgemm as SG
from . import wgrad as W

# Kernel-path switches (module constants; tests monkeypatch them to reach the other branch):
USE_CONV1X1_GEMM = True   # bf16 1x1 convolutions with >= 128 input channels as GEMMs (else MIOpen)
# stride-2 input gradients handed through a GradSink subsampled (_StridedGrad) instead of as a
# zero-filled full-resolution tensor
USE_STRIDED_SINK = True
USE_GRAD_SINK = True      # GradSink shortcut-gradient hand-offs (else autograd adds them)
# expansion 1x1 convolutions (K = 64 / 128 / 256 in) with the BN statistics in the GEMM epilogue
# (gemm_bnstats.hip, conv1x1_f32.hip; ResNet-50 bf16 23.78 -> 23.15 ms); VODA_GEMM_BNSTATS=0 is the
# A/B switch
USE_GEMM_BNSTATS = os.environ.get("VODA_GEMM_BNSTATS", "1") != "0"
# Input gradients dX = dY . W of the memory-bound 1x1 shapes (K = Cout in {64, 128, 256}) that
# overwrite their output, on the MFMA GEMM of gemm_bnstats.hip / conv1x1_f32.hip instead of
# hipBLASLt / MIOpen (benchmarks/bench_dgrad_gemm.py: 802816 x 256 -> 64 167 -> 102 us, 64 -> 256
# 142 -> 108, 128 -> 256 168 -> 130, 200704 x 128 -> 512 77 -> 59; profiles/r3/raw/mfma_dgrad/).
# The accumulate (beta = 1) form of the same GEMMs is kept as a tested kernel feature, but the
# models use hipBLASLt's beta = 1 (or, fp32 identity blocks, the fused input gradient below):
# the own read-add-write epilogue measured 2x slower in the step (profiles/r4/sink_gemm_ab.md)
USE_MFMA_DGRAD = True
# fp32 (the reference's precision): 1x1 convolutions as GEMMs with the f32-MFMA kernels of
# conv1x1_f32.hip -- forward with the BN statistics in the epilogue and input gradient for
# K = 64 / 128 / 256, hipBLASLt for the rest -- and the GradSink hand-offs of the bf16 path (no
# residual-gradient adds).  Weight gradients stay on MIOpen (the own split-K / streaming fp32
# weight-gradient kernels measured slower and were removed in round 5), except the
# short-reduction, wide-output ones below.  VODA_CONV1X1_F32=0: fp32 1x1 convolutions stay on
# MIOpen (A/B switch)
USE_CONV1X1_F32 = os.environ.get("VODA_CONV1X1_F32", "1") != "0"
USE_GEMM_F32 = True
# ... the short-reduction, wide-output fp32 weight gradients (stage 4 of ResNet-50: 7x7 maps,
# M = 12544 pixels into 1M-2M weights), where one hipBLASLt GEMM with beta = 1 into the flat
# gradient runs 189-199 us vs MIOpen's 214-226 us plus the fold-in add, and 353 vs 417-434 us on
# the stride-2 1024 -> 2048 shortcut (profiles/r4/resnet50_fp32_1x1_wgrad_*.jsonl).  MIOpen wins
# everywhere M >= 50176.
USE_BLAS_WGRAD_F32 = True
BLAS_WGRAD_F32_MAX_M = 16384
BLAS_WGRAD_F32_MIN_OUT = 1 << 20


# fp32 1x1 GEMMs the f32-MFMA kernels above do not take (K >= 512 forwards, the input gradients
# with K = Cout >= 512, also into a sink) on the split-bf16 MFMA GEMM (ops/splitgemm.py: fp32
# accuracy on the bf16 matrix cores) instead of hipBLASLt.  Early in round 6 (the dual-accumulator
# variant 0) the split GEMM lost to the libraries in the step (same-box A/B 65.06 -> 66.75 ms,
# profiles/r6/ab_split_resnet50_fp32.jsonl); SPLIT_VARIANT 1 (one accumulator, software-pipelined
# split; error still <= hipBLASLt fp32's) runs the 13 library shapes 170-335 us vs 174-351 us for
# variant 0 and 186-463 us for UNTUNED hipBLASLt (profiles/r6/resnet50_1x1_split_probe.jsonl), but
# the step uses the shipped tuned hipBLASLt solutions and still loses: 60.85 -> 61.97 ms (same-box
# A/B, profiles/r6/ab_split_1x1_v1_resnet50_fp32.jsonl).  Stays off.
USE_SPLIT_GEMM_F32 = False
# None: the split GEMM's own plan (variant 8, three workgroups per CU, since the 96-B K-contiguous
# layout; variant 1 before)
SPLIT_VARIANT = None
# ... but the FORWARDS with K >= 512 input channels alone do win: a per-call rocprof of the step with
# every library 1x1 GEMM on the split kernel (profiles/r6/rocprof_resnet50_fp32_split_1x1_calls.md)
# has the ten K >= 512 forwards 0-10 % faster than the tuned hipBLASLt solutions (-160 us per
# step), while the K = 64 forward lost 76 -> 221 us and the input gradients +1.4 ms.  Routed
# alone, the same-box step A/B still lost: 59.11 -> 59.67 ms (profiles/r6/
# ab_split_fwd_1x1_resnet50_fp32.jsonl), so it stays off
USE_SPLIT_FWD_F32 = False
SPLIT_FWD_MIN_K = 512
# the fp32 1x1 weight gradients (reduction over the pixels) on the split-bf16 GEMM, split-K to
# ~1024 workgroups (else MIOpen / hipBLASLt as before): ResNet-50 fp32 60.49 -> 60.37 ms
# (same-box A/B, profiles/r6/ab_split_1x1_wgrad_resnet50_fp32.jsonl)
USE_SPLIT_WGRAD_F32 = True
# ... with the 64 x 256 / 256 x 64 tiles where the output has a 64-wide side (stage 1: [64][256],
# [256][64], [64][64]) instead of half-empty 128 x 128 tiles
USE_THIN_TILES = True
# ... split-K to ~this many workgroups (one round of the 512 resident ones; 1024 before round 6's
# sweep, profiles/r6/resnet50_wgrad_splits_probe_b.jsonl)
WGRAD_TARGET_WG = 512
# ... and on the 128 x 128 tile as GEMM variant 8 (one accumulator, three workgroups per CU; A/B switch)
WGRAD_V8 = True


def _sx(a: torch.Tensor, b: torch.Tensor) -> bool:
    return USE_SPLIT_GEMM_F32 and a.dtype == torch.float32 and SG.supported(a, b)


def _mm(a: torch.Tensor, b: torch.Tensor) -> torch.Tensor:
    """a @ b on the split-bf16 GEMM when it takes the fp32 operands, else the library."""
    return SG.matmul(a, b, variant=SPLIT_VARIANT) if _sx(a, b) else a @ b


def _addmm_(c: torch.Tensor, a: torch.Tensor, b: torch.Tensor) -> None:
    """c += a @ b (c [M, N] with unit column stride)."""
    if _sx(a, b) and c.dtype == torch.float32 and c.stride(1) == 1:
        SG.matmul(a, b, out=c, accumulate=True, variant=SPLIT_VARIANT)
    else:
        c.addmm_(a, b)


def blas_wgrad_f32_ok(m: int, cout: int, cin: int) -> bool:
    """fp32 1x1 weight gradient [cout, cin] = dY[m, cout]^T . X[m, cin] on hipBLASLt?"""
    return USE_BLAS_WGRAD_F32 and m <= BLAS_WGRAD_F32_MAX_M and cout * cin >= BLAS_WGRAD_F32_MIN_OUT


# fp32 identity bottlenecks: conv1's input gradient reads the masked shortcut gradient and
# accumulates the previous block's bn3 backward sums in its epilogue (gemm_f32_dgrad_bn,
# ops/batchnorm.BwdHandoff / MaskedGrad; ResNet-50 fp32 68.0 -> 67.1 ms,
# profiles/r5/ab_fused_dgrad_bn_resnet50_fp32.jsonl).  VODA_FUSED_DGRAD_BN=0: hipBLASLt beta = 1 +
# separate BN reduce pass (A/B switch)
USE_FUSED_DGRAD_BN = os.environ.get("VODA_FUSED_DGRAD_BN", "1") != "0"


def fused_dgrad_bn_ok(m: int, cin: int, cout: int) -> bool:
    """Does gemm_f32_dgrad_bn cover dX [m, cin] = dY [m, cout] . W [cout, cin]?"""
    return USE_FUSED_DGRAD_BN and bool(N.hip().gemm_f32_dgrad_bn_supported(m, cin, cout))


def fused_dgrad_bn(dy2: torch.Tensor, w2: torch.Tensor, acc, handoff) -> torch.Tensor | None:
    """dX [M, N] = dY [M, K] . W [K, N] + acc.g * relu_bits(acc.mask) on the fused kernel, with
    the previous block's bn3 backward sums put into ``handoff`` when it describes dX; None when
    the kernel does not cover the operands (the caller materialises the masked gradient)."""
    from .batchnorm import BwdHandoff

    M, K = dy2.shape
    Nn = w2.shape[1]
    g = acc.g
    if (not USE_FUSED_DGRAD_BN or dy2.dtype != torch.float32 or g.dtype != torch.float32 or not dy2.is_contiguous()
            or dy2.data_ptr() % 16 or not w2.is_contiguous() or g.numel() != M * Nn
            or not g.is_contiguous(memory_format=torch.channels_last) or acc.mask.numel() * 8 != M * Nn):
        return None
    h = N.hip()
    if not h.gemm_f32_dgrad_bn_supported(M, Nn, K):
        return None
    hand = handoff if isinstance(handoff, BwdHandoff) and handoff.mask is not None else None
    if hand is not None and (hand.x.numel() != M * Nn or hand.x.dtype != torch.float32
                             or (hand.x2 is not None and hand.x2.numel() != M * Nn)):
        hand = None
    ns = 0 if hand is None else (3 if hand.x2 is not None else 2)
    G = h.gemm_f32_dgrad_bn_groups(M, Nn, K, ns)
    out = torch.empty(M, Nn, dtype=torch.float32, device=dy2.device)
    part = torch.empty(max(1, ns * G * Nn), dtype=torch.float32, device=dy2.device) if ns else None
    h.gemm_f32_dgrad_bn(dy2.data_ptr(), w2.data_ptr(), out.data_ptr(), g.data_ptr(), acc.mask.data_ptr(),
                        N.ptr(hand.mask) if hand else 0, N.ptr(hand.x) if hand else 0,
                        N.ptr(hand.x2) if hand and hand.x2 is not None else 0, N.ptr(part), M, Nn, K, G, ns,
                        N.stream_of(dy2))
    if hand is not None:
        hand.put(part, G, out)
    return out


class GradSink:
    """One-shot hand-off of an activation gradient between the two backward nodes of a
    tensor with two consumers (a residual block input feeds the block's first 1x1
    convolution and the shortcut).  Autograd would materialise both gradients and add
    them in a separate elementwise kernel (three full passes over the activation: 16 per
    ResNet-50 step, ~1.4 ms on MI355X, profiles/raw/r1_steady_kernels_resnet_gemm.csv).
    Instead the shortcut's backward node ``put``s its gradient here and returns None for
    that input, and the first convolution's input-gradient GEMM accumulates into it with
    beta = 1 and returns it.  The consumer runs after the producer by construction: its
    output gradient only exists once the whole residual branch (which ends at the
    producer) has been back-propagated."""

    __slots__ = ("buf", "lazy")

    def __init__(self, lazy: bool = False):
        self.buf = None
        # the consumer runs the fused input gradient: the producer may hand over a MaskedGrad
        self.lazy = lazy

    def put(self, g: torch.Tensor) -> None:
        self.buf = g

    def take(self) -> torch.Tensor | None:
        g, self.buf = self.buf, None
        return g


class _StridedGrad:
    """Input gradient of a stride-s 1x1 convolution, handed through a GradSink WITHOUT the
    zero-filled full-resolution tensor: ``g`` holds the gradient of the subsampled pixels
    (every s-th row / column).  The consumer's GEMM writes its own full gradient (beta = 0)
    and adds ``g`` into the strided positions -- instead of a full-size zero fill + scatter
    that the GEMM then re-reads as its C operand (ResNet-50 downsample blocks: ~1 GB of
    traffic per step less)."""

    __slots__ = ("g", "stride", "shape")

    def __init__(self, g: torch.Tensor, stride: int, shape):
        self.g, self.stride, self.shape = g, stride, shape

    def dense(self) -> torch.Tensor:
        N_, C_, H_, W_ = self.shape
        s = self.stride
        dx = self.g.new_zeros((N_, H_, W_, C_)).permute(0, 3, 1, 2)  # channels_last
        dx[:, :, ::s, ::s] = self.g
        return dx


def _sub_ok(t: torch.Tensor) -> bool:
    return (t.is_cuda and t.dim() == 4 and t.dtype in (torch.bfloat16, torch.float32) and t.shape[1] % 8 == 0
            and t.is_contiguous(memory_format=torch.channels_last) and t.data_ptr() % 16 == 0)


def subsample(x: torch.Tensor, s: int) -> torch.Tensor:
    """``x[:, :, ::s, ::s]`` as a dense channels_last tensor (pool.hip ``subsample2d`` for
    channels_last bf16; a strided copy otherwise)."""
    if not _sub_ok(x):
        return x[:, :, ::s, ::s].contiguous(memory_format=torch.channels_last)
    n, c, h, w = x.shape
    y = torch.empty(n, c, (h + s - 1) // s, (w + s - 1) // s, dtype=x.dtype, device=x.device,
                    memory_format=torch.channels_last)
    N.hip().subsample2d(x.data_ptr(), y.data_ptr(), n, h, w, c, s, False, N.dtype_code(x.dtype), N.stream_of(x))
    return y


def subsample_add_(dx: torch.Tensor, g: torch.Tensor, s: int) -> None:
    """``dx[:, :, ::s, ::s] += g`` in place."""
    n, c, h, w = dx.shape
    if _sub_ok(dx) and _sub_ok(g) and tuple(g.shape) == (n, c, (h + s - 1) // s, (w + s - 1) // s):
        N.hip().subsample2d(g.data_ptr(), dx.data_ptr(), n, h, w, c, s, True, N.dtype_code(dx.dtype),
                            N.stream_of(dx))
    else:
        dx[:, :, ::s, ::s].add_(g)


class StatsHolder:
    """Side channel from a forward GEMM that computed its output's BN partial statistics to
    the module, which attaches them to the returned tensor (ops/batchnorm.attach_stats)."""

    __slots__ = ("stats",)

    def __init__(self):
        self.stats = None


def _f32_ok(*ts: torch.Tensor) -> bool:
    return all(t.dtype == torch.float32 and t.is_contiguous() and t.data_ptr() % 16 == 0 for t in ts)


def gemm_f32_2d(x2: torch.Tensor, w2: torch.Tensor, holder: StatsHolder | None = None,
                out: torch.Tensor | None = None, w_kn: bool = False) -> torch.Tensor | None:
    """fp32 Y = X W^T (+ ``out`` in place) on the f32-MFMA kernel (conv1x1_f32.hip), with the
    BN statistics of Y's columns when a holder wants them; None when K is not 64 / 128 / 256
    or the operands are not dense fp32 (the caller keeps its library path).  ``w_kn``: ``w2``
    is W^T, stored [K][N] (Y = X . w2)."""
    if not USE_GEMM_F32 or not x2.is_cuda or not _f32_ok(x2, w2):
        return None
    M, K = x2.shape
    Nc = w2.shape[1] if w_kn else w2.shape[0]
    h = N.hip()
    if not h.gemm_f32_stats_supported(M, Nc, K):
        return None
    if out is not None and (out.dtype != torch.float32 or not out.is_contiguous() or tuple(out.shape) != (M, Nc)):
        return None
    G = h.gemm_f32_stats_groups(M, Nc, K)
    y2 = out if out is not None else torch.empty(M, Nc, dtype=torch.float32, device=x2.device)
    ws = None
    if holder is not None:
        ws = torch.empty(max(2 * G * Nc + 3 * Nc, h.bn_workspace_floats(M, Nc)), dtype=torch.float32,
                         device=x2.device)
    h.gemm_f32_stats(x2.data_ptr(), w2.data_ptr(), y2.data_ptr(), N.ptr(ws), M, Nc, K, G, N.stream_of(x2),
                     out is not None, w_kn)
    if holder is not None:
        holder.stats = (ws, G)
    return y2


def gemm_bnstats_2d(x2: torch.Tensor, w2: torch.Tensor, holder: StatsHolder | None) -> torch.Tensor | None:
    """Y = X W^T on the MFMA kernel with the BN statistics of Y's columns (gemm_bnstats.hip,
    or conv1x1_f32.hip for fp32) when the shapes are covered and a holder wants them; else
    None."""
    if holder is None or not USE_GEMM_BNSTATS or not x2.is_cuda:
        return None
    if x2.dtype == torch.float32:
        return gemm_f32_2d(x2, w2, holder)
    M, K = x2.shape
    Nc = w2.shape[0]
    if (x2.dtype != torch.bfloat16 or w2.dtype != torch.bfloat16 or not x2.is_contiguous() or not w2.is_contiguous()
            or x2.data_ptr() % 16 or w2.data_ptr() % 16):
        return None
    h = N.hip()
    if not h.gemm_bnstats_supported(M, Nc, K):
        return None
    G = h.gemm_bnstats_groups(M, Nc, K)
    y2 = torch.empty(M, Nc, dtype=torch.bfloat16, device=x2.device)
    ws = torch.empty(max(2 * G * Nc + 3 * Nc, h.bn_workspace_floats(M, Nc)), dtype=torch.float32, device=x2.device)
    h.gemm_bnstats(x2.data_ptr(), w2.data_ptr(), y2.data_ptr(), ws.data_ptr(), M, Nc, K, G, N.stream_of(x2))
    holder.stats = (ws, G)
    return y2


def mfma_dgrad(dy2: torch.Tensor, w2: torch.Tensor, acc2: torch.Tensor | None = None) -> torch.Tensor | None:
    """dX [M, Cin] = dY [M, Cout] . W [Cout, Cin] (+ acc2 in place) on the MFMA GEMM when the
    shape is covered; None otherwise (the caller keeps its library path)."""
    if not USE_MFMA_DGRAD or not dy2.is_cuda:
        return None
    if dy2.dtype == torch.float32:
        return gemm_f32_2d(dy2, w2, None, acc2, w_kn=True)  # W [Cout][Cin] = the kernel's [K][N]
    M, K = dy2.shape
    Nc = w2.shape[1]
    if (dy2.dtype != torch.bfloat16 or w2.dtype != torch.bfloat16 or not dy2.is_contiguous()
            or dy2.data_ptr() % 16):
        return None
    if acc2 is not None and (acc2.dtype != torch.bfloat16 or not acc2.is_contiguous() or acc2.data_ptr() % 16
                             or tuple(acc2.shape) != (M, Nc)):
        return None
    h = N.hip()
    if not h.gemm_bnstats_supported(M, Nc, K):
        return None
    G = h.gemm_bnstats_groups(M, Nc, K)
    wt = w2.t().contiguous()  # [Cin][Cout]: the kernel's [N][K] operand
    out = acc2 if acc2 is not None else torch.empty(M, Nc, dtype=torch.bfloat16, device=dy2.device)
    ws = torch.empty(2 * G * Nc, dtype=torch.float32, device=dy2.device)  # statistics of dY . W: unused
    h.gemm_bnstats(dy2.data_ptr(), wt.data_ptr(), out.data_ptr(), ws.data_ptr(), M, Nc, K, G, N.stream_of(dy2),
                   acc2 is not None)
    return out


def _direct(p: torch.Tensor) -> bool:
    return flat_grad(p) is not None


def _ready(p: torch.Tensor) -> None:
    fn = getattr(p, "_voda_grad_ready", None)
    if fn is not None:
        fn(p)


def _as_2d(t: torch.Tensor) -> torch.Tensor:
    """[N, C, H, W] channels_last -> [N*H*W, C] (a view when dense channels_last)."""
    n, c, h, w = t.shape
    return t.permute(0, 2, 3, 1).reshape(n * h * w, c)


class _Conv1x1Fn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, weight, stride: int, sink_in: GradSink | None = None, sink_out: GradSink | None = None,
                holder: StatsHolder | None = None):
        """``sink_in``: accumulate the input gradient into the tensor a producer left there
        (stride 1 only); ``sink_out``: hand the input gradient to a consumer instead of
        returning it; ``holder``: receives the output's BN partial statistics when the
        statistics GEMM covers the shape."""
        xs = subsample(x, stride) if stride > 1 else x
        n, cin, h, w = xs.shape
        cout = weight.shape[0]
        x2 = _as_2d(xs)
        w2 = weight.reshape(cout, cin)
        y2 = gemm_bnstats_2d(x2, w2, holder)
        if y2 is None and x2.dtype == torch.float32:
            y2 = gemm_f32_2d(x2, w2)
        if y2 is None and (USE_SPLIT_FWD_F32 and not USE_SPLIT_GEMM_F32 and x2.dtype == torch.float32
                           and x2.shape[1] >= SPLIT_FWD_MIN_K and SG.supported(x2, w2.t())):
            y2 = SG.matmul(x2, w2.t(), variant=SPLIT_VARIANT)
        if y2 is None:
            y2 = _mm(x2, w2.t())
        ctx.save_for_backward(x2, weight)
        ctx.meta = (x.shape, stride, n, h, w)
        ctx.sink_in = sink_in if stride == 1 else None
        ctx.sink_out = sink_out
        # the previous block's bn3 backward handoff (ops/batchnorm.BwdHandoff): filled by the
        # fused input gradient below
        from .batchnorm import HANDOFF_ATTR

        ctx.handoff = getattr(x, HANDOFF_ATTR, None) if sink_in is not None else None
        return y2.view(n, h, w, cout).permute(0, 3, 1, 2)  # channels_last NCHW

    @staticmethod
    def backward(ctx, dy):
        x2, weight = ctx.saved_tensors
        in_shape, stride, n, h, w = ctx.meta
        cout, cin = weight.shape[0], weight.shape[1]
        dy2 = _as_2d(dy)
        if dy2.dtype != weight.dtype:
            dy2 = dy2.to(weight.dtype)
        if dy2.stride(1) != 1 or dy2.stride(0) != cout:
            dy2 = dy2.contiguous()
        w2 = weight.reshape(cout, cin)
        dx = None
        acc = ctx.sink_in.take() if ctx.sink_in is not None and ctx.needs_input_grad[0] else None
        from .batchnorm import MaskedGrad

        if isinstance(acc, MaskedGrad):
            dx2 = fused_dgrad_bn(dy2, w2, acc, ctx.handoff)
            if dx2 is not None:
                acc = None
                dx = dx2.view(n, h, w, cin).permute(0, 3, 1, 2)
            else:
                acc = acc.dense()
        strided = None
        if isinstance(acc, _StridedGrad):
            if tuple(acc.shape) == tuple(in_shape) and acc.g.dtype == dy2.dtype:
                strided, acc = acc, None
            else:
                acc = acc.dense()
        if acc is not None and (acc.shape != in_shape or acc.dtype != dy2.dtype
                                or not acc.is_contiguous(memory_format=torch.channels_last)):
            acc = acc.to(dy2.dtype).contiguous(memory_format=torch.channels_last)  # still owned here
        if strided is not None:
            dx2 = mfma_dgrad(dy2, w2)
            dx = (dx2 if dx2 is not None else _mm(dy2, w2)).view(n, h, w, cin).permute(0, 3, 1, 2)
            s_ = strided.stride
            subsample_add_(dx, strided.g, strided.stride)
        elif acc is not None:
            _addmm_(_as_2d(acc), dy2, w2)  # dX = shortcut gradient + dY . W (one GEMM, beta = 1)
            dx = acc
        elif dx is not None:
            pass  # the fused input gradient above
        elif ctx.needs_input_grad[0]:
            dx2 = mfma_dgrad(dy2, w2)
            dxs = (dx2 if dx2 is not None else _mm(dy2, w2)).view(n, h, w, cin).permute(0, 3, 1, 2)
            if stride > 1 and ctx.sink_out is not None and USE_STRIDED_SINK:
                dx = _StridedGrad(dxs, stride, in_shape)  # the consumer adds it in place
            elif stride > 1:
                N_, C_, H_, W_ = in_shape
                dx = dxs.new_zeros((N_, H_, W_, C_)).permute(0, 3, 1, 2)  # channels_last
                dx[:, :, ::stride, ::stride] = dxs
            else:
                dx = dxs
        dw = None
        if ctx.needs_input_grad[1]:
            g2 = flat_grad(weight).view(cout, cin) if _direct(weight) else None
            if (dy2.dtype == torch.float32 and g2 is not None and g2.dtype == torch.float32
                    and USE_SPLIT_WGRAD_F32 and SG.supported(dy2.t(), x2)):
                # split-K into the flat gradient, ~1024 workgroups over the pixels
                tile = SG.thin_tile(cout, cin) if USE_THIN_TILES else 0
                SG.matmul(dy2.t(), x2, out=g2, accumulate=True, tile=tile,
                          splits=SG.conv_wgrad_splits(cout, cin, dy2.shape[0], tile, WGRAD_TARGET_WG),
                          variant=8 if WGRAD_V8 and tile == 0 else None)
                _ready(weight)
            elif (dy2.dtype == torch.float32 and g2 is not None and g2.dtype == torch.float32
                    and blas_wgrad_f32_ok(dy2.shape[0], cout, cin)):
                g2.addmm_(dy2.t(), x2)
                _ready(weight)
            elif dy2.dtype == torch.float32:  # MIOpen's weight-only convolution backward
                xs4 = x2.view(n, h, w, cin).permute(0, 3, 1, 2)
                dy4 = dy2.view(n, h, w, cout).permute(0, 3, 1, 2)
                dw4 = torch.ops.aten.convolution_backward(dy4, xs4, weight, None, [1, 1], [0, 0], [1, 1], False,
                                                          [0, 0], 1, [False, True, False])[1]
                if g2 is not None:
                    g2.add_(dw4.view(cout, cin))
                    _ready(weight)
                else:
                    dw = dw4
            elif g2 is not None and W.supported(dy2, x2, g2):
                W.wgrad_accumulate_(dy2, x2, g2)
                _ready(weight)
            elif g2 is not None:
                if g2.dtype == dy2.dtype:
                    g2.addmm_(dy2.t(), x2)
                else:  # fp32 flat gradient of a bf16 weight (cast first: see utils/flat.FOLD_CAST)
                    g2.add_((dy2.t() @ x2).to(g2.dtype))
                _ready(weight)
            else:
                dw = (dy2.t() @ x2).view(cout, cin, 1, 1)
        if ctx.sink_out is not None and dx is not None:
            ctx.sink_out.put(dx)
            dx = None
        return dx, dw, None, None, None, None


class _Conv1x1StatsFn(torch.autograd.Function):
    """Stride-1 1x1 convolution whose forward is the statistics GEMM (gemm_bnstats.hip) and
    whose backward is MIOpen's (the Cin = 64 layers, which stay off the hipBLASLt path)."""

    @staticmethod
    def forward(ctx, x, weight, holder):
        n, cin, h, w = x.shape
        cout = weight.shape[0]
        y2 = gemm_bnstats_2d(_as_2d(x), weight.reshape(cout, cin), holder)
        ctx.save_for_backward(x, weight)
        return y2.view(n, h, w, cout).permute(0, 3, 1, 2)

    @staticmethod
    def backward(ctx, dy):
        x, weight = ctx.saved_tensors
        if not dy.is_contiguous(memory_format=torch.channels_last):
            dy = dy.contiguous(memory_format=torch.channels_last)
        mask = [bool(ctx.needs_input_grad[0]), bool(ctx.needs_input_grad[1]), False]
        dx = dw = None
        if mask[0]:  # the input gradient on the MFMA GEMM where it covers the shape
            n, cin, h, w = x.shape
            cout = weight.shape[0]
            dx2 = mfma_dgrad(_as_2d(dy), weight.reshape(cout, cin))
            if dx2 is not None:
                dx = dx2.view(n, h, w, cin).permute(0, 3, 1, 2)
                mask[0] = False
        if mask[0] or mask[1]:
            dx_m, dw, _ = torch.ops.aten.convolution_backward(dy, x, weight, None, [1, 1], [0, 0], [1, 1], False,
                                                              [0, 0], 1, mask)
            if mask[0]:
                dx = dx_m
        if mask[1]:
            g2 = flat_grad(weight) if _direct(weight) else None
            if g2 is not None:  # fold into the optimizer's flat gradient (see utils/flat.FOLD_CAST)
                g2.add_(dw.to(g2.dtype) if FOLD_CAST else dw)
                _ready(weight)
                dw = None
        return dx, dw, None


def _attach(y: torch.Tensor, holder: StatsHolder | None) -> torch.Tensor:
    if holder is not None and holder.stats is not None:
        from .batchnorm import attach_stats

        attach_stats(y, *holder.stats)
    return y


class Conv1x1(torch.nn.Conv2d):
    """``nn.Conv2d(cin, cout, 1, stride, bias=False)`` with the GEMM formulation on GPU."""

    def __init__(self, in_channels: int, out_channels: int, stride: int = 1, **kw):
        super().__init__(in_channels, out_channels, 1, stride=stride, bias=False, **kw)

    def _gemm_ok(self, x: torch.Tensor) -> bool:
        if x.is_cuda and x.dtype == torch.float32:
            return (USE_CONV1X1_F32 and x.dim() == 4 and self.weight.dtype == torch.float32 and self.groups == 1
                    and self.padding == (0, 0) and self.dilation == (1, 1) and self.stride[0] == self.stride[1]
                    and x.is_contiguous(memory_format=torch.channels_last)
                    and self.in_channels % 32 == 0 and self.out_channels % 32 == 0)
        return (USE_CONV1X1_GEMM and x.is_cuda and x.dim() == 4 and x.dtype == torch.bfloat16
                and self.weight.dtype == torch.bfloat16 and self.groups == 1 and self.padding == (0, 0)
                and self.dilation == (1, 1) and self.stride[0] == self.stride[1]
                and x.is_contiguous(memory_format=torch.channels_last)
                and self.in_channels >= 128 and self.in_channels % 8 == 0 and self.out_channels % 8 == 0)

    def _stats_ok(self, x: torch.Tensor) -> bool:
        """The output feeds a training-mode BN and the statistics GEMM covers the layer
        (K = 64 / 128 / 256 input channels, channels_last bf16)."""
        if (USE_GEMM_F32 and USE_GEMM_BNSTATS and self.training and torch.is_grad_enabled() and x.is_cuda
                and x.dim() == 4 and x.dtype == torch.float32 and self.weight.dtype == torch.float32
                and self.in_channels in (64, 128, 256) and self.groups == 1 and self.padding == (0, 0)
                and self.dilation == (1, 1) and x.is_contiguous(memory_format=torch.channels_last)):
            s = self.stride[0]
            m = x.shape[0] * ((x.shape[2] + s - 1) // s) * ((x.shape[3] + s - 1) // s)
            return bool(N.hip().gemm_f32_stats_supported(m, self.out_channels, self.in_channels))
        if not (USE_GEMM_BNSTATS and self.training and torch.is_grad_enabled() and x.is_cuda and x.dim() == 4
                and x.dtype == torch.bfloat16 and self.weight.dtype == torch.bfloat16
                and self.in_channels in (64, 128, 256) and self.groups == 1 and self.padding == (0, 0)
                and self.dilation == (1, 1) and x.is_contiguous(memory_format=torch.channels_last)
                and self.weight.is_contiguous()):
            return False
        s = self.stride[0]
        m = x.shape[0] * ((x.shape[2] + s - 1) // s) * ((x.shape[3] + s - 1) // s)
        return bool(N.hip().gemm_bnstats_supported(m, self.out_channels, self.in_channels))

    def forward(self, x, sink_in: GradSink | None = None, sink_out: GradSink | None = None):
        """``sink_in`` / ``sink_out``: see GradSink.  A caller passes ``sink_in`` only after
        checking ``_gemm_ok(x)`` (the consumer must run on this path); ``sink_out`` is
        ignored on the fallback paths (the gradient is then returned normally)."""
        if x.is_cuda and x.dtype != self.weight.dtype and torch.is_autocast_enabled("cuda"):
            x = x.to(self.weight.dtype)
        holder = StatsHolder() if self._stats_ok(x) else None
        if self._gemm_ok(x):
            with torch.autocast("cuda", enabled=False):
                y = _Conv1x1Fn.apply(x, self.weight, self.stride[0], sink_in, sink_out, holder)
            return _attach(y, holder)
        assert sink_in is None, "a GradSink consumer must run on the GEMM path"
        if holder is not None and self.stride == (1, 1) and self.in_channels == 64:
            with torch.autocast("cuda", enabled=False):
                y = _Conv1x1StatsFn.apply(x, self.weight, holder)
            return _attach(y, holder)
        return super().forward(x)
