"""Transformer feed-forward block ``fc2(gelu_tanh(fc1(x)))`` with the GELU fused into the
hipBLASLt GEMM epilogues (csrc/hip/blaslt_epi.cpp), when the installed hipBLASLt has kernels
for them (``epilogues_available``; NOT the case on gfx950 / ROCm 7.x, where the FFN keeps the
HIP GELU kernels of ops/activation.py):

    forward   h, y = X W1^T + b1, gelu(h)      one GEMM, GELU_AUX_BIAS epilogue (h kept)
              out  = y W2^T + b2               hipBLASLt
    backward  fc2 weight / bias gradients      split-K MFMA kernel into the flat gradient
              dh   = (dOut W2) * gelu'(h)      one GEMM, DGELU epilogue
              fc1 weight / bias gradients      split-K MFMA kernel
              dX   = dh W1 (+ residual-stream gradient, beta = 1, ops/conv1x1.GradSink)

instead of fc1 GEMM + GELU kernel and fc2 input-gradient GEMM + GELU-backward kernel (two
launches and ~150 MB of activation traffic per BERT-base layer).  Same parameters / state
dict as two ``FusedLinear`` layers; numerics: GELU in fp32 registers on the fp32 GEMM
accumulator, h / y / dh rounded once to bf16.  Used by ``models/layers.FeedForward`` (act =
"gelu") on GPU bf16 tensors; everything else runs the unfused composition.
"""
from __future__ import annotations

import math
import os

import torch
import torch.nn.functional as F

from . import _native as N
from .dense import _dgrad, linear_weight_grads

# VODA_GELU_EPILOGUE=0: the FFN runs FusedLinear -> GELU kernel -> FusedLinear (A/B switch)
USE_GELU_EPILOGUE = os.environ.get("VODA_GELU_EPILOGUE", "1") != "0"

_WS_BYTES = 32 << 20
_WS: dict[torch.device, torch.Tensor] = {}


def _workspace(device: torch.device) -> torch.Tensor:
    w = _WS.get(device)
    if w is None:
        w = _WS[device] = torch.empty(_WS_BYTES, dtype=torch.uint8, device=device)
    return w


def gelu_tanh_ref(h: torch.Tensor) -> torch.Tensor:
    return F.gelu(h, approximate="tanh")


def gelu_tanh_grad_ref(h: torch.Tensor) -> torch.Tensor:
    """d gelu_tanh / dh (fp32, or fp64 for fp64 input)."""
    h = h if h.dtype == torch.float64 else h.float()
    c = math.sqrt(2.0 / math.pi)
    u = c * (h + 0.044715 * h ** 3)
    t = torch.tanh(u)
    return 0.5 * (1 + t) + 0.5 * h * (1 - t * t) * c * (1 + 3 * 0.044715 * h * h)


def gemm_gelu_aux(x2: torch.Tensor, w: torch.Tensor, b: torch.Tensor) -> tuple[torch.Tensor, torch.Tensor]:
    """(h, y) = (x2 W^T + b, gelu_tanh(h)); x2 [M, K], w [N, K], b [N]."""
    M, K = x2.shape
    Nn = w.shape[0]
    if not x2.is_cuda:
        h = F.linear(x2, w, b)
        return h, gelu_tanh_ref(h)
    for t, nm in ((x2, "x"), (w, "w")):
        N.check_gpu_tensor(t, nm, align=16)
    bb = b.to(x2.dtype).contiguous()
    h = torch.empty(M, Nn, dtype=x2.dtype, device=x2.device)
    y = torch.empty_like(h)
    ws = _workspace(x2.device)
    N.hip().gemm_gelu_aux(x2.data_ptr(), w.data_ptr(), bb.data_ptr(), h.data_ptr(), y.data_ptr(), M, Nn, K,
                          ws.data_ptr(), ws.numel(), N.stream_of(x2))
    return h, y


def gemm_dgelu(dy2: torch.Tensor, w: torch.Tensor, h: torch.Tensor) -> torch.Tensor:
    """dh = (dy2 W) * gelu_tanh'(h); dy2 [M, N], w [N, K], h [M, K]."""
    M, Nn = dy2.shape
    K = w.shape[1]
    if not dy2.is_cuda:
        g = dy2 @ w
        return (g.to(torch.promote_types(g.dtype, torch.float32)) * gelu_tanh_grad_ref(h)).to(dy2.dtype)
    for t, nm in ((dy2, "dy"), (w, "w"), (h, "h")):
        N.check_gpu_tensor(t, nm, align=16)
    dh = torch.empty(M, K, dtype=dy2.dtype, device=dy2.device)
    ws = _workspace(dy2.device)
    N.hip().gemm_dgelu(dy2.data_ptr(), w.data_ptr(), h.data_ptr(), dh.data_ptr(), M, Nn, K, ws.data_ptr(),
                       ws.numel(), N.stream_of(dy2))
    return dh


class _FFNGeluFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, w1, b1, w2, b2, sink_in=None):
        d = x.shape[-1]
        x2 = x.reshape(-1, d)
        if not x2.is_contiguous():
            x2 = x2.contiguous()
        with torch.autocast(x.device.type, enabled=False):
            h, y = gemm_gelu_aux(x2, w1, b1)
            out = F.linear(y, w2, b2.to(w2.dtype))
        ctx.save_for_backward(x2, w1, w2, h, y)
        ctx.biases = (b1, b2)
        ctx.sink_in = sink_in
        ctx.x_shape = x.shape
        return out.view(*x.shape[:-1], w2.shape[0])

    @staticmethod
    def backward(ctx, dout):
        x2, w1, w2, h, y = ctx.saved_tensors
        b1, b2 = ctx.biases
        do2 = dout.reshape(-1, w2.shape[0])
        if do2.dtype != w2.dtype:
            do2 = do2.to(w2.dtype)
        if not do2.is_contiguous():
            do2 = do2.contiguous()
        need = ctx.needs_input_grad
        dw2, db2 = linear_weight_grads(do2, y, w2, b2, need[3], need[4])
        dh = gemm_dgelu(do2, w2, h)
        dw1, db1 = linear_weight_grads(dh, x2, w1, b1, need[1], need[2])
        dx = None
        acc = ctx.sink_in.take() if ctx.sink_in is not None and need[0] else None
        if acc is not None:
            if acc.shape != ctx.x_shape or acc.dtype != dh.dtype or not acc.is_contiguous():
                acc = acc.to(dh.dtype).contiguous()
            acc.view(-1, w1.shape[1]).addmm_(dh, w1)  # residual-stream gradient + dh . W1
            dx = acc
        elif need[0]:
            dx = _dgrad(dh, w1).view(ctx.x_shape)
        return dx, dw1, db1, dw2, db2, None


def disable_epilogue(reason: str) -> None:
    """Fall back to the unfused FFN for the rest of the process (hipBLASLt found no epilogue
    kernel); said once on stderr."""
    global USE_GELU_EPILOGUE
    if USE_GELU_EPILOGUE:
        import sys

        print(f"[vodascheduler_amd] GELU-epilogue GEMM unavailable, unfused FFN from now on: {reason}",
              file=sys.stderr, flush=True)
    USE_GELU_EPILOGUE = False


_EPI_OK: dict[int, bool] = {}
EPI_GELU_AUX_BIAS, EPI_DGELU = 164, 192  # hipblasLtEpilogue_t values


def epilogues_available(device: torch.device) -> bool:
    """Does this GPU's hipBLASLt ship bf16 kernels for BOTH epilogues?  Probed once per device
    (heuristic query, no launch).  On gfx950 with ROCm 7.x it does not: GELU / GELU_BIAS have
    kernels, GELU_AUX(_BIAS) / DGELU return no algorithm (profiles/raw/r2_blaslt_epilogue_probe.jsonl,
    benchmarks/blaslt_epilogue_probe.py), so the FFN keeps the HIP GELU kernels there."""
    idx = device.index if device.index is not None else torch.cuda.current_device()
    ok = _EPI_OK.get(idx)
    if ok is None:
        h = N.hip()
        with torch.cuda.device(idx):
            ok = (h.gemm_epilogue_algos(EPI_GELU_AUX_BIAS, True, 3072, 8192, 768) > 0
                  and h.gemm_epilogue_algos(EPI_DGELU, False, 3072, 8192, 768) > 0)
        _EPI_OK[idx] = ok
    return ok


def supported(x: torch.Tensor, w1: torch.Tensor, b1, w2: torch.Tensor, b2) -> bool:
    return (USE_GELU_EPILOGUE and x.is_cuda and epilogues_available(x.device) and x.dtype == torch.bfloat16 and w1.dtype == torch.bfloat16
            and w2.dtype == torch.bfloat16 and b1 is not None and b2 is not None
            and w1.is_contiguous() and w2.is_contiguous() and x.shape[-1] % 8 == 0 and w1.shape[0] % 8 == 0
            and w2.shape[0] % 8 == 0)


def ffn_gelu(x: torch.Tensor, w1: torch.Tensor, b1: torch.Tensor, w2: torch.Tensor, b2: torch.Tensor,
             sink_in=None) -> torch.Tensor:
    """``fc2(gelu_tanh(fc1(x)))`` on the epilogue-fused path (callers check ``supported``)."""
    return _FFNGeluFn.apply(x, w1, b1, w2, b2, sink_in)
