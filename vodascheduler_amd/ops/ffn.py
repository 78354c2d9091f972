"""Transformer feed-forward block ``fc2(gelu_tanh(fc1(x)))`` with the GELU fused into the
hipBLASLt GEMM epilogues (csrc/hip/blaslt_epi.cpp):

    forward   h, y = X W1^T + b1, gelu(h)      one GEMM, GELU_AUX_BIAS epilogue (h kept)
              out  = y W2^T + b2               hipBLASLt
    backward  fc2 weight / bias gradients      into the flat gradients (ops/dense.py)
              dh   = (dOut W2) * gelu'(h)      one GEMM, DGELU epilogue
              fc1 weight / bias gradients      into the flat gradients
              dX   = dh W1 (+ residual-stream gradient, beta = 1, ops/conv1x1.GradSink)

instead of fc1 GEMM + GELU kernel and fc2 input-gradient GEMM + GELU-backward kernel (two
launches and ~300 MB of fp32 activation traffic per BERT-base layer).  On gfx950 with ROCm 7.2
hipBLASLt has both epilogues for fp32 operands and neither for bf16
(profiles/r5/blaslt_epilogue_probe_fp32.jsonl, profiles/raw/r2_blaslt_epilogue_probe.jsonl), so
this is the reference-precision (fp32) FFN path; a one-time capability probe per (device, dtype)
decides, and bf16 keeps the HIP GELU kernels.  Same parameters / state dict as two
``FusedLinear`` layers.  Reference: the Keras Transformer FFN of
examples/py/tensorflow2/neural_machine_translation_with_transformer.py (dense -> activation ->
dense), BERT's GELU FFN.
"""
from __future__ import annotations

import math
import os

import torch
import torch.nn.functional as F

from . import _native as N
from . import dense as D
from . import splitgemm as SG

# VODA_GELU_EPILOGUE=0: the FFN runs FusedLinear -> GELU kernel -> FusedLinear (A/B switch)
USE_GELU_EPILOGUE = os.environ.get("VODA_GELU_EPILOGUE", "1") != "0"

EPI_GELU_AUX_BIAS, EPI_DGELU = 164, 192  # hipblasLtEpilogue_t values
_WS_BYTES = 32 << 20
_WS: dict[torch.device, torch.Tensor] = {}
_EPI_OK: dict[tuple[int, torch.dtype], bool] = {}
_SHAPE_OK: dict[tuple[int, torch.dtype, int, int, int], bool] = {}


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
        h = F.linear(x2, w, b.to(w.dtype))
        return h, gelu_tanh_ref(h)
    for t, nm in ((x2, "x"), (w, "w")):
        N.check_gpu_tensor(t, nm, align=16)
    bb = b.to(x2.dtype).contiguous()
    h = torch.empty(M, Nn, dtype=x2.dtype, device=x2.device)
    y = torch.empty_like(h)
    ws = _workspace(x2.device)
    N.hip().gemm_gelu_aux(x2.data_ptr(), w.data_ptr(), bb.data_ptr(), h.data_ptr(), y.data_ptr(), M, Nn, K,
                          N.dtype_code(x2.dtype), ws.data_ptr(), ws.numel(), N.stream_of(x2))
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
    N.hip().gemm_dgelu(dy2.data_ptr(), w.data_ptr(), h.data_ptr(), dh.data_ptr(), M, Nn, K, N.dtype_code(dy2.dtype),
                       ws.data_ptr(), ws.numel(), N.stream_of(dy2))
    return dh


class _FFNGeluFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, w1, b1, w2, b2, sink_in=None, bias_handoff=None):
        """``sink_in`` (ops/conv1x1.GradSink): dX accumulates into the residual-stream gradient a
        producer left there; ``bias_handoff`` (ops/dense.BiasHandoff): fc2's bias gradient may
        come from the next op's backward (the post-LN LayerNorm)."""
        d = x.shape[-1]
        x2 = x.reshape(-1, d)
        if not x2.is_contiguous():
            x2 = x2.contiguous()
        with torch.autocast(x.device.type, enabled=False):
            ctx.split = _split_ok(x2, w1, w2)
            if ctx.split:  # fp32: split-bf16 MFMA GEMMs with the GELU in their epilogues
                h = torch.empty(x2.shape[0], w1.shape[0], dtype=torch.float32, device=x2.device)
                y = SG.matmul(x2, w1.t(), bias=b1, epi=SG.EPI_GELU, aux=h)
                out = SG.matmul(y, w2.t(), bias=b2)
            else:
                h, y = gemm_gelu_aux(x2, w1, b1)
                out = F.linear(y, w2, b2.to(w2.dtype))
        ctx.save_for_backward(x2, w1, w2, h, y)
        ctx.biases = (b1, b2)
        ctx.sink_in = sink_in
        ctx.bias_handoff = bias_handoff
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
        need_b2 = need[4]
        hb = ctx.bias_handoff
        if need_b2 and hb is not None and hb.done:
            need_b2 = False  # summed into the flat gradient by the LayerNorm backward
            hb.done = False
        dw2, db2 = D.linear_weight_grads(do2, y, w2, b2, need[3], need_b2)
        if ctx.split and SG.supported(do2, w2):
            dh = SG.matmul(do2, w2, epi=SG.EPI_DGELU, aux=h)
        else:
            try:
                dh = gemm_dgelu(do2, w2, h)
            except RuntimeError as e:  # no DGELU kernel after all: unfused, same math
                disable_epilogue(str(e))
                g = do2 @ w2
                dh = (g.float() * gelu_tanh_grad_ref(h)).to(do2.dtype)
        dw1, db1 = D.linear_weight_grads(dh, x2, w1, b1, need[1], need[2])
        dx = None
        acc = ctx.sink_in.take() if ctx.sink_in is not None and need[0] else None
        if acc is not None:
            if acc.shape != ctx.x_shape or acc.dtype != dh.dtype or not acc.is_contiguous():
                acc = acc.to(dh.dtype).contiguous()
            if SG.supported(dh, w1):
                SG.matmul(dh, w1, out=acc.view(-1, w1.shape[1]), accumulate=True)
            else:
                acc.view(-1, w1.shape[1]).addmm_(dh, w1)  # residual-stream gradient + dh . W1
            dx = acc
        elif need[0]:
            dx = D._dgrad(dh, w1).view(ctx.x_shape)
        return dx, dw1, db1, dw2, db2, None, None


def disable_epilogue(reason: str) -> None:
    """Fall back to the unfused FFN for the rest of the process; said once on stderr."""
    global USE_GELU_EPILOGUE
    if USE_GELU_EPILOGUE:
        import sys

        print(f"[vodascheduler_amd] GELU-epilogue GEMM unavailable, unfused FFN from now on: {reason}",
              file=sys.stderr, flush=True)
    USE_GELU_EPILOGUE = False


def epilogues_available(device: torch.device, dtype: torch.dtype = torch.float32) -> bool:
    """Does this GPU's hipBLASLt ship kernels of ``dtype`` for BOTH epilogues?  Probed once per
    (device, dtype) by a heuristic query (no launch): on gfx950 / ROCm 7.2 fp32 yes, bf16 no."""
    if dtype not in (torch.float32, torch.bfloat16):
        return False
    idx = device.index if device.index is not None else torch.cuda.current_device()
    ok = _EPI_OK.get((idx, dtype))
    if ok is None:
        h = N.hip()
        dt = N.dtype_code(dtype)
        with torch.cuda.device(idx):
            ok = (h.gemm_epilogue_algos(EPI_GELU_AUX_BIAS, dt, True, 3072, 8192, 768) > 0
                  and h.gemm_epilogue_algos(EPI_DGELU, dt, False, 3072, 8192, 768) > 0)
        _EPI_OK[(idx, dtype)] = ok
    return ok


def shape_available(device: torch.device, dtype: torch.dtype, M: int, d_model: int, d_ff: int) -> bool:
    """Does hipBLASLt have kernels for BOTH epilogue GEMMs of THIS token count?  The forward
    (GELU_AUX_BIAS, h [M, d_ff] = X W1^T) and the backward's DGELU GEMM (dh [M, d_ff] = dOut W2)
    are queried for the real (M, N, K) before the fused path is taken, so a shape with a forward
    kernel but no DGELU kernel never reaches the backward (cached per shape, no launch)."""
    idx = device.index if device.index is not None else torch.cuda.current_device()
    key = (idx, dtype, M, d_model, d_ff)
    ok = _SHAPE_OK.get(key)
    if ok is None:
        h = N.hip()
        dt = N.dtype_code(dtype)
        with torch.cuda.device(idx):
            ok = (h.gemm_epilogue_algos(EPI_GELU_AUX_BIAS, dt, True, d_ff, M, d_model) > 0
                  and h.gemm_epilogue_algos(EPI_DGELU, dt, False, d_ff, M, d_model) > 0)
        _SHAPE_OK[key] = ok
    return ok


def _split_ok(x2: torch.Tensor, w1: torch.Tensor, w2: torch.Tensor) -> bool:
    """Both FFN GEMMs on the split-bf16 kernel: fp32 operands of supported shapes."""
    M, d = x2.shape
    return (SG.supported(x2, w1.t()) and w2.shape[1] == w1.shape[0] and w1.shape[0] % 16 == 0
            and w2.shape[0] % 4 == 0 and w2.dtype == torch.float32 and w2.is_contiguous())


def supported(x: torch.Tensor, w1: torch.Tensor, b1, w2: torch.Tensor, b2) -> bool:
    dt = w1.dtype
    if (USE_GELU_EPILOGUE and b1 is not None and b2 is not None and x.is_cuda and x.dtype == dt == w2.dtype == torch.float32
            and w1.is_contiguous() and w2.is_contiguous() and x.shape[-1] % 16 == 0 and x.is_contiguous()
            and _split_ok(x.reshape(-1, x.shape[-1]), w1, w2)):
        return True  # split-bf16 path: needs no hipBLASLt epilogue kernels
    if not (USE_GELU_EPILOGUE and x.is_cuda and x.dtype == dt and w2.dtype == dt and b1 is not None
            and b2 is not None and w1.is_contiguous() and w2.is_contiguous() and x.shape[-1] % 8 == 0
            and w1.shape[0] % 8 == 0 and w2.shape[0] % 8 == 0 and epilogues_available(x.device, dt)):
        return False
    M = x.numel() // x.shape[-1]
    return M > 0 and shape_available(x.device, dt, M, x.shape[-1], w1.shape[0])


def ffn_gelu(x: torch.Tensor, w1: torch.Tensor, b1: torch.Tensor, w2: torch.Tensor, b2: torch.Tensor,
             sink_in=None, bias_handoff=None) -> torch.Tensor:
    """``fc2(gelu_tanh(fc1(x)))`` on the epilogue-fused path (callers check ``supported``)."""
    return _FFNGeluFn.apply(x, w1, b1, w2, b2, sink_in, bias_handoff)
