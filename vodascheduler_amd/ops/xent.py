"""Fused softmax cross-entropy for vocab-sized classifier heads (csrc/hip/xent.hip).

``softmax_cross_entropy(logits, labels, num_classes, ignore_index)`` returns ``(loss, correct,
n_valid)`` as device tensors: the mean loss over the rows whose label is not ``ignore_index``
(``F.cross_entropy(logits[:, :num_classes].float(), labels, ignore_index=...)``), the number
of those rows whose first-maximum class equals the label (the accuracy metric of the
reference's Keras ``metrics=["accuracy"]`` / masked accuracy), and their count.

On MI355X the stock chain -- ``logits.float()``, ``log_softmax``, ``nll_loss``, ``argmax`` and
the same backwards -- moves the [rows, vocab] logits through HBM about eight times in fp32
(BERT-base MLM head 1280 x 30522, NMT head 10240 x 15000; profiles/r2_rocprof_bert_final.md).
The HIP kernels read the bf16 logits once forward, once backward and write the bf16 gradient
once.  ``num_classes`` may be smaller than the logits' row length: the extra columns are the
padding of a vocab rounded up to a 16-byte row (models/transformer.py), excluded from the
softmax and given zero gradient.  Everything stays on the device (no host sync), so the op
is hipGraph-capturable.  A loss with every row ignored is 0 here (PyTorch: NaN).
"""
from __future__ import annotations

import os

import torch
import torch.nn.functional as F

from . import _native as N

USE_FUSED_XENT = True
# host-synchronising check that every label lies in [0, V) or is ignore_index (debug only)
DEBUG_LABELS = os.environ.get("VODA_DEBUG_LABELS", "0") == "1"


def _supported(logits: torch.Tensor, labels: torch.Tensor, num_classes: int) -> bool:
    if not (logits.is_cuda and labels.is_cuda) or logits.dim() != 2 or logits.dtype not in (torch.bfloat16,
                                                                                          torch.float32):
        return False
    vec = 8 if logits.dtype == torch.bfloat16 else 4
    return (logits.stride(1) == 1 and logits.stride(0) % vec == 0 and logits.data_ptr() % 16 == 0
            and num_classes <= logits.shape[1] and logits.shape[0] > 0 and labels.dtype == torch.int64
            and labels.numel() == logits.shape[0] and labels.is_contiguous())


def xent_ref(logits: torch.Tensor, labels: torch.Tensor, num_classes: int | None = None,
             ignore_index: int = -100) -> tuple[torch.Tensor, torch.Tensor, torch.Tensor]:
    """PyTorch (fp32) reference of :func:`softmax_cross_entropy`."""
    V = logits.shape[1] if num_classes is None else num_classes
    x = logits[:, :V].float()
    valid = labels != ignore_index
    n = valid.sum()
    loss = F.cross_entropy(x, labels, ignore_index=ignore_index, reduction="sum") / n.clamp(min=1).float()
    correct = ((x.argmax(1) == labels) & valid).sum()
    return loss, correct, n


class _XentFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, logits, labels, V, ignore_index):
        R, ld = logits.shape[0], logits.stride(0)
        h = N.hip()
        f32 = dict(dtype=torch.float32, device=logits.device)
        lse, rl, rc = torch.empty(R, **f32), torch.empty(R, **f32), torch.empty(R, **f32)
        h.xent_fwd(logits.data_ptr(), R, ld, V, N.dtype_code(logits.dtype), labels.data_ptr(), ignore_index,
                   lse.data_ptr(), rl.data_ptr(), rc.data_ptr(), N.stream_of(logits))
        # the kernel's validity predicate (xent.hip): ignore_index rows AND labels outside
        # [0, V) carry no loss / gradient, so neither counts toward the mean
        n = ((labels != ignore_index) & (labels >= 0) & (labels < V)).sum()
        if DEBUG_LABELS and bool((((labels < 0) | (labels >= V)) & (labels != ignore_index)).any()):
            raise ValueError(f"softmax_cross_entropy: label outside [0, {V}) (F.cross_entropy would raise)")
        nf = n.clamp(min=1).float()
        loss = rl.sum() / nf
        correct = rc.sum()
        ctx.save_for_backward(logits, labels, lse, nf)
        ctx.V, ctx.ignore = V, ignore_index
        ctx.mark_non_differentiable(correct, n)
        return loss, correct, n

    @staticmethod
    def backward(ctx, gloss, _gc, _gn):
        logits, labels, lse, nf = ctx.saved_tensors
        scale = (gloss.float() / nf).reshape(1).contiguous()
        R, ld = logits.shape[0], logits.stride(0)
        dx = torch.empty((R, ld), dtype=logits.dtype, device=logits.device)  # padding columns get zeros
        N.hip().xent_bwd(logits.data_ptr(), dx.data_ptr(), R, ld, ctx.V, N.dtype_code(logits.dtype),
                         labels.data_ptr(), ctx.ignore, lse.data_ptr(), scale.data_ptr(), N.stream_of(logits))
        return dx[:, :logits.shape[1]], None, None, None


def softmax_cross_entropy(logits: torch.Tensor, labels: torch.Tensor, num_classes: int | None = None,
                          ignore_index: int = -100) -> tuple[torch.Tensor, torch.Tensor, torch.Tensor]:
    """Mean cross-entropy over the first ``num_classes`` columns of ``logits`` [rows, >=V]
    (fp32 math), plus the #correct and #valid rows; see the module docstring."""
    V = logits.shape[1] if num_classes is None else int(num_classes)
    labels = labels.reshape(-1)
    if logits.dim() != 2:
        logits = logits.reshape(-1, logits.shape[-1])
    if USE_FUSED_XENT and logits.is_cuda:
        if logits.stride(1) != 1:  # a row-padded view (unit column stride) is used as it is
            logits = logits.contiguous()
        if labels.dtype != torch.int64 or not labels.is_contiguous():
            labels = labels.to(torch.int64).contiguous()
        if _supported(logits, labels, V):
            return _XentFn.apply(logits, labels, V, int(ignore_index))
    return xent_ref(logits, labels, V, ignore_index)
