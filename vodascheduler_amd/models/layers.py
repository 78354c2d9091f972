"""Transformer building blocks on the framework's fused ops.

``MultiHeadAttention`` mirrors the vendored Keras MultiHeadAttention of the reference's
Transformer workload (reference examples/py/tensorflow2/layers_tf25.py:123-470: einsum
projections to [B, T, H, key_dim], scores scaled by 1/sqrt(key_dim), masked softmax with the
additive -1e9, dropout, weighted sum, output projection).  Projections / score GEMMs run on
hipBLASLt (bf16 MFMA); the masked softmax is the hand-written HIP kernel, and on GPU
the whole score->softmax->PV chain uses the fused MFMA attention kernel when the head
dimension is supported.  LayerNorm is the HIP FusedLayerNorm.
"""
from __future__ import annotations

import math
import os

import torch
from torch import nn

from ..ops import ffn as _ffn
from ..ops.activation import GeluTanh
from ..ops.attention import attention_q_kvpacked, attention_qkvpacked
from ..ops.conv1x1 import USE_GRAD_SINK, GradSink
from ..ops.dense import BiasHandoff, FusedLinear, residual_add
from ..ops.layernorm import FusedLayerNorm

# residual add of each post-LN sublayer fused into the LayerNorm kernel (FUSED_RESIDUAL_LN = False:
# a separate add, for A/B runs)
FUSED_RESIDUAL_LN = True
# FFN GELU on the HIP kernel (ops/activation.py; HIP_GELU = False: PyTorch's)
HIP_GELU = True
# a post-LN sublayer's output-projection bias gradient summed by the LayerNorm backward
# (ops/dense.BiasHandoff; BIAS_HANDOFF = False: the projection's own column-sum pass)
BIAS_HANDOFF = True


class MultiHeadAttention(nn.Module):
    def __init__(self, d_model: int, num_heads: int, key_dim: int | None = None, dropout: float = 0.0,
                 bias: bool = True, cross: bool = False):
        super().__init__()
        self.h = num_heads
        self.dk = key_dim or d_model // num_heads
        inner = self.h * self.dk
        # Self-attention: Q, K and V projections as ONE [d_model -> 3*inner] GEMM; the
        # weight-gradient GEMMs (K = batch*tokens) of 768x768 outputs tile only 36 128x128
        # blocks on 256 CUs and ran at ~190 TFLOP/s on MI355X (profiles/), the fused 2304-wide
        # one is 3x the tiles.  Cross-attention (``cross=True``): a Q projection of the query
        # stream and ONE [d_model -> 2*inner] K/V projection of the memory, each its own
        # FusedLinear, so both gradients go straight into the flat fp32 buffers (an earlier
        # version sliced one packed weight and let autograd assemble the slice gradients).
        # The fused weights are the concatenation of Keras/PyTorch's separate q/k/v kernels.
        self.cross = cross
        if cross:
            self.q = FusedLinear(d_model, inner, bias=bias)
            self.kv = FusedLinear(d_model, 2 * inner, bias=bias)
        else:
            self.qkv = FusedLinear(d_model, 3 * inner, bias=bias)
        self.o = FusedLinear(inner, d_model, bias=bias)
        self.inner = inner
        self.dropout = dropout

    def forward(self, x: torch.Tensor, kv: torch.Tensor | None = None, key_mask: torch.Tensor | None = None,
                causal: bool = False, sink_in=None, bias_handoff=None) -> torch.Tensor:
        """x: [B, Tq, D]; kv: [B, Tk, D] (default x); key_mask: [B, Tk] (nonzero = attend);
        sink_in: GradSink of the residual stream x (self-attention only); bias_handoff: the
        output projection's bias gradient comes from the next op (ops/dense.BiasHandoff)."""
        B, Tq, _ = x.shape
        E = self.inner
        drop = self.dropout if self.training else 0.0
        scale = 1.0 / math.sqrt(self.dk)
        if kv is None:
            qkv = self.qkv(x, sink_in).view(B, Tq, 3, self.h, self.dk)
            o = attention_qkvpacked(qkv, key_mask, causal, scale, drop)
        else:
            if not self.cross:
                raise ValueError("kv given to a self-attention module (build it with cross=True)")
            Tk = kv.shape[1]
            q = self.q(x).view(B, Tq, self.h, self.dk)
            kvp = self.kv(kv).view(B, Tk, 2, self.h, self.dk)
            o = attention_q_kvpacked(q, kvp, key_mask, causal, scale, drop)
        return self.o(o.reshape(B, Tq, E), bias_handoff=bias_handoff)


class FeedForward(nn.Module):
    def __init__(self, d_model: int, d_ff: int, act: str = "relu"):
        super().__init__()
        self.fc1 = FusedLinear(d_model, d_ff)
        self.fc2 = FusedLinear(d_ff, d_model)
        if act == "gelu":
            self.act = GeluTanh() if HIP_GELU else nn.GELU(approximate="tanh")
        else:
            self.act = nn.ReLU()

    def forward(self, x, sink_in=None, bias_handoff=None):
        if isinstance(self.act, GeluTanh) and x.is_cuda:
            if x.dtype != self.fc1.weight.dtype and torch.is_autocast_enabled("cuda"):
                x = x.to(self.fc1.weight.dtype)
            if _ffn.supported(x, self.fc1.weight, self.fc1.bias, self.fc2.weight, self.fc2.bias):
                # fp32: GELU in the hipBLASLt GEMM epilogues (ops/ffn.py), no GELU kernels
                try:
                    return _ffn.ffn_gelu(x, self.fc1.weight, self.fc1.bias, self.fc2.weight, self.fc2.bias,
                                         sink_in, bias_handoff)
                except (RuntimeError, ValueError) as e:  # no epilogue kernel for this shape
                    _ffn.disable_epilogue(repr(e))
        # Otherwise (bf16: hipBLASLt on gfx950 has no GELU_AUX / DGELU bf16 kernels, probe:
        # profiles/raw/r2_blaslt_epilogue_probe.jsonl) GELU runs as the HIP activation kernels.
        # fc1's bias gradient stays a column-sum pass: folding it into a row-mapped GELU
        # backward (gelu_tanh_bwd_colsum) measured 72-94 us vs 69 us for the flat GELU kernel +
        # column sum (BERT-base fp32, profiles/r5/gelu_colsum.jsonl; the fused kernel was removed).
        # fc2's comes from the next LayerNorm's backward when the caller hands over ``bias_handoff``
        return self.fc2(self.act(self.fc1(x, sink_in)), bias_handoff=bias_handoff)


def _sink(module: nn.Module, x: torch.Tensor) -> GradSink | None:
    return GradSink() if (USE_GRAD_SINK and module.training and torch.is_grad_enabled()
                          and x.requires_grad) else None


class EncoderLayer(nn.Module):
    """Post-LN encoder block (Keras TransformerEncoder / BERT layout)."""

    def __init__(self, d_model, heads, d_ff, key_dim=None, act="relu", dropout=0.0, eps=1e-5):
        super().__init__()
        self.attn = MultiHeadAttention(d_model, heads, key_dim, dropout)
        self.ln1 = FusedLayerNorm(d_model, eps=eps)
        self.ff = FeedForward(d_model, d_ff, act)
        self.ln2 = FusedLayerNorm(d_model, eps=eps)
        self.drop = nn.Dropout(dropout)

    def forward(self, x, key_mask=None):
        # the residual stream x feeds the sublayer's first GEMM and the residual add: its
        # gradient from the add is accumulated by that GEMM's input-gradient GEMM (beta = 1)
        # instead of by a separate autograd add (ops/conv1x1.GradSink)
        # the add itself runs inside the LayerNorm kernel (FusedLayerNorm(x, residual=...))
        s1 = _sink(self, x)
        if FUSED_RESIDUAL_LN and BIAS_HANDOFF and (self.drop.p == 0 or not self.training):
            # no dropout between the sublayer's last projection and the LayerNorm: the
            # LayerNorm backward sums that projection's bias gradient (ops/dense.BiasHandoff)
            h1 = BiasHandoff(self.attn.o.bias)
            x = self.ln1(self.attn(x, key_mask=key_mask, sink_in=s1, bias_handoff=h1), residual=x, sink=s1,
                         bias_handoff=h1)
            s2 = _sink(self, x)
            h2 = BiasHandoff(self.ff.fc2.bias)
            return self.ln2(self.ff(x, sink_in=s2, bias_handoff=h2), residual=x, sink=s2, bias_handoff=h2)
        a = self.drop(self.attn(x, key_mask=key_mask, sink_in=s1))
        x = self.ln1(a, residual=x, sink=s1) if FUSED_RESIDUAL_LN else self.ln1(residual_add(x, a, s1))
        s2 = _sink(self, x)
        f = self.drop(self.ff(x, sink_in=s2))
        return self.ln2(f, residual=x, sink=s2) if FUSED_RESIDUAL_LN else self.ln2(residual_add(x, f, s2))


class DecoderLayer(nn.Module):
    def __init__(self, d_model, heads, d_ff, key_dim=None, dropout=0.0, eps=1e-5):
        super().__init__()
        self.self_attn = MultiHeadAttention(d_model, heads, key_dim, dropout)
        self.ln1 = FusedLayerNorm(d_model, eps=eps)
        self.cross = MultiHeadAttention(d_model, heads, key_dim, dropout, cross=True)
        self.ln2 = FusedLayerNorm(d_model, eps=eps)
        self.ff = FeedForward(d_model, d_ff)
        self.ln3 = FusedLayerNorm(d_model, eps=eps)

    def forward(self, y, enc, tgt_mask=None, src_mask=None):
        if not FUSED_RESIDUAL_LN:
            y = self.ln1(y + self.self_attn(y, key_mask=tgt_mask, causal=True))
            y = self.ln2(y + self.cross(y, kv=enc, key_mask=src_mask))
            return self.ln3(y + self.ff(y))
        y = self.ln1(self.self_attn(y, key_mask=tgt_mask, causal=True), residual=y)
        y = self.ln2(self.cross(y, kv=enc, key_mask=src_mask), residual=y)
        return self.ln3(self.ff(y), residual=y)
