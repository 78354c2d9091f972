"""Transformer NMT (eng->spa) and BERT-base.

* ``TransformerNMT``: the reference's Keras example (reference
  examples/py/tensorflow2/neural_machine_translation_with_transformer.py:89-94,191-315):
  vocab 15000, sequence length 20, embedding 256, FFN 2048, 8 heads with key_dim 256,
  1 encoder + 1 decoder layer, token + position embeddings, softmax head over the vocab.
* ``BertBase``: BERT-base encoder (12 x [768, 12 heads, FFN 3072], seq 128-512) with an MLM
  head -- the BASELINE.json "mixed ResNet-50 + BERT-base" AFS-L config.
"""
from __future__ import annotations

import torch
from torch import nn

from ..ops.dense import FusedLinear
from ..ops.embedding import FusedEmbedding, add_rows
from ..ops.layernorm import FusedLayerNorm
from .layers import HIP_GELU, DecoderLayer, EncoderLayer, GeluTanh


class PositionalEmbedding(nn.Module):
    def __init__(self, seq_len: int, vocab: int, dim: int):
        super().__init__()
        self.tok = FusedEmbedding(vocab, dim)
        self.pos = FusedEmbedding(seq_len, dim)

    def forward(self, ids):
        return add_rows(self.tok(ids), self.pos.weight, 0, ids.shape[1])


class TransformerNMT(nn.Module):
    def __init__(self, vocab: int = 15000, seq_len: int = 20, d_model: int = 256, d_ff: int = 2048,
                 heads: int = 8, key_dim: int = 256, layers: int = 1, dropout: float = 0.0):
        super().__init__()
        self.src_emb = PositionalEmbedding(seq_len, vocab, d_model)
        self.tgt_emb = PositionalEmbedding(seq_len, vocab, d_model)
        self.enc = nn.ModuleList([EncoderLayer(d_model, heads, d_ff, key_dim, dropout=dropout) for _ in range(layers)])
        self.dec = nn.ModuleList([DecoderLayer(d_model, heads, d_ff, key_dim, dropout=dropout) for _ in range(layers)])
        self.head = FusedLinear(d_model, vocab)
        self.num_classes = vocab

    def forward(self, src, tgt):
        src_mask = (src != 0)
        x = self.src_emb(src)
        for l in self.enc:
            x = l(x, key_mask=src_mask)
        y = self.tgt_emb(tgt)
        for l in self.dec:
            y = l(y, x, tgt_mask=(tgt != 0), src_mask=src_mask)
        return self.head(y)


def padded_vocab(vocab: int, multiple: int = 64) -> int:
    return -(-vocab // multiple) * multiple


class BertBase(nn.Module):
    """The token table and the tied MLM decoder have ``padded_vocab(vocab)`` rows (30522 ->
    30528, as NVIDIA's BERT does): 16-byte rows for the decoder's HIP weight-gradient kernel
    and the fused cross-entropy, which takes only the first ``num_classes`` = ``vocab``
    columns into the softmax (ops/xent.py), so the loss is the unpadded model's.  The padding
    rows are never looked up and get zero gradient (weight decay only)."""

    def __init__(self, vocab: int = 30522, seq_len: int = 128, d_model: int = 768, heads: int = 12,
                 d_ff: int = 3072, layers: int = 12, dropout: float = 0.0):
        super().__init__()
        self.num_classes = vocab
        vp = padded_vocab(vocab)
        self.emb = PositionalEmbedding(seq_len, vp, d_model)
        self.type_emb = nn.Embedding(2, d_model)
        self.emb_ln = FusedLayerNorm(d_model, eps=1e-12)
        self.layers = nn.ModuleList([EncoderLayer(d_model, heads, d_ff, act="gelu", dropout=dropout, eps=1e-12)
                                     for _ in range(layers)])
        self.mlm_dense = FusedLinear(d_model, d_model)
        self.mlm_ln = FusedLayerNorm(d_model, eps=1e-12)
        self.mlm_out = FusedLinear(d_model, vp)
        self.mlm_out.weight = self.emb.tok.weight  # tied embeddings, as in BERT
        self.act = GeluTanh() if HIP_GELU else nn.GELU(approximate="tanh")
        for m in self.modules():
            if isinstance(m, (nn.Linear, nn.Embedding)):
                nn.init.normal_(m.weight, std=0.02)
            if isinstance(m, nn.Linear) and m.bias is not None:
                nn.init.zeros_(m.bias)

    def forward(self, ids, attention_mask=None, masked_positions=None):
        """``masked_positions`` [B, P] (the standard BERT pretraining input
        ``masked_lm_positions``): the MLM head runs on those B*P rows only -- the loss is
        identical (unmasked tokens carry no label) and the vocab GEMMs + softmax shrink by
        T/P (6.4x at T=128, P=20).  Returns [rows, padded vocab] logits; the classes are the
        first ``num_classes`` columns."""
        x = self.emb_ln(add_rows(self.emb(ids), self.type_emb.weight, 0, 1))
        for l in self.layers:
            x = l(x, key_mask=attention_mask)
        if masked_positions is not None:
            B, T, D = x.shape
            flat = (masked_positions + torch.arange(B, device=x.device)[:, None] * T).reshape(-1)
            x = x.reshape(B * T, D).index_select(0, flat)
        return self.mlm_out(self.mlm_ln(self.act(self.mlm_dense(x))))
