"""Attention + feed-forward transformer layer (north-star config "attention+FF, 2D mesh, fp8").

The reference declares the FF layer in comments only (``case6_attention.py:36-40``,
``y = Relu(Win x) Wout``) and maps its ``hidden`` logical axis to ``model``
(``case6_attention.py:186``).  This layer is the case6 attention block followed
by that FF block, each with a residual connection; ``fp8=True`` runs the FF
GEMMs on CDNA4's e4m3 MFMA path.
"""
from __future__ import annotations

from typing import Any

import torch

from ..nn.layers import FeedForward
from ..nn.module import Module
from ..ops import core
from .attention import MultiHeadAttention, attention_block_flops

__all__ = ["TransformerLayer", "transformer_layer_flops"]


class TransformerLayer(Module):
    query_dim: int
    heads: int = 8
    dim_head: int = 64
    ff_dim: int = 2560
    dtype: Any = torch.bfloat16
    fp8: bool = False

    def setup(self):
        self.attn = MultiHeadAttention(self.query_dim, self.heads, self.dim_head, dtype=self.dtype, name="attn")
        self.ff = FeedForward(self.ff_dim, dtype=self.dtype, fp8=self.fp8, name="ff")

    def __call__(self, x):
        # h = x + attn(x); y = h + ff(h), both skip connections fused into the output GEMMs'
        # epilogues (x is read in f32 and rounded to the compute dtype there, as convert(x) would)
        h = self.attn(x, residual=x)
        return self.ff(h, residual=h)


def transformer_layer_flops(batch, seq, dim, heads, dim_head, ff_dim, train: bool) -> float:
    att = attention_block_flops(batch, seq, dim, heads, dim_head, train)
    ff = 2 * 2 * batch * seq * dim * ff_dim
    return att + (3 * ff if train else ff)
