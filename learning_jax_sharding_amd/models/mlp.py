"""Matmul-chain model for the FSDP / fully-sharded benchmark config (case3 at scale).

``case3_fully_sharded.py:23-46`` shards both matmul operands over the whole mesh and
lets GSPMD gather ("all gather happens", ``:57``).  At training scale that is FSDP:
every weight lives sharded over the ``data`` axis (``parallel.fsdp.fsdp_shardings``),
the partitioner all-gathers it at its use and autograd reduce-scatters its gradient.
``DenseStack`` is ``layers`` bias-free ``dim x dim`` Dense layers with ReLU between
them - a chain of sharded matmuls whose gathers the side-stream collectives overlap
with the previous layer's GEMMs.
"""
from __future__ import annotations

from typing import Any

import torch

from .. import dtypes as _dt
from ..nn.layers import Dense
from ..nn.module import Module
from ..ops import core

__all__ = ["DenseStack", "dense_stack_flops", "feed_forward_flops"]


class DenseStack(Module):
    dim: int
    layers: int = 4
    dtype: Any = torch.bfloat16

    def setup(self):
        self.blocks = [Dense(self.dim, use_bias=False, dtype=self.dtype, name=f"dense_{i}")
                       for i in range(self.layers)]

    def __call__(self, x):
        dt = _dt.canonicalize(self.dtype)
        for i, blk in enumerate(self.blocks):
            # ReLU fused into the GEMM epilogue (Dense itself has no activation)
            x = core.dense(x, [blk.kernel_param(x.shape[-1])], None, compute_dtype=dt,
                           relu=i + 1 < len(self.blocks))[0]
        return x


def dense_stack_flops(batch: int, seq: int, dim: int, layers: int, train: bool) -> float:
    """Matmul FLOPs; the input is not a parameter, so the first layer has no dX GEMM."""
    one = 2.0 * batch * seq * dim * dim
    return layers * one + ((2 * layers - 1) * one if train else 0.0)


def feed_forward_flops(batch: int, seq: int, dim: int, ff_dim: int, train: bool) -> float:
    """``relu(x Win) Wout`` (``case6_attention.py:36-40`` comments; case4's FC layer)."""
    one = 2.0 * batch * seq * dim * ff_dim
    return 2 * one + (3 * one if train else 0.0)
